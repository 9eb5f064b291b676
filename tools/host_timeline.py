#!/usr/bin/env python3
"""Host timeline of one bench step: every library call with its start offset,
duration and the host time spent outside the library before it (Python).

Usage (GPU box): python tools/host_timeline.py [bench args...]  e.g. --emulate-ranks 8
Runs 30 steps and prints step 25.  Diagnostic only."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["KARMA_CALL_TIMES"] = "seq"
import bench  # noqa: E402
from karma_amd import _lib, distributed  # noqa: E402

sys.argv = ["bench.py", "--cpu-baseline", "off", "--no-e2e", "--no-timing", "--no-parity", "--steps", "30",
            "--warmup", "2"] + sys.argv[1:]
run0 = distributed.ShardedBuild.run
marks = []


STREAM = os.environ.get("HTL_STREAM") == "1"  # steps as the bench's timed stream (count=False)


def run(self, *a, **k):
    if STREAM and not k.get("keep") and not k.get("sequential"):
        k["count"] = False
    marks.append((len(_lib.CALL_SEQ), time.perf_counter()))
    try:
        return run0(self, *a, **k)
    finally:
        marks.append((len(_lib.CALL_SEQ), time.perf_counter()))


distributed.ShardedBuild.run = run
try:
    bench.main()
except TypeError:  # HTL_STREAM: the last step has no edge count either; the timeline is what we want
    pass
(i0, t0), (i1, t1) = marks[2 * 25], marks[2 * 25 + 1]
nxt = marks[2 * 26][1] if len(marks) > 2 * 26 else None
prev = t0
print(f"step 25: {1e6 * (t1 - t0):.1f} us in run(); next run() starts {1e6 * (nxt - t1):.1f} us later" if nxt else "")
for name, s, e in _lib.CALL_SEQ[i0:i1]:
    print(f"{1e6 * (s - t0):8.1f} +{1e6 * (e - s):7.1f}  (py {1e6 * (s - prev):6.1f})  {name}")
    prev = e
print(f"{1e6 * (t1 - t0):8.1f} end (py {1e6 * (t1 - prev):6.1f})")
