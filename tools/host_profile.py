#!/usr/bin/env python3
"""cProfile of bench.py's step loop (host side: Python + ctypes + HIP API time).

Usage (GPU box): python tools/host_profile.py [bench args...]   e.g. --strong --emulate-ranks 8
Diagnostic only."""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["KARMA_CALL_TIMES"] = "1"
import bench  # noqa: E402

sys.argv = ["bench.py", "--cpu-baseline", "off", "--no-e2e", "--no-timing", "--steps", "50", "--warmup", "5"] \
    + sys.argv[1:]
pr = cProfile.Profile()
orig = bench.ShardedBuild if hasattr(bench, "ShardedBuild") else None
from karma_amd import _lib, distributed  # noqa: E402

run0 = distributed.ShardedBuild.run
count = {"n": 0}


def run(self, *a, **k):
    count["n"] += 1
    if count["n"] == 6:
        pr.enable()
        _lib.CALL_TIMES.clear()
    try:
        return run0(self, *a, **k)
    finally:
        if count["n"] == 55:
            pr.disable()


distributed.ShardedBuild.run = run
bench.main()
calls = sorted(_lib.CALL_TIMES.items(), key=lambda kv: -kv[1][1])
print("per-step host time by entry point (us):", file=sys.stderr)
for name, (n, t) in calls:
    print(f"  {name:40s} {n / 50:5.1f} calls  {t / 50 * 1e6:8.1f} us", file=sys.stderr)
st = pstats.Stats(pr, stream=sys.stderr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
