#!/usr/bin/env python3
"""Latency of one karma_adj_view_summary call (a 40-node cluster of a config-2-like
eq graph): wall time per call; run under rocprofv3 --kernel-trace for the kernel's
own duration.  Usage (GPU box): python tools/diag_summary.py [--n 5000]"""
import argparse
import os
import sys
import tempfile
import time
from collections import OrderedDict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from karma_amd import synth  # noqa: E402
from karma_amd.read_graph import ReadGraph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=5000)
ap.add_argument("--cluster", type=int, default=40)
ap.add_argument("--calls", type=int, default=500)
a = ap.parse_args()
classes = synth.eq_classes(2, a.n, a.n * 200, True)
names = [f"ctg{i}" for i in range(a.n)]
path = os.path.join(tempfile.mkdtemp(), "eq.txt")
with open(path, "w") as f:
    f.write(synth.eq_file_text(names, classes))
g = ReadGraph.from_equivalence_classes(path, OrderedDict((">" + x, "") for x in names))
root = g._device_mirror()
pos = root.pos()
nodes = list(g.nodes())
order = np.array([pos[x] for x in nodes[100:100 + a.cluster]], np.int64)
for text in (False, True):
    root.adj.view_summary(order, root.names, text)
    t = time.perf_counter()
    for _ in range(a.calls):
        root.adj.view_summary(order, root.names, text)
    print(f"with_text={text}: {(time.perf_counter() - t) / a.calls * 1e6:.1f} us per call", flush=True)
from karma_amd import _lib  # noqa: E402
ctx = _lib.default_context()
t = time.perf_counter()
for _ in range(a.calls):
    ctx.sync()
print(f"empty stream sync: {(time.perf_counter() - t) / a.calls * 1e6:.1f} us per call", flush=True)
