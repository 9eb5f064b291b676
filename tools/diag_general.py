#!/usr/bin/env python3
"""Diagnostic: reads the classify kernel sends to the general path on bench's
config-3 records (KARMA_DEBUG_GEN prints the device count) against a numpy
count of non-compact reads (distinct contigs spanning > 4 ids) and reads of
> 8 records.  Usage (GPU box): python tools/diag_general.py [--frags N]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KARMA_DEBUG_GEN"] = "1"
from karma_amd import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200_000)
ap.add_argument("--frags", type=int, default=10_000_000)
a = ap.parse_args()
genes = engine.synth_genes(3, a.n)
rec = engine.synth_records(3, a.n, 0, a.frags, True, genes=genes)
r = rec.astype(np.int64)
starts = np.flatnonzero(np.r_[True, r[1:, 0] != r[:-1, 0]])
ends = np.r_[starts[1:], len(r)]
mn = np.minimum.reduceat(r[:, 1], starts)
mx = np.maximum.reduceat(r[:, 1], starts)
ln = ends - starts
print(f"reads {len(starts)}, span>3 {int(np.count_nonzero(mx - mn > 3))}, >8 records {int(np.count_nonzero(ln > 8))}, "
      f"m0 >= N-3 {int(np.count_nonzero(mn >= a.n - 3))}", flush=True)
e = engine.graph_from_records(rec, a.n)
print("edges", len(e.a), flush=True)
