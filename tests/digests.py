"""Canonical SHA-256 digests of the hot path's outputs at BASELINE config sizes.

Test infrastructure (imported by tests/ and tests/golden/make_digests.py only).
The encodings follow SURVEY.md §8(c) golden plan item (iii):
  profile   float64 N x M, C order, little-endian bytes   (kmer.py:206-233)
  columns   column keys in column order, '\\n'-joined, latin-1 (kmer.py:172-177)
  edges     canonical a < b, sorted by (a, b):
              ab      u32 a[E] bytes then u32 b[E] bytes
              weight  f64 w[E]                           (read_graph.py:128-130)
              shared  i64 s[E]                           (shared fragments / summed counts)
  totals    i64 per-contig fragment totals [n_contigs]   (read_graph.py:86-92)
  profile_blocks  sha256 of the concatenated sha256 digests of the profile's
            BLOCK_ROWS-row blocks (a checksum of checksums: hashed in parallel)
Large arrays are hashed in place (memoryview), so a 16 GB profile needs no copy.
"""

import hashlib
import os
import sys
from argparse import Namespace

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

BLOCK_ROWS = 8192
DIGEST_FILE = os.path.join(REPO, "tests", "golden", "digests.json")

# name -> bench.py arguments (the bench's exact workloads, bench.make_inputs)
WORKLOADS = {
    # BASELINE configs[1]: 50k contigs, 10M paired fragments, 5p6, one GPU
    "config2": dict(config="config2", emulate_ranks=1, strong=False),
    # BASELINE configs[2]: 200k contigs, 100M paired fragments, 5p6 (the headline)
    "config3": dict(config="config3", emulate_ranks=1, strong=False),
    # BASELINE configs[4]: rank 0's share of the 8-GPU job -- 125k contigs, k=7
    # (M = 16,384), fragments [0, 62.5M) over 1M global contig ids
    "config5_rank0of8": dict(config="config5", emulate_ranks=8, strong=False),
    # BASELINE configs[4] whole on one GPU: 1M contigs, 500M paired fragments
    # (1.54e9 records), k=7 -- a 131 GB profile, resident in 288 GB of HBM
    "config5_1gpu": dict(config="config5_1gpu", emulate_ranks=1, strong=False),
}


def bench_args(name, **over):
    a = dict(config="config3", emulate_ranks=1, strong=False, shuffle_contigs=False)
    a.update(WORKLOADS.get(name, {}))
    a.update(over)
    return Namespace(**a)


def bench_inputs(name, rank=0, world=1, **over):
    """The inputs bench.py times for this workload (its make_inputs)."""
    import bench

    return bench.make_inputs(bench_args(name, **over), rank, world)


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        if a.size:
            h.update(memoryview(a).cast("B"))
    return h.hexdigest()


def columns_digest(cols):
    return hashlib.sha256("\n".join(cols).encode("latin-1")).hexdigest()


def profile_digest(prof):
    assert prof.dtype == np.float64 and prof.flags.c_contiguous
    return sha(prof)


def edge_digests(a, b, weight, shared=None, totals=None):
    a = np.asarray(a, dtype="<u4")
    b = np.asarray(b, dtype="<u4")
    out = {"E": int(len(a)), "ab": sha(a, b), "weight": sha(np.asarray(weight, dtype="<f8"))}
    if shared is not None:
        out["shared"] = sha(np.asarray(shared, dtype="<i8"))
    if totals is not None:
        out["totals"] = sha(np.asarray(totals, dtype="<i8"))
    return out


def load():
    import json

    with open(DIGEST_FILE) as f:
        return json.load(f)
