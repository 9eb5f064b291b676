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
  profile_rows    sha256 of the concatenated sha256 digests of the profile's
            rows: independent of how the rows are sharded, so the ranks of a
            multi-GPU run hash their own rows and rank 0 combines 32 B per row
            (bench.py's in-run parity check)
Large arrays are hashed in place (memoryview), so a 16 GB profile needs no copy.
bench.py imports this module for its in-run parity check (hashing only; it
never imports the oracle outside its cpu_baseline leg).
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


def row_digests(prof, threads=8):
    """bytes: the sha256 digest of every row of a C-order float64 [n, M] array,
    in row order (hashed on a thread pool; hashlib releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    assert prof.dtype == np.float64 and prof.flags.c_contiguous and prof.ndim == 2
    n = prof.shape[0]
    mv = memoryview(prof.reshape(n, -1)).cast("B")
    row_b = prof.shape[1] * 8

    def blk(lo):
        hi = min(n, lo + BLOCK_ROWS)
        return b"".join(hashlib.sha256(mv[i * row_b:(i + 1) * row_b]).digest() for i in range(lo, hi))

    with ThreadPoolExecutor(threads) as pool:
        return b"".join(pool.map(blk, range(0, n, BLOCK_ROWS)))


def profile_rows_digest(prof=None, rows=None):
    """sha256 over the per-row digests (of `prof`, or given as `rows` bytes)."""
    return hashlib.sha256(row_digests(prof) if rows is None else rows).hexdigest()


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
