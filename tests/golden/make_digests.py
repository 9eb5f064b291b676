#!/usr/bin/env python3
"""tests/golden/digests.json: SHA-256 digests of the oracle's outputs on the
bench's exact workloads at BASELINE config sizes (and, with --reference, of the
REFERENCE's own outputs on config 2).

Runs in the build container only (the GPU box never runs it): the GPU tests
(tests/test_gpu_configs.py) recompute the same digests from the HIP path and
compare, so no CPU oracle time is spent on the GPU box.

Per workload (tests/digests.py WORKLOADS = bench.py make_inputs):
  * k-mer profile: oracle_omp_kmer_profile (oracle/oracle.c, the OpenMP twin
    of the scalar restatement of kmer.py:199-264) -> columns + profile digests;
  * readset graph: oracle_omp_graph_reads (read_graph.py:19-50 semantics on the
    records) -> edge digests (ab, weight, shared, totals);
  * eq-class graph: the same fragments as salmon eq classes through the scalar
    oracle_graph_groups (read_graph.py:61-148) -> must equal the readset
    graph's digests (each fragment's dedup set is its class), asserted here.
--reference (config 2): the reference itself, imported as in make_golden.py:
  KmerClustering.__calc_kmer_profile at 50k contigs / 5p6 (kmer.py:199-264) and
  ReadGraph.from_equivalence_classes on the config-2 eq file
  (read_graph.py:61-148); the graph is canonicalised to a < b, sorted.

Usage: python tests/golden/make_digests.py [--only config2,config3] [--reference]
"""

import argparse
import hashlib
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import digests as D  # noqa: E402
from karma_amd import engine  # noqa: E402
from oracle import oracle  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def sequences(inp):
    blob, offs = inp["blob"], inp["offs"]
    c_lo = inp["c_lo"]
    seqs = OrderedDict()
    for i in range(inp["n_loc"]):
        seqs[f">ctg{c_lo + i}"] = bytes(blob[offs[i]:offs[i + 1]]).decode("latin-1")
    assert all(len(k) == int(x) for k, x in zip(seqs, inp["key_len"])), "key_len must be len(FASTA key)"
    return seqs


def eq_arrays(inp):
    cls_off, mem, cnt = engine.synth_eq_classes(inp["seed"], inp["n_glob"], inp["f_lo"], inp["f_lo"] + inp["f_loc"],
                                                inp["paired"], genes=inp["genes"])
    skip = (np.diff(cls_off) == 1).astype(np.uint8)  # eq_size token "1" (read_graph.py:99)
    return cls_off, mem, cnt, skip


def oracle_workload(name):
    inp = D.bench_inputs(name)
    kmer, n_glob = inp["kmer"], inp["n_glob"]
    t0 = time.time()
    seqs = sequences(inp)
    raw, M = oracle.kmer_columns(seqs, kmer)
    cols = oracle.decode_keys(raw, M)
    del seqs
    # row blocks hashed in order (a 131 GB profile never exists in host memory)
    # plus the digest of per-block digests (D.BLOCK_ROWS rows each), which the
    # GPU test can hash on several threads
    h = hashlib.sha256()
    blocks, rows = [], []
    offs, key_len, n = inp["offs"], inp["key_len"], inp["n_loc"]
    for lo in range(0, n, D.BLOCK_ROWS):
        hi = min(n, lo + D.BLOCK_ROWS)
        blk = oracle.omp_kmer_profile_packed(inp["blob"], offs[lo:hi + 1], key_len[lo:hi], kmer, raw, M)
        h.update(memoryview(blk).cast("B"))
        blocks.append(hashlib.sha256(memoryview(blk).cast("B")).digest())
        rows.append(D.row_digests(blk))
        del blk
    out = {"bench_args": D.WORKLOADS[name], "N": inp["n_loc"], "n_glob": n_glob, "c_lo": inp["c_lo"],
           "fragments": inp["f_loc"], "kmer": kmer, "M": int(M), "columns": D.columns_digest(cols),
           "profile": h.hexdigest(), "profile_blocks": hashlib.sha256(b"".join(blocks)).hexdigest(),
           "profile_rows": D.profile_rows_digest(rows=b"".join(rows))}
    t1 = time.time()
    rec = inp["rec"]
    starts = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    g = oracle.omp_graph_reads(np.r_[starts, len(rec)].astype(np.int64), rec[:, 1], n_glob)
    assert not g["zero_div"]
    out["records"] = int(len(rec))
    out["edges"] = D.edge_digests(g["a"], g["b"], g["weight"], g["shared"], g["totals"])
    t2 = time.time()
    cls_off, mem, cnt, skip = eq_arrays(inp)
    o = oracle.graph_groups(cls_off, mem, cnt, skip, n_glob, dedup=False)
    eqd = D.edge_digests(o["a"], o["b"], o["weight"], o["shared"], o["totals"])
    assert eqd == out["edges"], f"{name}: eq-class graph differs from the readset graph"
    out["eq_classes"] = int(len(cnt))
    out["eq_members"] = int(len(mem))
    log(f"{name}: M={M} E={out['edges']['E']} profile {t1 - t0:.1f}s graph {t2 - t1:.1f}s eq {time.time() - t2:.1f}s")
    return out


def reference_config2():
    """The reference's own outputs on the config-2 workload."""
    from make_golden import import_reference

    KC, RG, _, scratch = import_reference()
    inp = D.bench_inputs("config2")
    seqs = sequences(inp)
    t0 = time.time()
    k = KC(OrderedDict(seqs), scratch, inp["kmer"], 8)
    prof = k._KmerClustering__calc_kmer_profile()  # kmer.py:199-264
    cols = [km for km, _ in sorted(k.kmers.items(), key=lambda kv: kv[1])]
    out = {"M": int(prof.shape[1]), "columns": D.columns_digest(cols),
           "profile": D.profile_digest(np.ascontiguousarray(prof, dtype="<f8"))}
    del prof, k
    t1 = time.time()
    cls_off, mem, cnt, _ = eq_arrays(inp)
    n = inp["n_glob"]
    names = [f"ctg{i}" for i in range(n)]
    lines = [str(n), str(len(cnt))] + names
    for c in range(len(cnt)):
        ids = mem[cls_off[c]:cls_off[c + 1]]
        lines.append("\t".join([str(len(ids))] + [str(int(i)) for i in ids] + [str(int(cnt[c]))]))
    path = os.path.join(scratch, "config2.eq.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    g = RG.from_equivalence_classes(path, OrderedDict((">" + x, "") for x in names))  # read_graph.py:61-148
    idx = {x: i for i, x in enumerate(names)}
    e = []
    for u, v, d in g.edges(data=True):
        a, b = sorted((idx[u], idx[v]))
        e.append((a, b, d["weight"]))
    e.sort()
    out["edges"] = D.edge_digests([x[0] for x in e], [x[1] for x in e], [x[2] for x in e])
    out["nodes"] = g.number_of_nodes()
    log(f"reference config2: profile {t1 - t0:.1f}s, eq graph {time.time() - t1:.1f}s, E={len(e)}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(D.WORKLOADS))
    ap.add_argument("--reference", action="store_true")
    args = ap.parse_args()
    try:
        allw = D.load()
    except OSError:
        allw = {"generator": "tests/golden/make_digests.py", "encoding": D.__doc__.split("\n\n")[0]}
    for name in [x for x in args.only.split(",") if x]:
        allw[name] = oracle_workload(name)
    if args.reference:
        sys.path.insert(0, HERE)
        allw["reference_config2"] = reference_config2()
    with open(D.DIGEST_FILE, "w") as f:
        json.dump(allw, f, indent=1)
    log("wrote", D.DIGEST_FILE)


if __name__ == "__main__":
    main()
