#!/usr/bin/env python3
"""Time the REFERENCE (lmfaber/karma, imported read-only) on the bench's exact
config-3 workload, in this container only (the GPU box never runs it), and
check its outputs against tests/golden/digests.json.

What is timed is the path karma.py runs (karma.py:190, :197-210, :240), on the
files bench.py's drop-in leg writes (same names, same bytes):
  read_fasta_file     karma.py:40-61 (taken from karma.py's syntax tree: the
                      shipped karma.py does not import)
  __calc_kmer_profile kmer.py:199-264, threads=8 (the Pool of kmer.py:218)
  from_equivalence_classes  read_graph.py:61-148 on the fragments as salmon
                      eq classes (the readset path, read_graph.py:19-50, is
                      O(N^2): ~21 h at 200k contigs, not timed)
The reference's profile and eq graph are hashed with tests/digests.py's
encodings; they must equal the oracle's config-3 digests, which pins the
config-3 digests by the reference itself (key "reference_config3").

Usage: python tests/golden/time_reference.py [--config config3] [--threads 8]
Writes tests/golden/reference_<config>.json and adds reference_<config> to
tests/golden/digests.json.
"""

import argparse
import json
import os
import resource
import sys
import time
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), HERE]

import digests as D  # noqa: E402
from karma_amd import engine  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def write_inputs(inp, fasta_path, eq_path):
    """The FASTA (one sequence line per contig) and salmon eq_classes.txt of a
    workload: the same writer as bench.py's drop-in leg (dropin_files)."""
    import bench

    return bench.dropin_files(inp, fasta_path, eq_path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--skip-profile", action="store_true")
    args = ap.parse_args()

    from make_golden import import_reference
    from make_golden_ingest import reference_read_fasta_file

    gold = D.load()[args.config]
    KC, RG, _, scratch = import_reference()
    rff = reference_read_fasta_file()
    inp = D.bench_inputs(args.config)
    fasta_path = os.path.join(scratch, f"{args.config}.fa")
    eq_path = os.path.join(scratch, f"{args.config}.eq_classes.txt")
    t0 = time.time()
    write_inputs(inp, fasta_path, eq_path)
    log(f"wrote {fasta_path} ({os.path.getsize(fasta_path)} B), {eq_path} ({os.path.getsize(eq_path)} B) "
        f"in {time.time() - t0:.1f}s")
    out = {"config": args.config, "threads": args.threads, "cpu": os.cpu_count(),
           "fasta_bytes": os.path.getsize(fasta_path), "eq_bytes": os.path.getsize(eq_path),
           "contigs": inp["n_loc"], "fragments": inp["f_loc"]}

    t0 = time.perf_counter()
    seqs = rff(fasta_path)  # karma.py:40-61
    out["read_fasta_file_s"] = round(time.perf_counter() - t0, 3)
    assert len(seqs) == inp["n_loc"]
    log(f"read_fasta_file {out['read_fasta_file_s']} s")

    ref = {}
    if not args.skip_profile:
        k = KC(seqs, scratch, inp["kmer"], args.threads)
        t0 = time.perf_counter()
        prof = k._KmerClustering__calc_kmer_profile()  # kmer.py:199-264
        out["calc_kmer_profile_s"] = round(time.perf_counter() - t0, 3)
        cols = [km for km, _ in sorted(k.kmers.items(), key=lambda kv: kv[1])]
        prof = np.ascontiguousarray(prof, dtype="<f8")
        ref.update(M=int(prof.shape[1]), columns=D.columns_digest(cols), profile=D.profile_digest(prof),
                   profile_rows=D.profile_rows_digest(prof))
        del prof, k
        log(f"calc_kmer_profile {out['calc_kmer_profile_s']} s, M={ref['M']}")
        out["profile_matches_oracle"] = (ref["M"], ref["columns"], ref["profile"]) == \
            (gold["M"], gold["columns"], gold["profile"])

    t0 = time.perf_counter()
    g = RG.from_equivalence_classes(eq_path, seqs)  # read_graph.py:61-148
    out["from_equivalence_classes_s"] = round(time.perf_counter() - t0, 3)
    names = {f"ctg{inp['c_lo'] + i}": i for i in range(inp["n_loc"])}
    e = []
    for u, v, d in g.edges(data=True):
        a, b = sorted((names[u], names[v]))
        e.append((a, b, d["weight"]))
    e.sort()
    ref["edges"] = D.edge_digests([x[0] for x in e], [x[1] for x in e], [x[2] for x in e])
    ref["nodes"] = g.number_of_nodes()
    ge = gold["edges"]
    out["edges_match_oracle"] = ref["edges"] == {k: ge[k] for k in ("E", "ab", "weight")}
    log(f"from_equivalence_classes {out['from_equivalence_classes_s']} s, E={len(e)}")
    out["peak_rss_gb"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2)
    out["peak_rss_children_gb"] = round(resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 2**20, 2)
    if "calc_kmer_profile_s" in out:
        tot = out["read_fasta_file_s"] + out["calc_kmer_profile_s"] + out["from_equivalence_classes_s"]
        out["total_s"] = round(tot, 3)
        out["units_per_s"] = round((inp["n_loc"] + inp["f_loc"]) / tot, 1)

    os.makedirs(os.path.join(REPO, "profiles", "r03"), exist_ok=True)
    with open(os.path.join(REPO, "tests", "golden", f"reference_{args.config}.json"), "w") as f:
        json.dump(out, f, indent=1)
    if not args.skip_profile:
        allw = D.load()
        allw[f"reference_{args.config}"] = ref
        with open(D.DIGEST_FILE, "w") as f:
            json.dump(allw, f, indent=1)
    log(json.dumps(out))


if __name__ == "__main__":
    main()
