#!/usr/bin/env python3
"""Capture golden vectors by running the REFERENCE (lmfaber/karma) in this container.

Run only where /root/reference exists (the build container); the GPU box never
runs this.  Outputs are committed under tests/golden/ and pin the oracle
(oracle/) and the HIP path.  The reference is imported read-only with the
shims listed in SURVEY.md §8(c):
  * stub modules hdbscan / umap / seaborn (unused by the hot path),
  * numpy>=1.24 lacks np.float -> alias to float (kmer.py:207),
  * KmerClustering.__is_palindrome is called but never defined (kmer.py:79,
    :194 -> name-mangled AttributeError) -> alias to is_palindrome (kmer.py:47),
  * cwd = a scratch dir because karma/logs.py:14 writes karma.log into cwd.

Usage:  python tests/golden/make_golden.py [--out tests/golden]
"""

import argparse
import hashlib
import json
import os
import sys
import tempfile
import types
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from karma_amd import synth  # noqa: E402  (pure-Python generator spec)

REF = "/root/reference"


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    scratch = tempfile.mkdtemp(prefix="karma_ref_")
    os.chdir(scratch)
    sys.path[:0] = [REF]
    sys.path.append(os.path.join(REF, "karma"))
    for m in ("hdbscan", "umap", "seaborn"):
        sys.modules[m] = types.ModuleType(m)
    import numpy as np

    np.float = float
    import logging

    from karma.kmer import KmerClustering

    KmerClustering._KmerClustering__is_palindrome = staticmethod(KmerClustering.is_palindrome)
    import contig as ref_contig
    import read_graph as ref_graph

    for name in ("karma.logs", "logs"):
        if name in sys.modules:
            sys.modules[name].logger.setLevel(logging.CRITICAL)
    return KmerClustering, ref_graph.ReadGraph, ref_contig.Contig, scratch


def profile_case(KC, seqs, kmer, scratch, threads=2):
    """Run KmerClustering.__calc_kmer_profile (kmer.py:199-264)."""
    k = KC(OrderedDict(seqs), scratch, kmer, threads)
    try:
        prof = k._KmerClustering__calc_kmer_profile()
    except SystemExit as e:  # kmer.py:248/:258 exit(1)
        return {"exit": int(e.code) if e.code is not None else 0}
    except Exception as e:  # e.g. ZeroDivisionError in the Pool
        return {"raises": type(e).__name__}
    kmers = sorted(k.kmers.items(), key=lambda kv: kv[1])
    rows, cols = prof.nonzero()
    return {
        "shape": list(prof.shape),
        "columns": [km for km, _ in kmers],
        "nz": [[int(r), int(c), float(prof[r, c])] for r, c in zip(rows, cols)],
        "sha256": hashlib.sha256(prof.astype("<f8").tobytes(order="C")).hexdigest(),
    }


def graph_dump(g):
    return {
        "nodes": [str(n) for n in g.nodes()],
        "edges": [[str(a), str(b), float(d["weight"])] for a, b, d in g.edges(data=True)],
    }


def eq_case(RG, text, fasta_keys, scratch, name):
    path = os.path.join(scratch, f"{name}.eq.txt")
    with open(path, "w") as f:
        f.write(text)
    try:
        g = RG.from_equivalence_classes(path, OrderedDict((k, "") for k in fasta_keys))
    except Exception as e:
        return {"raises": type(e).__name__}
    return graph_dump(g)


def make_contigs(Contig, names, readsets):
    out = []
    for n, reads in zip(names, readsets):
        c = Contig(n)
        c.load_from_iterator([f"{r}\t0\t{n}\t1\t60\t*" for r in reads])
        out.append(c)
    return out


def readset_case(RG, Contig, names, readsets):
    try:
        g = RG.from_contigs(make_contigs(Contig, names, readsets))
    except Exception as e:
        return {"raises": type(e).__name__}
    return graph_dump(g)


def update_case(RG, Contig, orig_names, orig_sets, new_names, new_sets, base_edges=None):
    g = RG()
    for a, b, w in base_edges or []:
        g.add_edge(a, b, weight=w)
    g.set_original_contigs(make_contigs(Contig, orig_names, orig_sets))
    try:
        g.update_graph(make_contigs(Contig, new_names, new_sets))
    except Exception as e:
        return {"raises": type(e).__name__}
    return graph_dump(g)


def records_to_readsets(recs, n):
    sets = [[] for _ in range(n)]
    seen = [set() for _ in range(n)]
    for r, c in recs:
        if r not in seen[c]:
            seen[c].add(r)
            sets[c].append(f"r{r}")
    return sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    out_dir = os.path.abspath(args.out)
    KC, RG, Contig, scratch = import_reference()

    gold = {"generator": "tests/golden/make_golden.py", "reference": "lmfaber/karma (v0)"}

    # --- reference's own test (tests/test_kmer.py:7-8) + extra predicate probes
    gold["is_palindrome"] = {s: KC.is_palindrome(s) for s in
                             ["ACGT", "AAAA", "ACGGCA", "ACGTTGCA", "ACCA", "A", "", "AN NA", "acgGCA"]}

    # --- k-mer profile: hand cases (SURVEY §8(a) A1-A7 edge cases)
    hand = OrderedDict()
    hand["probe_5p6"] = ([(">c1", "ACGTACGTAA"), (">c22 x", "ACANAGGTTGGA")], "5p6")
    hand["mixed_len_order"] = ([(">a", "AAAAAACAAAAGAAAAT"), (">bb", "AAAAANAAAAAA"), (">ccc", "acgtaACGTA")], "5p6")
    hand["header_norm_k5"] = ([(">x", "ACGTAC"), (">longer_header_name", "ACGTACGT"), (">y\r", "TTTTTTT")], 5)
    hand["crlf_and_iupac_k3"] = ([(">s1", "ACGRYN\r"), (">s2", "NNNNNN"), (">s3", "AC\tGT")], 3)
    hand["k1"] = ([(">p", "ACGTN"), (">q", "GGGG")], 1)
    hand["k7"] = ([(">p", "ACGTACGTTGCA"), (">q", "GGGGGGGGA")], 7)
    hand["k8_bytes"] = ([(">p", "ACGT\x00CGTAC"), (">q", "ZZZZZZZZZ")], 8)
    hand["palin_6_only"] = ([(">p", "ACGGCA"), (">q", "TTAATT")], "5p6")
    hand["short_contig_exit"] = ([(">p", "ACGTACGT"), (">q", "ACG")], 5)
    hand["all_short_exit"] = ([(">p", "AC"), (">q", "ACG")], "5p6")
    hand["empty_dict"] = ([], 5)
    hand["zero_len_key"] = ([("", "ACGTACGT")], 5)
    gold["profile_hand"] = {k: {"seqs": v[0], "kmer": v[1], "out": profile_case(KC, v[0], v[1], scratch)}
                            for k, v in hand.items()}

    # --- k-mer profile: randomized fixtures with N injection
    rnd = {}
    for name, (seed, n, kmer, n_rate, lmin, lspan) in {
        "rand64_5p6_N": (11, 64, "5p6", 40, 5, 300),
        "rand16_5p6_short_exit": (15, 16, "5p6", 0, 2, 10),
        "rand64_k5_N": (12, 64, 5, 60, 4, 200),
        "rand48_k7": (13, 48, 7, 0, 50, 400),
        "rand32_k3_N": (14, 32, 3, 7, 1, 60),
    }.items():
        seqs = synth.contig_sequences(seed, n, lmin, lspan, n_rate)
        rnd[name] = {"seed": seed, "n": n, "kmer": kmer, "n_rate": n_rate, "len_min": lmin,
                     "len_span": lspan, "out": profile_case(KC, list(seqs.items()), kmer, scratch)}
    gold["profile_rand"] = rnd

    # --- config 1 (BASELINE.json configs[0]): 1k contigs, k=5 -> digest only
    seqs1 = synth.contig_sequences(1, 1000)
    c1 = profile_case(KC, list(seqs1.items()), 5, scratch, threads=8)
    c1.pop("nz")
    gold["profile_config1"] = {"seed": 1, "n": 1000, "kmer": 5, "out": c1}

    # --- eq-class graph (read_graph.py:61-148): hand cases
    eqh = {}
    eqh["basic"] = ("4\n3\nc0\nc1\nc2\nc3\n2\t0\t1\t10\n1\t2\t5\n3\t0\t1\t2\t3\n", [">c0", ">c1", ">c2", ">c3", ">c4", ">c5"])
    eqh["size_token_1_skips_pairs"] = ("3\n2\na\nb\nc\n1\t0\t1\t7\n2\t1\t2\t4\n", [">a", ">b", ">c"])
    eqh["dup_ids_self_loop"] = ("2\n1\nu\nv\n3\t0\t0\t1\t6\n", [">u", ">v"])
    eqh["zero_count_pair"] = ("3\n3\na\nb\nc\n2\t0\t1\t0\n1\t0\t3\n1\t1\t2\n2\t1\t2\t5\n", [">a", ">b", ">c"])
    eqh["unordered_ids_crlf"] = ("3\n1\nx\ny\nz\n3\t2\t0\t1\t9\r\n2\t1\t0\t+3\n", [">x", ">y", ">z"])
    eqh["no_classes"] = ("2\n0\np\nq\n", [">p", ">q", ">r"])
    eqh["zero_div"] = ("2\n2\na\nb\n2\t0\t1\t5\n1\t0\t-5\n", [">a", ">b"])
    eqh["bad_id"] = ("2\n1\na\nb\n2\t0\t7\t5\n", [">a", ">b"])
    eqh["dup_names"] = ("2\n1\na\na\n2\t0\t1\t5\n", [">a"])
    eqh["extra_eq_node"] = ("2\n1\na\nb\n2\t0\t1\t5\n", [">a"])
    gold["eq_hand"] = {k: {"text": t, "fasta": f, "out": eq_case(RG, t, f, scratch, k)} for k, (t, f) in eqh.items()}

    # --- eq-class graph: synthetic config-1-shaped and a paired small case
    eqr = {}
    for name, (seed, n, nf, paired) in {"config1_se": (1, 1000, 100_000, False),
                                         "small_pe": (21, 300, 20_000, True)}.items():
        classes = synth.eq_classes(seed, n, nf, paired)
        names = [f"ctg{i}" for i in range(n)]
        text = synth.eq_file_text(names, classes)
        res = eq_case(RG, text, [">" + x for x in names], scratch, name)
        eqr[name] = {"seed": seed, "n": n, "n_frags": nf, "paired": paired,
                     "n_classes": len(classes), "out": res}
    gold["eq_synth"] = eqr

    # --- readset graph (read_graph.py:19-50) + Contig (contig.py)
    rsh = {}
    rsh["basic"] = (["c0", "c1", "c2", "c3"], [["r1", "r2", "r3"], ["r2", "r3"], [], ["r9"]])
    rsh["mates_dedup"] = (["a", "b"], [["q1", "q1", "q2"], ["q1", "q2", "q2", "q3"]])
    rsh["single_contig"] = (["solo"], [["r1"]])
    rsh["all_empty"] = (["a", "b", "c"], [[], [], []])
    rsh["identical_sets"] = (["a", "b", "c"], [["x", "y"], ["y", "x"], ["x"]])
    gold["readset_hand"] = {k: {"names": n, "readsets": s, "out": readset_case(RG, Contig, n, s)}
                            for k, (n, s) in rsh.items()}
    rsr = {}
    for name, (seed, n, nf, paired) in {"config1_se": (1, 1000, 100_000, False),
                                         "small_pe": (21, 300, 20_000, True)}.items():
        recs = synth.read_records(seed, n, nf, paired)
        sets = records_to_readsets(recs, n)
        rsr[name] = {"seed": seed, "n": n, "n_frags": nf, "paired": paired, "n_records": len(recs),
                     "out": readset_case(RG, Contig, [f"ctg{i}" for i in range(n)], sets)}
    gold["readset_synth"] = rsr

    # --- update_graph (read_graph.py:192-221)
    upd = {}
    upd["basic"] = (["o1", "o2"], [["r1", "r2"], ["r3"]], ["n1", "n2", "o2"], [["r2"], [], ["r3"]], [])
    upd["existing_edge_overwrite"] = (["a"], [["x", "y"]], ["b"], [["y"]], [["a", "b", 0.25], ["b", "z", 1.0]])
    upd["no_originals"] = ([], [], ["n1"], [["r1"]], [])
    gold["update_hand"] = {k: {"orig_names": a, "orig_sets": b, "new_names": c, "new_sets": d, "base_edges": e,
                               "out": update_case(RG, Contig, a, b, c, d, e)}
                           for k, (a, b, c, d, e) in upd.items()}

    # --- Contig.load_from_iterator / load_contig_info_from_sam (contig.py:16-35)
    sam = ["r1\t0\tc\t5\t60\t*", "r1\t16\tc\t9\t60\t*", "r2\t0\tc\t1", "r3\t0\tc\t1\textra\tcols"]
    c = Contig("c")
    c.load_from_iterator(sam)
    gold["contig"] = {"sam": sam, "readset": sorted(c.readset)}

    with open(os.path.join(out_dir, "golden.json"), "w") as f:
        json.dump(gold, f, indent=0, sort_keys=False)
    print("wrote", os.path.join(out_dir, "golden.json"))


if __name__ == "__main__":
    main()
