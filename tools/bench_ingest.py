#!/usr/bin/env python3
"""Host ingestion timing: the C++ readers (csrc/ingest.cpp) vs the reference's
Python reading of the same files, on config-3-sized synthetic inputs.

  FASTA : 200k contigs (mean 800 bp, 60-column lines), karma.py:40-61
  eq    : salmon eq_classes.txt of 3.4e5 classes over 200k contigs, read_graph.py:75-92
  SAM   : 4M alignment lines (SAM-lite, 6 columns), contig.py:24,34

Usage: python tools/bench_ingest.py [--threads T] [--dir /tmp/karma_ingest]
"""
import argparse
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from karma_amd import contig, fasta, ingest, read_graph  # noqa: E402
from karma_amd.synth import contig_sequences  # noqa: E402


def make_inputs(d):
    os.makedirs(d, exist_ok=True)
    fa = os.path.join(d, "c3.fa")
    if not os.path.exists(fa):
        seqs = contig_sequences(3, 200_000)
        with open(fa, "w") as f:
            for k, v in seqs.items():
                f.write(k + " len=%d\n" % len(v))
                for j in range(0, len(v), 60):
                    f.write(v[j:j + 60] + "\n")
    eq = os.path.join(d, "c3.eq.txt")
    if not os.path.exists(eq):
        rng = random.Random(3)
        n, c = 200_000, 340_000
        with open(eq, "w") as f:
            f.write(f"{n}\n{c}\n")
            for i in range(n):
                f.write(f"ctg{i}\n")
            for _ in range(c):
                g0 = rng.randrange(n - 4)
                ids = sorted(rng.sample(range(g0, g0 + 4), rng.randrange(1, 5)))
                f.write("\t".join([str(len(ids))] + [str(x) for x in ids] + [str(rng.randrange(1, 3000))]) + "\n")
    sam = os.path.join(d, "c3.sam")
    if not os.path.exists(sam):
        rng = random.Random(4)
        with open(sam, "w") as f:
            for r in range(2_000_000):
                g0 = rng.randrange(200_000 - 4)
                for m in range(2):
                    f.write(f"frag{r}\t{m * 16}\tctg{g0 + rng.randrange(4)}\t{rng.randrange(1, 800)}\t60\t*\n")
    return fa, eq, sam


def timed(fn, *a):
    t = time.perf_counter()
    r = fn(*a)
    return r, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--dir", default="/tmp/karma_ingest")
    args = ap.parse_args()
    fa, eq, sam = make_inputs(args.dir)
    out = {}
    data = ingest._read(fa)
    _, out["fasta_cpp_parse_s"] = timed(ingest.parse_fasta, data, args.threads)
    _, out["fasta_read_fasta_file_s"] = timed(fasta.read_fasta_file, fa, args.threads)
    _, out["fasta_python_reference_s"] = timed(fasta._read_fasta_text, fa)
    data = ingest._read(eq)
    _, out["eq_cpp_parse_s"] = timed(ingest.parse_eq, data, args.threads)
    _, out["eq_parse_eq_classes_s"] = timed(read_graph.parse_eq_classes, eq, args.threads)
    _, out["eq_python_reference_s"] = timed(read_graph._parse_eq_text, eq)
    data = ingest._read(sam)
    _, out["sam_cpp_parse_s"] = timed(ingest.parse_sam, data, True, args.threads)

    def py_sam():  # contig.py:34 per line, grouped by RNAME
        groups = {}
        with open(sam) as f:
            for line in f:
                read, _, name, position, *_ = line.split("\t")
                groups.setdefault(name, set()).add(read)
        return groups
    _, out["sam_python_reference_s"] = timed(py_sam)
    out["bytes"] = {"fasta": os.path.getsize(fa), "eq": os.path.getsize(eq), "sam": os.path.getsize(sam)}
    out["threads"] = args.threads or os.cpu_count()
    for k, v in out.items():
        print(f"{k}: {v if not isinstance(v, float) else round(v, 4)}")


if __name__ == "__main__":
    main()
