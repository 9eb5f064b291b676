#!/usr/bin/env python3
"""Per-kernel table of one tools/pmc_ab.sh label directory: average duration
(kernel trace) and per-dispatch PMC values (FETCH_SIZE / WRITE_SIZE in MB as
counted -- FETCH_SIZE reads 128-B requests as 64 B for 16-B/lane streams on
gfx950, MI355X_MICROARCH.md, so x2 for those -- and the SQ counters).
Usage: python tools/pmc_table.py DIR [--json OUT]"""
import collections
import csv
import json
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:44]


def main():
    root = sys.argv[1]
    stats = {}
    p = os.path.join(root, "trace", "trace_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    pm = collections.defaultdict(dict)
    for sub in sorted(os.listdir(root)):
        f = os.path.join(root, sub, "pmc_counter_collection.csv")
        if not sub.startswith("pmc_") or not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            for c, v in cs.items():
                pm[k][c] = sum(v) / len(v)
    cols = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES"]
    print(f"{'kernel':44s} {'n':>3s} {'avg_us':>8s} {'fetchMB':>8s} {'writeMB':>8s} " +
          " ".join(f"{c[3:]:>14s}" for c in cols))
    out = {}
    for k, (n, us) in sorted(stats.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        c = pm.get(k, {})
        fm, wm = c.get("FETCH_SIZE", float("nan")) / 1024, c.get("WRITE_SIZE", float("nan")) / 1024
        print(f"{k:44s} {n:3d} {us:8.1f} {fm:8.1f} {wm:8.1f} " +
              " ".join(f"{c.get(x, float('nan')) / 1e6:13.2f}M" for x in cols))
        out[k] = {"calls": n, "avg_us": us, "fetch_MB": fm, "write_MB": wm, **{x: c.get(x) for x in c}}
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
