#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + PMC passes) per kernel.

Usage: python profiles/pmc_summary.py gpurun_out  [--json out.json]
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts
128-B requests as 64 B for wide streaming reads (MI355X_MICROARCH.md §HBM), so
the reported read bytes are a lower bound (x2 for 16-B/lane streams).
"""
import collections
import csv
import json
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:48]


def agg(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return d
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    root = sys.argv[1]
    stats = {}
    p = os.path.join(root, "prof_trace", "trace_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["Percentage"]))
    pm = {}
    for sub in ("prof_pmc1", "prof_pmc2", "prof_pmc3"):
        for k, cs in agg(os.path.join(root, sub, "pmc_counter_collection.csv")).items():
            for c, v in cs.items():
                pm.setdefault(k, {})[c] = sum(v) / len(v)
    out = {}
    print(f"{'kernel':48s} {'calls':>5s} {'avg_us':>9s} {'%':>6s} {'FETCH_MB':>9s} {'WRITE_MB':>9s}")
    for k, (calls, us, pct) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        c = pm.get(k, {})
        fm = c.get("FETCH_SIZE", float("nan")) / 1024
        wm = c.get("WRITE_SIZE", float("nan")) / 1024
        print(f"{k:48s} {calls:5d} {us:9.1f} {pct:6.2f} {fm:9.1f} {wm:9.1f}")
        out[k] = {"calls": calls, "avg_us": us, "pct": pct, "fetch_MB": fm, "write_MB": wm,
                  "counters": {n: v for n, v in c.items() if n not in ("FETCH_SIZE", "WRITE_SIZE")}}
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
