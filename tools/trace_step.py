#!/usr/bin/env python3
"""One step of a rocprofv3 kernel trace (between the last two launches of a
kernel), with start offsets, durations and streams.
Usage: python tools/trace_step.py TRACE_DIR [KERNEL_SUBSTRING]"""
import csv
import sys

d = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "classify2"
rows = sorted(csv.DictReader(open(f"{d}/trace_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s:e]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("rocprim::ROCPRIM_400200_NS::detail::", "")[:64]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} s{r['Stream_Id']} {n}")
