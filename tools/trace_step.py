#!/usr/bin/env python3
"""Steps of a rocprofv3 kernel trace (between launches of a marker kernel),
with start offsets, durations and streams, and per window the time the GPU ran
no kernel at all (idle: the host or a dependency held it).
Usage: python tools/trace_step.py TRACE_DIR [KERNEL_SUBSTRING] [STEPS]"""
import csv
import sys

d = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "classify2"
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rows = sorted(csv.DictReader(open(f"{d}/trace_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
s, e = idx[-1 - nsteps], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
t_end = int(rows[e]["Start_Timestamp"])
busy, cur_s, cur_e = 0, None, None
for r in rows[s:e]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("rocprim::ROCPRIM_400200_NS::detail::", "")[:64]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} s{r['Stream_Id']} {n}")
    en = min(en, t_end)
    if cur_e is None or st > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = st, en
    else:
        cur_e = max(cur_e, en)
if cur_e is not None:
    busy += cur_e - cur_s
span = t_end - t0
print(f"window {span / 1e3:.1f} us over {nsteps} step(s): some kernel running {busy / 1e3:.1f} us, "
      f"none {(span - busy) / 1e3:.1f} us")
