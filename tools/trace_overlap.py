#!/usr/bin/env python3
"""Timeline of the last N steps of a rocprofv3 kernel trace (bench.py's timed
loop): per step, when classify, the segment reduce, the final kernel and the
profile ran, and how long classify of step i+1 overlapped the profile of step
i.  Usage: trace_overlap.py DIR/trace_kernel_trace.csv [N]"""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(path)))
ks = []
for r in rows:
    name = r["Kernel_Name"]
    short = None
    for key, lab in (("classify2_kernel", "classify"), ("profile_wave_kernel", "profile"),
                     ("code_seg_reduce_kernel", "reduce"), ("final_kernel", "final"),
                     ("presence_kernel", "presence"), ("columns_kernel", "columns"),
                     ("step_status_kernel", "status"), ("step_edge_write", "edge_w")):
        if key in name:
            short = lab
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short or name.split("(")[0][-30:],
               r["Queue_Id"], int(r["VGPR_Count"]), int(r["LDS_Block_Size"])))
ks.sort()
cls = [k for k in ks if k[2] == "classify"][-n:]
prof = [k for k in ks if k[2] == "profile"]
t0 = cls[0][0]
print(f"classify VGPR {cls[0][4]} LDS {cls[0][5]}; profile VGPR {prof[-1][4]} LDS {prof[-1][5]}")
tot_ovl = 0.0
for i, c in enumerate(cls):
    # the profile that started last before this classify (the previous step's)
    pv = [p for p in prof if p[0] < c[0]]
    p = pv[-1] if pv else None
    ovl = max(0, min(c[1], p[1]) - max(c[0], p[0])) / 1e3 if p else 0.0
    tot_ovl += ovl
    nxt = [p2 for p2 in prof if p2[0] >= c[0]]
    pn = nxt[0] if nxt else None
    print(f"step {i:2d}: classify {(c[0]-t0)/1e3:9.1f} +{(c[1]-c[0])/1e3:6.1f} us (q{c[3]}) | prev profile ends "
          f"{((p[1]-t0)/1e3 if p else 0):9.1f} overlap {ovl:6.1f} | own profile {(pn[0]-t0)/1e3 if pn else 0:9.1f} "
          f"+{(pn[1]-pn[0])/1e3 if pn else 0:6.1f} (q{pn[3] if pn else '-'})")
span = (cls[-1][0] - cls[0][0]) / 1e3 / (len(cls) - 1)
print(f"classify-to-classify {span:.1f} us per step; mean overlap with the previous profile {tot_ovl/len(cls):.1f} us")
