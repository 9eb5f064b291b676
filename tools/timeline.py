#!/usr/bin/env python3
"""Timeline of the last step(s) of a rocprofv3 trace (kernel + HIP API + copies).

Usage: python tools/timeline.py TRACE_DIR [--last-ms 1.0] [--prefix tr]
Prints every kernel, copy and (non-trivial) HIP API call in the window, sorted by
start time, with its start offset, duration and the idle gap on the GPU before
each kernel/copy.  Diagnostic only.
"""
import argparse
import csv
import os


def load(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--prefix", default="tr")
    ap.add_argument("--last-ms", type=float, default=1.0)
    ap.add_argument("--min-api-us", type=float, default=2.0)
    ap.add_argument("--back-ms", type=float, default=0.0, help="end the window this long before the last kernel")
    a = ap.parse_args()
    ev = []
    for r in load(os.path.join(a.dir, f"{a.prefix}_kernel_trace.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
        ev.append(("K", int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:48], r["Stream_Id"]))
    for r in load(os.path.join(a.dir, f"{a.prefix}_memory_copy_trace.csv")):
        ev.append(("C", int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""),
                   r["Stream_Id"]))
    for r in load(os.path.join(a.dir, f"{a.prefix}_hip_api_trace.csv")):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if (e - s) / 1e3 >= a.min_api_us:
            ev.append(("A", s, e, r["Function"], r["Thread_Id"]))
    ev.sort(key=lambda x: x[1])
    t_end = max(x[2] for x in ev if x[0] == "K") - int(a.back_ms * 1e6)
    t0 = t_end - int(a.last_ms * 1e6)
    gpu_busy_until = None
    busy = 0
    for kind, s, e, name, sid in ev:
        if s > t_end:
            break
        if e < t0:
            if kind != "A":
                gpu_busy_until = max(gpu_busy_until or 0, e)
            continue
        gap = ""
        if kind != "A":
            if gpu_busy_until is not None and s > gpu_busy_until:
                gap = f"gap {(s - gpu_busy_until) / 1e3:7.1f}"
            gpu_busy_until = max(gpu_busy_until or 0, e)
            busy += e - max(s, t0)
        print(f"{(s - t0) / 1e3:9.1f} us  {kind} {(e - s) / 1e3:8.1f} us  {gap:>12}  s{sid:>3} {name}")
    print(f"window {a.last_ms} ms: GPU busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
