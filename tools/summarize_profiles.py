#!/usr/bin/env python3
"""Fold measurement scratch under profiles/ into one summary table per experiment.

Every A/B and preview directory (profiles/r0*/ab_*, meas_*) becomes a single
SUMMARY.md: one row per bench line (ms/step, parity, the roofline kernel's
launch time, the kernels above 12 us), per kernel-trace CSV (the top kernels by
total time), and the names of the text files it held.  Older rocprof
directories that DESIGN.md no longer cites are folded the same way into
profiles/r0X/ROCPROF_INDEX.md.  The raw files are then removed from the tree
(git history keeps them).  CPU only.

  python tools/summarize_profiles.py [--dry-run]
"""
import argparse
import csv
import glob
import json
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
# rocprof directories kept whole (cited as the evidence of the current numbers)
KEEP_ROCPROF = {"r03/rocprof_z", "r03/rocprof_emu8_n", "r02/rocprof_j", "r01/rocprof_v11"}


def short(name, n=48):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.split("(")[0] if not name.startswith("void") else name[5:].split("(")[0]
    return name[:n]


def bench_row(path):
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except (ValueError, IndexError, OSError):
        return None
    k = d.get("kernels_ms_per_step") or {}
    big = ", ".join(f"{n} {v}" for n, v in sorted(k.items(), key=lambda x: -x[1]) if v > 0.012)
    roof = d.get("roofline") or {}
    return (f"| {os.path.basename(path)} | {d.get('ms_per_step')} | {d.get('parity')} | "
            f"{roof.get('kernel', '')} {roof.get('avg_launch_ms', '')} | {big} |")


def csv_rows(path, top=6):
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        return None
    if not rows or "TotalDurationNs" not in rows[0]:
        return None
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    cells = "; ".join(f"{short(r['Name'])} x{r['Calls']} avg {float(r['AverageNs']) / 1e3:.1f} us" for r in rows[:top])
    return f"| {os.path.basename(path)} | {cells} |"


def summarize(d, title):
    files = sorted(glob.glob(os.path.join(d, "*")))
    out = [f"# {title}", "",
           "Folded from the raw files of this directory (tools/summarize_profiles.py; git history holds them).", ""]
    benches = [r for r in (bench_row(f) for f in files if f.endswith(".json")) if r]
    if benches:
        out += ["| bench line | ms/step | parity | roofline kernel (avg ms) | kernels > 12 us (ms/step) |",
                "|---|---|---|---|---|"] + benches + [""]
    traces = [r for r in (csv_rows(f) for f in files if f.endswith(".csv")) if r]
    if traces:
        out += ["| kernel trace | top kernels by total time |", "|---|---|"] + traces + [""]
    other = [os.path.basename(f) for f in files if not f.endswith((".json", ".csv", ".md"))]
    if other:
        out += ["Other files (text traces, notes): " + ", ".join(other), ""]
        for f in files:
            if f.endswith(".txt") and os.path.getsize(f) < 4000:
                out += [f"## {os.path.basename(f)}", "", "```", open(f).read().rstrip(), "```", ""]
    return "\n".join(out) + "\n", files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args()
    removed = 0
    for d in sorted(glob.glob(os.path.join(PROF, "r0*", "*"))):
        if not os.path.isdir(d):
            continue
        rel = os.path.relpath(d, PROF)
        base = os.path.basename(d)
        if base.startswith(("ab_", "meas_")):
            text, files = summarize(d, rel)
            target = os.path.join(d, "SUMMARY.md")
        elif base.startswith("rocprof") and rel not in KEEP_ROCPROF:
            text, files = summarize(d, rel)
            target = None
        else:
            continue
        drop = [f for f in files if not f.endswith("SUMMARY.md")]
        if a.dry_run:
            print(rel, len(drop), "files")
            continue
        if target:
            with open(target, "w") as f:
                f.write(text)
        else:
            idx = os.path.join(os.path.dirname(d), "ROCPROF_INDEX.md")
            with open(idx, "a") as f:
                f.write(text.replace("# ", "## ", 1) + "\n")
        subprocess.run(["git", "rm", "-q", "-r", "--cached", "--ignore-unmatch", *drop], cwd=REPO, check=True)
        for f in drop:
            os.remove(f)
        if not target:
            os.rmdir(d)
        removed += len(drop)
    print("removed", removed, "files")


if __name__ == "__main__":
    main()
