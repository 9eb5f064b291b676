#!/usr/bin/env python3
"""profiles/pmc_traffic.json: HBM bytes per launch of the bench's kernels.

Input: the per-kernel JSON of profiles/pmc_summary.py (rocprofv3 FETCH_SIZE and
WRITE_SIZE passes, KiB per dispatch, reported there as MB).  Correction as
MI355X_MICROARCH.md §HBM prescribes: on gfx950 FETCH_SIZE reports 1/2 of a
wide (16 B/lane) streaming read, so reads are doubled; WRITE_SIZE is exact for
16-B stores.  graph_classify, the partition and kmer_profile move 16 B per lane.
The code reduces read short runs (~110 B per chunk and bucket) for which
FETCH_SIZE counts the bytes themselves (calibrated in round 6 with
tools/micro/seg_read.hip: x 0.986 on a known byte count), so their reads are
not doubled -- except where the binned classify writes whole 128-byte slots
(config 3, "slotted"): the reduce then reads aligned 128-byte segments, the
wide case (fix such entries by hand; profiles/pmc_traffic.json says which).

The output is keyed by workload (bench.py pmc_traffic(): "<config>[_strong]
[_shuffled]_n<ranks>"), so a number is only ever reported for the workload
whose PMC runs produced it; other keys in an existing out.json are kept.

Usage: python tools/pmc_traffic.py pmc_summary.json out.json WORKLOAD_KEY [SOURCE]
"""
import json
import sys

# rocprof kernel name (template arguments dropped) -> bench.py kernel (KARMA_LAUNCH) name
NAMES = {
    "classify_kernel": "graph_classify",
    "classify2_kernel": "graph_classify",
    "code_append_kernel": "graph_code_partition",
    "partition_kernel<CodeStream": "graph_code_partition",
    "code_reduce_kernel": "graph_code_reduce",
    "code_seg_reduce_kernel": "graph_code_reduce",
    "profile_kernel": "kmer_profile",
    "profile_wave_kernel": "kmer_profile",
    "presence_kernel": "kmer_presence",
}


def bench_name(k):
    base = k.split("<")[0]
    if base == "partition_kernel":  # the pair partition is another kernel name in bench.py
        return NAMES["partition_kernel<CodeStream"] if "CodeStream" in k else None
    return NAMES.get(base)


def main():
    src = json.load(open(sys.argv[1]))
    out = {}
    for k, v in src.items():
        name = bench_name(k)
        if name and v.get("fetch_MB") == v.get("fetch_MB"):  # skip NaN
            fx = 1 if name == "graph_code_reduce" else 2
            out[name] = int(round((fx * v["fetch_MB"] + v["write_MB"]) * 1024 * 1024))
    dst, key = sys.argv[2], sys.argv[3]
    try:
        allw = json.load(open(dst))
    except (OSError, ValueError):
        allw = {}
    if len(sys.argv) > 4:
        out["_source"] = sys.argv[4]
    allw[key] = out
    json.dump(allw, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(allw[key]))


if __name__ == "__main__":
    main()
