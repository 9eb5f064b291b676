#!/usr/bin/env python3
"""Benchmark: k-mer profile + shared-read graph build on MI355X (BASELINE.json metric).

One step = the whole hot path over one batch of device-resident synthetic input
(SURVEY.md §8(d)), per GPU:
  k-mer profile of 200k contigs (mean 800 bp, k = 5p6): presence pass, column
  table, dense float64 profile (N x M) written to HBM;
  shared-read graph of 100M paired fragments (~309M (read, contig) records):
  one partition pass (a read -> one 2-byte (m0, M) code, or its pairs),
  LDS histogram / hash reduces, per-bucket merge, weights.
Inputs (2-bit packed contigs + records) are resident in HBM before timing.

Multi-GPU (torchrun, one rank per GPU): weak scaling — rank r owns contig rows
[r*200k, (r+1)*200k) and fragments [r*100M, (r+1)*100M) of a global problem
whose genes span all ranks; the step adds the presence OR-allreduce, the edge
partial all-to-all (pre-reduced pairs routed to the owner of contig a) and the
totals allgather over RCCL (karma_amd/distributed.py).

Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# kernels with an algorithmic-bytes figure: the roofline kernel is the slowest of these
ROOFLINE_KERNELS = ("kmer_profile", "kmer_presence", "graph_classify", "graph_code_partition", "graph_code_reduce")

CONFIGS = {
    # name: (seed, contigs per GPU, fragments per GPU, paired, kmer)
    "config3": (3, 200_000, 100_000_000, True, "5p6"),
    "config2": (2, 50_000, 10_000_000, True, "5p6"),
    "config1": (1, 1_000, 100_000, False, 5),
    "tiny": (7, 5_000, 500_000, True, "5p6"),
    # configs[4] (1M contigs, 500M paired fragments, k=7) as its per-GPU share on 8 GPUs,
    # and the whole problem on one GPU (a 131 GB profile + 1.5e9 records fit in 288 GB HBM)
    "config5": (5, 125_000, 62_500_000, True, 7),
    "config5_1gpu": (5, 1_000_000, 500_000_000, True, 7),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-sample", type=float, default=0.1,
                    help="fraction of the per-GPU workload the CPU baseline processes (0 disables)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP-event timing")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="diagnostic: one process runs rank 0's compute of a W-rank weak-scaled problem "
                         "(global contig ids over W x the per-GPU contigs; the exchange's local work - device split, "
                         "merge of W sorted slices, totals - without its collectives); not the metric")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch

    from karma_amd import _lib, engine
    from karma_amd.distributed import Comm, ShardedBuild

    seed, n_loc, f_loc, paired, kmer = CONFIGS[args.config]
    # KARMA_FORCE_DEVICE pins every rank to one device (multi-rank rehearsal on
    # a 1-GPU box together with KARMA_DIST_BACKEND=gloo); unset in real runs
    dev_index = int(os.environ.get("KARMA_FORCE_DEVICE", local_rank if world > 1 else 0))
    comm = Comm.create(world, rank, dev_index)
    ctx = _lib.Context(dev_index)
    torch.cuda.set_device(dev_index)

    # ---------------- synthetic input (host), then resident in HBM ----------------
    t_gen = time.time()
    emu = max(1, args.emulate_ranks) if world == 1 else 1
    n_glob, f_glob = n_loc * world * emu, f_loc * world * emu
    c_lo = rank * n_loc
    blob, offs, key_len = engine.synth_contigs(seed, n_loc, 400, 800, 0, first=c_lo)
    genes = engine.synth_genes(seed, n_glob)
    rec = engine.synth_records(seed, n_glob, rank * f_loc, (rank + 1) * f_loc, paired, genes=genes)
    A = len(rec)
    log(f"[rank {rank}] generated {n_loc} contigs ({int(offs[-1])} bases), {f_loc} fragments, {A} records "
        f"in {time.time() - t_gen:.1f}s")

    build = ShardedBuild(ctx, comm, engine.kmode_of(kmer), n_glob, c_lo, n_loc,
                         emulate_ranks=emu)  # sets the shared stream
    store = engine.ContigStore(ctx, blob, offs, key_len)
    rec_dev = torch.from_numpy(rec.view(np.int64).reshape(-1)).to(build.ops.dev)
    torch.cuda.synchronize()
    packed_bytes = int(np.sum((np.diff(offs) + 3) // 4))  # sum ceil(L/4)

    def step(keep=False):
        return build.run(store, rec_dev.data_ptr(), A, keep=keep)

    ctxs = build.contexts()  # main context (+ the concurrent graph build's)

    def sync_all():
        for c in ctxs:
            c.sync()

    def timed_pass(only=None):
        """args.steps steps with HIP-event timing (all kernels, or one) -> {kernel: (ms, launches)}."""
        for c in ctxs:
            c.timing(True, only)
            c.timing_reset()
        for _ in range(args.steps):
            step()
        sync_all()
        kern = {}
        for c in ctxs:
            for name, (ms, nl) in c.timing_read().items():
                prev = kern.get(name, (0.0, 0))
                kern[name] = (prev[0] + ms, prev[1] + nl)
            c.timing(False)
        return kern

    for _ in range(args.warmup):
        step()
    sync_all()
    # per-kernel breakdown (events on every launch), outside the timed region
    kern = timed_pass() if not args.no_timing else {}
    dom = max((k for k in kern if k in ROOFLINE_KERNELS), key=lambda k: kern[k][0], default=None)
    # timed region: events only around the dominant kernel's launches (two
    # per launch), so the wall time carries almost no instrumentation
    if dom:
        for c in ctxs:
            c.timing(True, dom)
            c.timing_reset()
    comm.barrier()
    torch.cuda.synchronize()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    sync_all()
    torch.cuda.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    dt = comm.max_float(t1 - t0)
    dom_live = None
    if dom:
        for c in ctxs:
            got = c.timing_read().get(dom)
            if got:
                dom_live = got if dom_live is None else (dom_live[0] + got[0], dom_live[1] + got[1])
            c.timing(False)
    n_reads = int(np.count_nonzero(rec[1:, 0] != rec[:-1, 0])) + 1 if A else 0

    units = world * (n_loc + f_loc) * args.steps
    value = units / dt
    M = res["M"]
    E = comm.sum_int(res["E_local"])
    # algorithmic bytes per launch, DESIGN.md §Measurement
    per_kernel_bytes = {
        "kmer_profile": packed_bytes + 8 * n_loc * M,
        "kmer_presence": packed_bytes,
        # records read once, one 4-byte code per (compact) read written
        "graph_classify": 8 * A + 4 * n_reads,
        # codes read, 2-byte bucket-local codes written
        "graph_code_partition": 6 * n_reads,
        "graph_code_reduce": 2 * n_reads,
    }
    roof = None
    if dom_live and dom in per_kernel_bytes:
        ms, nl = dom_live
        avg_s = ms / nl / 1e3
        achieved = per_kernel_bytes[dom] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": pmc_traffic(dom),
                "bytes_per_launch": per_kernel_bytes[dom], "avg_launch_ms": round(ms / nl, 4)}
    step_bytes = packed_bytes + 8 * n_loc * M + 8 * A + 16 * res["E_local"] + 8 * n_loc
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline(seed, n_loc, f_loc, paired, kmer, args.cpu_sample, blob, offs, rec)

    if rank == 0:
        line = {
            "metric": "contigs+reads/sec for k-mer vec + shared-read graph build; HBM GB/s vs roofline",
            "value": round(value, 1),
            "unit": "(contigs+fragments)/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 keys / i64 counts / f64 div",
            "data": "synthetic (SplitMix64 generator, SURVEY.md §8(d))",
            "config": {"workload": f"{args.config}: {n_loc} contigs (mean 800 bp) + {f_loc} "
                                   f"{'paired' if paired else 'single-end'} fragments per GPU, k={kmer}",
                       "contigs_per_gpu": n_loc, "fragments_per_gpu": f_loc, "records_per_gpu": A,
                       "columns_M": M, "edges": E, "parallelism": f"contig+fragment shards x{world}",
                       **({"emulated_ranks": emu, "global_contigs": n_glob} if emu > 1 else {})},
            "roofline": roof,
            "step_hbm_bytes_per_gpu": step_bytes,
            "step_achieved_GBs_per_gpu": round(step_bytes / (dt / args.steps) / 1e9, 1),
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in kern.items()},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    build.close()
    store.close()
    comm.close()


def pmc_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel)
    except (OSError, ValueError):
        return None


def cpu_baseline(seed, n_loc, f_loc, paired, kmer, frac, blob, offs, rec):
    """Oracle (single-threaded C restatement, oracle/) on a bounded sample."""
    try:
        from collections import OrderedDict

        from oracle import oracle
    except Exception as e:  # oracle not built on this box
        return {"error": f"oracle unavailable: {e}"}
    ns = max(1, int(n_loc * frac))
    fs = max(1, int(f_loc * frac))
    seqs = OrderedDict((f">ctg{i}", bytes(blob[offs[i]:offs[i + 1]]).decode()) for i in range(ns))
    t0 = time.perf_counter()
    oracle.calc_kmer_profile(seqs, kmer)
    t1 = time.perf_counter()
    r = rec[rec[:, 0] < fs].astype(np.int64)
    starts = np.flatnonzero(np.r_[True, r[1:, 0] != r[:-1, 0]])
    off = np.r_[starts, len(r)]
    t2 = time.perf_counter()
    oracle.graph_groups(off, r[:, 1], None, None, n_loc, dedup=True)
    t3 = time.perf_counter()
    secs = (t1 - t0) + (t3 - t2)
    return {"value": round((ns + fs) / secs, 1), "unit": "(contigs+fragments)/s", "cores": 1, "kind": "port",
            "sample": f"{ns} contigs k={kmer} profile ({t1 - t0:.2f}s) + graph of {fs} fragments / {len(r)} records "
                      f"({t3 - t2:.2f}s) = {frac:.0%} of the per-GPU workload, oracle/ C restatement, 1 thread"}


if __name__ == "__main__":
    main()
