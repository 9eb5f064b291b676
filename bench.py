#!/usr/bin/env python3
"""Benchmark: k-mer profile + shared-read graph build on MI355X (BASELINE.json metric).

One step = the whole hot path over one batch of device-resident synthetic input
(SURVEY.md §8(d)), per GPU:
  k-mer profile of 200k contigs (mean 800 bp, k = 5p6): presence pass, column
  table, dense float64 profile (N x M) written to HBM;
  shared-read graph of 100M paired fragments (~309M (read, contig) records):
  one classification pass (a read -> one 2-byte (m0, M) code, or its pairs),
  partition, LDS histogram / hash reduces, per-bucket merge, weights.
Inputs (2-bit packed contigs + records) are resident in HBM before timing.

Multi-GPU (torchrun, one rank per GPU, the library's own RCCL communicator;
no PyTorch in the process):
  default (strong) BASELINE configs[3]: config 3 itself (200k contigs, 100M
                  fragments) divided over the N ranks; a weak leg follows under
                  "weak" (--no-weak-leg skips it);
  --weak          headline = weak scaling: rank r owns contig rows
                  [r*200k, (r+1)*200k) and fragments [r*100M, (r+1)*100M) of a
                  global problem whose genes span all ranks.
The step adds the presence all-gather, the exception-key all-gather, the edge
partial all-to-all-v (pre-reduced pairs routed to the owner of contig a) and
the totals all-gather (karma_amd/distributed.py, karma_amd/comm.py).

Prints ONE JSON line on rank 0 (DESIGN.md §5 defines every field).
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
    ap.add_argument("--steps", type=int, default=100,
                    help="timed batches; the two-stream pipeline's fill and drain are paid once per timed loop "
                         "(DESIGN.md §5), so 100 batches measure the steady stream (20: +0.04 ms/step at 8 ranks)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--weak", action="store_true",
                    help="headline = weak scaling (every rank a whole config-sized share of a W x larger problem); "
                         "default strong (BASELINE configs[3]: the config divided over the ranks)")
    ap.add_argument("--strong", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--no-weak-leg", action="store_true",
                    help="N > 1: skip the extra weak-scaling leg reported under \"weak\"")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="diagnostic: one process runs rank 0's compute of a W-rank problem (weak: global contig "
                         "ids over W x the per-GPU contigs; strong: 1/W of the config) with the exchange's local "
                         "work (device split, merge of W sorted slices, totals) and no collectives; not the metric")
    ap.add_argument("--shuffle-contigs", action="store_true",
                    help="secondary number: contig ids randomly permuted (a FASTA without isoform adjacency; same "
                         "graph up to relabelling)")
    ap.add_argument("--cpu-baseline", choices=("full", "off"), default="full",
                    help="full: the oracle's OpenMP twin on the whole per-GPU workload (rank 0, N = 1)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP-event timing")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end, drop-in and eq-path legs")
    ap.add_argument("--no-parity", action="store_true", help="skip the in-run digest check")
    ap.add_argument("--records", choices=("flagged", "pairs"), default="flagged",
                    help="device format of the read->contig records the step takes: flagged (KARMA_REC_FLAGGED, "
                         "u32 contig | read-start << 31: the graph depends only on which records share a read) or "
                         "pairs ({u32 read id, u32 contig}); the other format is timed too, as records_other")
    ap.add_argument("--no-other-format", action="store_true", help="skip the records_other leg")
    a = ap.parse_args()
    a.strong = not a.weak
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Watchdog:
    """Ends the process (non-zero, without teardown) when no phase or step
    has ticked for `limit` seconds: a rank whose peer stopped issuing
    collectives would otherwise wait in a device synchronisation until the
    driver's own timeout.  os._exit, because teardown would wait on the same
    stalled streams."""

    def __init__(self):
        self.limit = float(os.environ.get("KARMA_BENCH_STALL_S", "300"))
        self.what, self.t = "start", time.monotonic()
        self.rank = 0
        self._thread = None

    def start(self, rank):
        import threading

        self.rank = rank
        if self.limit > 0 and self._thread is None:
            self._thread = threading.Thread(target=self._run, daemon=True, name="bench-watchdog")
            self._thread.start()

    def tick(self, what):
        self.what, self.t = what, time.monotonic()

    def _run(self):
        while True:
            time.sleep(min(5.0, self.limit / 4))
            idle = time.monotonic() - self.t
            if idle > self.limit:
                log(f"bench.py: rank {self.rank} made no progress for {idle:.0f} s after '{self.what}' "
                    f"(KARMA_BENCH_STALL_S={self.limit:g}); exiting without teardown")
                os._exit(5)


WATCHDOG = Watchdog()


def stalled_exit(rank, err):
    """A deferred step's status never arrived (KARMA_ERR_STALL: a peer's or the
    device's collectives stalled): report it and leave at once -- destroying the
    streams would wait on the stalled work."""
    log(f"bench.py: rank {rank}: {err}")
    os._exit(4)


def visible_devices():
    """HIP devices visible to a child process (this process must not touch HIP
    before it starts the ranks: karma_device_count runs in a child)."""
    import subprocess

    code = ("import ctypes, sys; sys.path.insert(0, %r); from karma_amd import _lib; n = ctypes.c_int(0); "
            "rc = _lib.load().karma_device_count(ctypes.byref(n)); print(n.value if rc == 0 else 0)" % REPO)
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else 0
    except (subprocess.TimeoutExpired, ValueError, OSError):
        return 0


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_envs(n, port, base=None):
    """The environment of each of n self-launched ranks (what torchrun would set)."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KARMA_BENCH_LAUNCHER="self")
        out.append(e)
    return out


def launch_ranks(n, cmd, envs, poll=0.2):
    """Start one child per rank (never exec: the parent stays a plain waiter),
    wait for all; when one fails, stop the others (their exact PIDs) and
    return its exit code.  Rank 0's stdout is the line (inherited)."""
    import subprocess

    procs = [subprocess.Popen(cmd, env=envs[r]) for r in range(n)]
    rc = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c
                    log(f"bench.py: rank {r} exited with {c}; stopping the other ranks")
                    for q in live:
                        procs[q].terminate()
            time.sleep(poll)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc


def self_launch(args):
    """--gpus N > 1 with no launcher (WORLD_SIZE unset): start N rank
    processes as torchrun would (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR
    127.0.0.1, MASTER_PORT), one per device, and return the first failing
    exit code (0 when all succeed).  Fewer visible devices than N is an error,
    unless KARMA_FORCE_DEVICE pins every rank to one device (the host-staged
    rehearsal on a one-GPU box: KARMA_DIST_BACKEND=host)."""
    n = args.gpus
    if os.environ.get("KARMA_FORCE_DEVICE") is None:
        nd = visible_devices()
        if nd < n:
            log(f"bench.py: --gpus {n} but {nd} HIP device(s) visible; refusing to report an {n}-GPU line")
            return 2
    log(f"bench.py: launching {n} ranks (no WORLD_SIZE in the environment)")
    return launch_ranks(n, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:],
                        rank_envs(n, free_port()))


def shard(total, world, rank):
    return total * rank // world, total * (rank + 1) // world


def make_inputs(args, rank, world):
    """This rank's contigs and records.  Returns a dict (see keys below)."""
    from karma_amd import engine

    seed, n_cfg, f_cfg, paired, kmer = CONFIGS[args.config]
    emu = max(1, args.emulate_ranks) if world == 1 else 1
    parts = world * emu
    if args.strong:
        n_glob, f_glob = n_cfg, f_cfg
        c_lo, c_hi = shard(n_glob, parts, rank)
        f_lo, f_hi = shard(f_glob, parts, rank)
    else:
        n_glob, f_glob = n_cfg * parts, f_cfg * parts
        c_lo, c_hi = rank * n_cfg, (rank + 1) * n_cfg
        f_lo, f_hi = rank * f_cfg, (rank + 1) * f_cfg
    blob, offs, key_len = engine.synth_contigs(seed, c_hi - c_lo, 400, 800, 0, first=c_lo)
    genes = engine.synth_genes(seed, n_glob)
    rec = engine.synth_records(seed, n_glob, f_lo, f_hi, paired, genes=genes)
    perm = None
    if args.shuffle_contigs:
        # the same graph with contig ids relabelled by a fixed random permutation
        perm = np.random.default_rng(12345).permutation(n_glob).astype(np.uint32)
        rec = np.ascontiguousarray(rec)
        rec[:, 1] = perm[rec[:, 1]]
    return dict(seed=seed, paired=paired, kmer=kmer, emu=emu, n_glob=n_glob, f_glob=f_glob, c_lo=c_lo,
                n_loc=c_hi - c_lo, f_lo=f_lo, f_loc=f_hi - f_lo, blob=blob, offs=offs, key_len=key_len,
                genes=genes, rec=rec, perm=perm)


class Leg:
    """One workload resident on this rank's GPU: inputs, ShardedBuild, device store and records."""

    def __init__(self, args, ctx, comm, rank, world):
        from karma_amd import _lib, engine
        from karma_amd.distributed import ShardedBuild

        t_gen = time.time()
        self.args, self.comm, self.rank, self.world = args, comm, rank, world
        self.inp = inp = make_inputs(args, rank, world)
        WATCHDOG.tick("inputs generated")
        self.A = len(inp["rec"])
        log(f"[rank {rank}] {'strong' if args.strong else 'weak'}: generated {inp['n_loc']} contigs "
            f"({int(inp['offs'][-1])} bases), {inp['f_loc']} fragments, {self.A} records in "
            f"{time.time() - t_gen:.1f}s")
        # the records on the device in the step's format: KARMA_REC_FLAGGED words
        # (4 bytes per record) or (read, contig) pairs (8), the same records
        self.flagged = args.records == "flagged"
        self.rec_bytes = 4 if self.flagged else 8
        self.build = ShardedBuild(ctx, comm, engine.kmode_of(inp["kmer"]), inp["n_glob"], inp["c_lo"], inp["n_loc"],
                                  emulate_ranks=inp["emu"], flagged=self.flagged)  # library-owned streams
        self.store = engine.ContigStore(ctx, inp["blob"], inp["offs"], inp["key_len"])
        self.rec_dev = _lib.DevBuf.from_numpy(ctx, engine.flag_records(inp["rec"]) if self.flagged
                                              else inp["rec"].view(np.int64).reshape(-1))
        ctx.sync()
        self.packed_bytes = int(np.sum((np.diff(inp["offs"]) + 3) // 4))  # sum ceil(L/4)
        self.ctxs = self.build.contexts()  # main context (+ the concurrent graph build's)

    def step(self, keep=False, sequential=False, count=True):
        return self.build.run(self.store, self.rec_dev.ptr, self.A, keep=keep, sequential=sequential, count=count)

    def sync_all(self):
        self.build.sync()  # every enqueued step, deferred checks included, and the contexts

    def timed(self, steps, warmup, kernel_timing=True):
        """W untimed steps, an optional per-kernel pass, then K steps bracketed by
        barrier + device sync; returns (max-over-ranks seconds, last result,
        per-kernel totals, dominant kernel, its live (ms, launches))."""
        comm = self.comm
        # with the native step the timed batches are deferred ones (below): the
        # warm-up runs that same kind of step, so both main streams' tail
        # buffers, control blocks and events exist before the timed region (the
        # sequential pass uses only the first; a first deferred batch on the
        # second stream grew them with every stream synchronised, inside the
        # timed loop: a fixed cost per loop that 20 short batches did not hide)
        native = self.build.native is not None and os.environ.get("KARMA_BENCH_LAST_SYNC", "0") != "1"
        for i in range(warmup):
            self.step(count=not native)
            WATCHDOG.tick(f"warmup step {i}")
        self.sync_all()
        WATCHDOG.tick("warmup synced")
        # Per-kernel breakdown, outside the timed region, with every launch timed
        # and the profile on the main stream (sequential): kernels do not share the
        # chip, so no launch is charged for time it spent queued behind another.
        kern = {}
        if kernel_timing:
            for c in self.ctxs:
                c.timing(True)
                c.timing_reset()
            for _ in range(steps):  # the same kernels as the timed steps (deferred where they are)
                self.step(sequential=True, count=False)
            self.sync_all()
            WATCHDOG.tick("per-kernel pass")
            for c in self.ctxs:
                for name, (ms, nl) in c.timing_read().items():
                    prev = kern.get(name, (0.0, 0))
                    kern[name] = (prev[0] + ms, prev[1] + nl)
                c.timing(False)
        dom = max((k for k in kern if k in ROOFLINE_KERNELS), key=lambda k: kern[k][0], default=None)
        # timed region: the production order (profile on the side stream), with
        # events only around the dominant kernel's launches (two per launch)
        if dom:
            for c in self.ctxs:
                c.timing(True, dom)
                c.timing_reset()
        from karma_amd import _lib

        comm.barrier()
        self.sync_all()
        calls0 = _lib.api_calls()
        info0 = self.build.native.info() if self.build.native is not None else None
        host = 0.0
        t0 = time.perf_counter()
        # a stream of batches: the outputs of every step but the last are not
        # read (ShardedBuild.run count=False), so in one process a step returns
        # without waiting for anything (karma_step's deferred path: its checks
        # arrive through mapped memory, a step needing the general path runs
        # again synchronously) and with an exchange the owner's edge count is
        # not read back; every kernel still runs, and the sync below waits for
        # all of them and checks every step
        # with the native step the last batch is deferred too: its column count
        # and edge count are read from its status after the sync (the same
        # kernels run; only the host's readback moves behind the sync)
        for i in range(steps):
            h0 = time.perf_counter()
            res = self.step(count=i == steps - 1 and not native)
            host += time.perf_counter() - h0
            WATCHDOG.tick(f"timed step {i}")
        info_loop = self.build.native.info() if self.build.native is not None else None
        d0 = time.perf_counter()
        self.sync_all()
        comm.barrier()
        t1 = time.perf_counter()
        # the drain after the loop (every step still in flight, its checks, the
        # barrier): part of the timed region, not of the step calls
        self.drain_us = (t1 - d0) * 1e6
        if native:
            info = self.build.native.info()
            res = dict(res, M=int(info[0]), E_local=int(info[1]))
        dt = comm.max_float(t1 - t0)
        self.host_us_per_step = host / steps * 1e6
        self.api_calls_per_step = (_lib.api_calls() - calls0) / steps
        self.step_info = self.build.native.info().tolist() if self.build.native is not None else None
        # of the host time inside the step calls: waiting for the device (a
        # deferred step's status kLag steps back) vs enqueueing the step; the
        # drain's waits (karma_step_sync after the loop) are reported apart
        self.host_wait_us_per_step = ((int(info_loop[9]) - int(info0[9])) / steps / 1e3
                                      if info0 is not None else None)
        self.drain_wait_us = (self.step_info[9] - int(info_loop[9])) / 1e3 if info0 is not None else None
        self.step_mode = self.build.native.mode() if self.build.native is not None else None
        dom_live = None
        if dom:
            for c in self.ctxs:
                got = c.timing_read().get(dom)
                if got:
                    dom_live = got if dom_live is None else (dom_live[0] + got[0], dom_live[1] + got[1])
                c.timing(False)
        return dt, res, kern, dom, dom_live

    def single_batch(self, reps=5):
        """One batch alone: from every stream idle (barrier + device sync) to
        its checked status (karma_step_sync), the latency a karma run sees when
        it builds this path once (karma.py:197-210, :240); a deferred step with
        the native driver, as in the timed loop.  Median over reps of the max
        over ranks (ms)."""
        native = self.build.native is not None
        ts = []
        for _ in range(reps):
            self.comm.barrier()
            self.sync_all()
            t0 = time.perf_counter()
            self.step(count=not native)
            self.sync_all()
            ts.append(self.comm.max_float(time.perf_counter() - t0) * 1e3)
        return {"ms": round(float(np.median(ts)), 4), "min_ms": round(min(ts), 4), "reps": reps,
                "step": "deferred" if native else "synchronous",
                "note": "one batch from idle streams to its synced, checked status (no pipelining with other "
                        "batches); median over reps of the max over ranks"}

    def other_format(self, steps, warmup):
        """The same workload with the records in the other device format (a
        second build on the same store; same step kinds, no per-kernel pass):
        {ms_per_step, value} so both formats are measured in one line."""
        from karma_amd import _lib, engine
        from karma_amd.distributed import ShardedBuild

        inp, ctx = self.inp, self.rec_dev.ctx
        flagged = not self.flagged
        build = ShardedBuild(ctx, self.comm, engine.kmode_of(inp["kmer"]), inp["n_glob"], inp["c_lo"], inp["n_loc"],
                             emulate_ranks=inp["emu"], flagged=flagged)
        dev = _lib.DevBuf.from_numpy(ctx, engine.flag_records(inp["rec"]) if flagged
                                     else inp["rec"].view(np.int64).reshape(-1))
        try:
            native = build.native is not None
            run = lambda: build.run(self.store, dev.ptr, self.A, count=not native)  # noqa: E731
            for _ in range(warmup):
                run()
            build.sync()
            self.comm.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                run()
            build.sync()
            self.comm.barrier()
            dt = self.comm.max_float(time.perf_counter() - t0)
        finally:
            build.close()
            dev.close()
        units = self.comm.sum_int(inp["n_loc"] + inp["f_loc"]) * steps
        return {"format": "flagged" if flagged else "pairs", "bytes_per_record": 4 if flagged else 8,
                "ms_per_step": round(dt / steps * 1e3, 3), "value": round(units / dt, 1), "steps": steps}

    def close(self):
        self.build.close()
        self.store.close()
        self.rec_dev.close()


def digest_key(args, world, emu):
    """The tests/golden/digests.json entry this run's union of outputs must hash to, or None."""
    if args.shuffle_contigs or emu > 1:
        return None  # emulated ranks compute rank 0's share only; shuffled ids need the inverse relabelling
    if world > 1 and not args.strong:
        return None  # the weak global problem (W x config) has no oracle digest
    return {"config2": "config2", "config3": "config3", "config5_1gpu": "config5_1gpu"}.get(args.config)


def _gather_compare(comm, inp, gold, M, rows, cols, e):
    """Every rank's share of one step's outputs (profile row digests, edges it
    owns, totals; the column digest when known) gathered to rank 0 and compared
    with the digests.  Returns (mismatches, edge digests) on rank 0, None elsewhere."""
    import digests as D

    meta = np.array([M, inp["c_lo"], inp["n_loc"], len(e.a)], np.int64)
    g_meta = comm.allgather_host(meta)
    g_rows = comm.allgather_host(np.frombuffer(rows, np.uint8))
    g_cols = comm.allgather_host(np.frombuffer(cols.encode(), np.uint8)) if cols is not None else None
    g_a = comm.allgather_host(np.asarray(e.a, np.uint32))
    g_b = comm.allgather_host(np.asarray(e.b, np.uint32))
    g_w = comm.allgather_host(np.asarray(e.weight, np.float64))
    g_s = comm.allgather_host(np.asarray(e.shared, np.int64))
    g_t = comm.allgather_host(np.asarray(e.totals, np.int64))
    if comm.rank != 0:
        return None
    order = np.argsort([int(m[1]) for m in g_meta], kind="stable")
    mism = []
    if any(int(m[0]) != gold["M"] for m in g_meta):
        mism.append("M")
    if g_cols is not None and any(bytes(c).decode() != gold["columns"] for c in g_cols):
        mism.append("columns")
    lo = 0
    for r in order:  # the shards tile [0, N) in rank order
        if int(g_meta[r][1]) != lo:
            mism.append("shards")
        lo += int(g_meta[r][2])
    if lo != gold["N"]:
        mism.append("N")
    if "profile_rows" not in gold:
        mism.append("profile_rows (absent from digests.json)")
    elif D.profile_rows_digest(rows=b"".join(bytes(g_rows[r]) for r in order)) != gold["profile_rows"]:
        mism.append("profile")
    got = D.edge_digests(np.concatenate([g_a[r] for r in order]), np.concatenate([g_b[r] for r in order]),
                         np.concatenate([g_w[r] for r in order]), np.concatenate([g_s[r] for r in order]),
                         g_t[0])
    for k in ("E", "ab", "weight", "shared", "totals"):
        if got.get(k) != gold["edges"].get(k):
            mism.append(f"edges.{k}")
    if any(not np.array_equal(t, g_t[0]) for t in g_t):
        mism.append("totals differ between ranks")
    return mism, got


def parity_check(leg, key):
    """In-run parity (outside the timed region), of two steps:
      timed_step  the LAST TIMED STEP itself, as the timed loop left it: with the
                  native step a deferred one, whose profile (karma_step_profile)
                  and edges (karma_step_newest_edges: the arrays its own tail
                  kernels wrote -- step_edge_count / step_edge_write, and with an
                  exchange step_pack / step_merge over the fixed slots) are the
                  outputs of exactly the code path the headline times;
      kept_step   one more, synchronous step with its outputs kept (the column
                  keys too).
    Every rank hashes its own profile rows, rank 0 gathers the row digests (32 B
    per row), the edges (each owned by the rank of contig a), the column digest
    and the totals, and compares the union with tests/golden/digests.json[key]
    (the oracle's digests; config 3's profile and edges are also the
    reference's own, tests/golden/time_reference.py).  A multi-GPU run is
    thereby its own RCCL parity test.  Returns the JSON object for the bench
    line (rank 0)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import digests as D
    from karma_amd import engine

    comm, inp = leg.comm, leg.inp
    gold = D.load().get(key) if key else None
    if gold is None:
        return {"parity": None, "reason": f"no digests for {key or 'this workload'}"}
    t0 = time.perf_counter()
    timed = None
    native = leg.build.native
    if native is not None:
        info = native.info()  # the timed loop ended with karma_step_sync
        prof = native.profile().numpy()
        rows = D.row_digests(prof)
        del prof
        e, deferred = native.newest_edges()
        g_def = comm.allgather_host(np.array([int(deferred)], np.int64))
        out = _gather_compare(comm, inp, gold, int(info[0]), rows, None, e)
        if out is not None:
            mism, got = out
            timed = {"step": "last timed step", "deferred_on_every_rank": all(int(d[0]) for d in g_def),
                     "outputs": "karma_step_profile + karma_step_newest_edges (the step's own tail buffers)",
                     "checked": ["M", "profile_rows", "edges.ab", "edges.weight", "edges.shared", "edges.totals"],
                     "mismatch": mism, "edges": got["E"]}
    res = leg.step(keep=True)
    leg.sync_all()
    prof = res["profile"].numpy()  # this rank's rows, D2H
    rows = D.row_digests(prof)
    del prof
    cols = D.columns_digest(engine.decode_keys(res["columns"], engine.kmode_of(inp["kmer"])))
    out = _gather_compare(comm, inp, gold, int(res["M"]), rows, cols, res["edges"])
    if comm.rank != 0:
        return None
    mism, got = out
    kept = {"step": "one more synchronous step, outputs kept (KARMA_STEP_KEEP)",
            "checked": ["M", "columns", "profile_rows", "edges.ab", "edges.weight", "edges.shared", "edges.totals"],
            "mismatch": mism, "edges": got["E"]}
    ok = not mism and (timed is None or (not timed["mismatch"] and timed["deferred_on_every_rank"]))
    src = " (oracle; config 3 profile and edges also the reference's own)" if key == "config3" else " (oracle)"
    return {"parity": ok,
            "against": ("the last timed (deferred) step's own outputs and a kept synchronous step, vs "
                        if timed is not None else "a kept synchronous step, vs ") + f"tests/golden/digests.json[{key}]"
                       + src,
            "timed_step": timed, "kept_step": kept,
            "mismatch": (timed["mismatch"] if timed else []) + mism, "edges": got["E"], "ranks": comm.world,
            "seconds": round(time.perf_counter() - t0, 2)}


def profiler_preloaded():
    """True under rocprofv3 (its options reach the program as ROCPROF_*
    variables, its tool library through LD_PRELOAD).  Its preload initialises
    the GPU before this program starts, so self_launch's fork + exec of rank
    processes would then come from a GPU-initialised process."""
    return any(k.startswith("ROCPROF_") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if profiler_preloaded():
            log("bench.py: --gpus N > 1 under a profiler: start the ranks with the launcher (torchrun, or "
                "RANK/WORLD_SIZE per process) and profile each rank, not bench.py's self-launch")
            return 2
        return self_launch(args)  # before anything here touches HIP
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    launcher = os.environ.get("KARMA_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else
                              ("env" if "WORLD_SIZE" in os.environ else "none"))
    WATCHDOG.start(rank)
    from karma_amd import _lib

    try:
        return run(args, rank, world, local_rank, launcher)
    except _lib.KarmaError as e:
        if e.code == _lib.KARMA_ERR_STALL:
            stalled_exit(rank, e)
        if world > 1:  # a failed rank leaves its peers inside collectives: no teardown
            import traceback

            traceback.print_exc()
            log(f"bench.py: rank {rank} failed; exiting without teardown")
            os._exit(1)
        raise


def run(args, rank, world, local_rank, launcher):
    from karma_amd import _lib, comm as comm_mod

    # KARMA_FORCE_DEVICE pins every rank to one device (multi-rank rehearsal on
    # a 1-GPU box together with KARMA_DIST_BACKEND=host); unset in real runs
    dev_index = int(os.environ.get("KARMA_FORCE_DEVICE", local_rank if world > 1 else 0))
    ctx = _lib.Context(dev_index)
    comm = comm_mod.create(ctx, world, rank)
    WATCHDOG.tick("communicator")
    # what joined: the processes (a host-side sum) and, for RCCL, the
    # communicator's own size as RCCL reports it
    transport = {"launcher": launcher, "backend": type(comm).__name__,
                 "ranks_joined": comm.sum_int(1) if world > 1 else 1,
                 "rccl_ranks": comm.info()[0] if hasattr(comm, "info") else None}
    build_info = _lib.build_info()
    if build_info.get("defines") and not os.environ.get("KARMA_ALLOW_VARIANT"):
        raise SystemExit(f"bench.py: libkarma_hip.so was built with non-default defines {build_info['defines']}; "
                         f"rebuild with `make -C karma_amd/csrc` (KARMA_ALLOW_VARIANT=1 to time a variant)")

    leg = Leg(args, ctx, comm, rank, world)
    rec_bytes, flagged = leg.rec_bytes, leg.flagged
    WATCHDOG.tick("inputs resident")
    inp, A = leg.inp, leg.A
    n_loc, f_loc = inp["n_loc"], inp["f_loc"]
    dt, res, kern, dom, dom_live = leg.timed(args.steps, args.warmup, not args.no_timing)
    rec = inp["rec"]
    n_reads = int(np.count_nonzero(rec[1:, 0] != rec[:-1, 0])) + 1 if A else 0

    units = comm.sum_int(n_loc + f_loc) * args.steps
    value = units / dt
    M = res["M"]
    E = comm.sum_int(res["E_local"])
    # algorithmic bytes per launch; intermediates are diagnostic only
    per_kernel_bytes = {
        "kmer_profile": leg.packed_bytes + 8 * n_loc * M,
        "kmer_presence": leg.packed_bytes,
        "graph_classify": leg.rec_bytes * A,  # the records, read once (4 or 8 bytes each by format)
    }
    # intermediate (not in the roofline bytes): the binned classify (<= 56 code
    # buckets) writes one 2-byte code per compact read into bucket runs, which
    # the code reduce reads; otherwise a 4-byte code per read, partitioned into
    # 2-byte runs (graph_sets.hip)
    binned = "graph_code_partition" not in kern
    intermediate_bytes = {
        "graph_classify": (2 if binned else 4) * n_reads,
        "graph_code_partition": 6 * n_reads,
        "graph_code_reduce": 2 * n_reads,
    }
    roof = None
    if dom_live:
        ms, nl = dom_live
        avg_s = ms / nl / 1e3
        b = per_kernel_bytes.get(dom, 0)
        achieved = b / avg_s / 1e9
        traffic = pmc_traffic(args, world, dom)
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic, "bytes_per_launch": b,
                "intermediate_bytes_per_launch": intermediate_bytes.get(dom, 0),
                "avg_launch_ms": round(ms / nl, 4), "launches": nl}
        solo = kern.get(dom)
        if solo and solo[1]:
            # the same kernel alone on the chip (the sequential pass): in the
            # timed stream a deferred batch's classify shares HBM with the
            # previous batch's profile, which lengthens its live launches
            solo_s = solo[0] / solo[1] / 1e3
            roof["solo_launch_ms"] = round(solo[0] / solo[1], 4)
            roof["solo_achieved"] = round(b / solo_s / 1e9, 1)
            roof["solo_frac"] = round(b / solo_s / 1e9 / PEAK_HBM_GBS, 4)
            roof["note"] = ("achieved/frac: live launches of the timed stream (deferred batches overlap: beside the "
                            "other stream's batch with two main streams, beside nothing of the profile with one); "
                            "solo_*: the sequential pass, alone on the chip")
    write_ceiling = profile_write_ceiling(ctx, leg, n_loc, M, kern, args.steps)
    step_bytes = leg.packed_bytes + 8 * n_loc * M + leg.rec_bytes * A + 16 * res["E_local"] + 8 * n_loc
    host_us, api_calls = leg.host_us_per_step, leg.api_calls_per_step
    si = leg.step_info
    step_driver = ({"native": True, "deferred_steps": si[5], "synchronous_steps": si[4], "rerun_steps": si[6],
                    "host_wait_us_per_step": round(leg.host_wait_us_per_step, 1),
                    "drain_us": round(leg.drain_us, 1), "drain_wait_us": round(leg.drain_wait_us, 1),
                    "mode": leg.step_mode,
                    "note": "karma_step (csrc/step.hip): one C ABI call per step; host_us_per_step is the time "
                            "inside those calls (host_wait_us_per_step of it waiting for the device: the status "
                            "of the step kLag = 3 back), api_calls_per_step the HIP/RCCL calls they made; "
                            "drain_us: the sync + barrier after the last step call (inside the timed region), "
                            "drain_wait_us of it waiting for deferred statuses"}
                   if si else {"native": False})
    step_s = dt / args.steps
    WATCHDOG.tick("timed loop done")
    parity = None
    if not args.no_parity:
        parity = parity_check(leg, digest_key(args, world, inp["emu"]))
        WATCHDOG.tick("parity")
    single = leg.single_batch()
    WATCHDOG.tick("single batch")
    other = None
    # (not for a profile of tens of GB: the second build would hold its own buffers beside the first's)
    if not args.no_other_format and 8 * n_loc * M < (32 << 30):
        other = leg.other_format(min(args.steps, 40), min(args.warmup, 5))
        WATCHDOG.tick("other records format")
    extra = {}
    if rank == 0 and world == 1 and not args.no_e2e and inp["emu"] == 1 and not args.shuffle_contigs:
        extra = end_to_end_legs(args, inp, ctx, leg.build, leg.store)
        WATCHDOG.tick("end-to-end legs")
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        cpu = cpu_baseline(inp)
        WATCHDOG.tick("cpu baseline")
    leg.close()
    del leg

    weak = None
    if world > 1 and args.strong and not args.no_weak_leg:
        # weak scaling as an extra key: every rank a whole config-sized share
        import copy

        wargs = copy.copy(args)
        wargs.strong = False
        wl = Leg(wargs, ctx, comm, rank, world)
        wdt, wres, _, _, _ = wl.timed(args.steps, args.warmup, kernel_timing=False)
        wunits = comm.sum_int(wl.inp["n_loc"] + wl.inp["f_loc"]) * args.steps
        weak = {"value": round(wunits / wdt, 1), "unit": "(contigs+fragments)/s",
                "ms_per_step": round(wdt / args.steps * 1e3, 3), "scaling": "weak",
                "workload": f"{args.config} per rank: {wl.inp['n_loc']} contigs + {wl.inp['f_loc']} fragments on "
                            f"each of {world} ranks (global {wl.inp['n_glob']} contigs / {wl.inp['f_glob']} "
                            f"fragments)"}
        wl.close()

    if rank == 0:
        emu = inp["emu"]
        ref = reference_measured(args.config)
        line = {
            "metric": "contigs+reads/sec for k-mer vec + shared-read graph build; HBM GB/s vs roofline",
            "value": round(value, 1),
            "unit": "(contigs+fragments)/s",
            "n_gpus": world,
            "transport": transport,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "single_batch_ms": single["ms"],
            "single_batch": single,
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            # BASELINE.md publishes no number for this metric
            "vs_baseline": None,
            "dtype": "u32 keys / i64 counts / f64 div",
            "data": "synthetic (SplitMix64 generator, SURVEY.md §8(d))"
                    + (", contig ids shuffled" if args.shuffle_contigs else ""),
            "config": {"workload": f"{args.config}{' strong' if args.strong else ' weak'}: {n_loc} contigs "
                                   f"(mean 800 bp) + {f_loc} {'paired' if inp['paired'] else 'single-end'} "
                                   f"fragments on rank 0 (global {inp['n_glob']} contigs / {inp['f_glob']} "
                                   f"fragments), k={inp['kmer']}",
                       "contigs_rank0": n_loc, "fragments_rank0": f_loc, "records_rank0": A,
                       "columns_M": M, "edges": E, "parallelism": f"contig+fragment shards x{world}",
                       **({"emulated_ranks": emu, "global_contigs": inp["n_glob"]} if emu > 1 else {})},
            "parity": parity["parity"] if parity else None,
            "parity_detail": parity,
            "roofline": roof,
            "profile_write_ceiling": write_ceiling,
            "step": {"hbm_bytes_per_gpu": step_bytes, "achieved_GBs": round(step_bytes / step_s / 1e9, 1),
                     "frac": round(step_bytes / step_s / 1e9 / PEAK_HBM_GBS, 4),
                     "formula": f"sum ceil(L/4) + 8*N*M + {rec_bytes}*A + 16*E + 8*N (SURVEY.md 8(d); "
                                f"{rec_bytes} bytes per record in the {args.records} format)"},
            "records_format": {"format": args.records,
                               "layout": ("u32 contig | (first record of its read) << 31 (KARMA_REC_FLAGGED)"
                                          if flagged else "{u32 read id, u32 contig} (KARMA_REC_SORTED)"),
                               "bytes_per_record": rec_bytes,
                               "note": "the same records (config's fragments); the graph depends only on which "
                                       "records share a read, so the read ids may be replaced by read-start flags; "
                                       "records_other times the other format"},
            **({"records_other": other} if other else {}),
            "host_us_per_step": round(host_us, 1),
            "api_calls_per_step": round(api_calls, 1),
            "step_driver": step_driver,
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in kern.items()},
            "kernels_ms_note": "sequential pass (profile on the main stream), every launch timed",
            **({"weak": weak} if weak else {}),
            **extra,
            "cpu_baseline": cpu,
            **({"vs_reference_measured": round(value / ref["units_per_s"], 1),
                "reference_measured": ref} if ref and args.strong and emu == 1 else {}),
            "build": build_info,
        }
        print(json.dumps(line), flush=True)
    comm.close()
    ctx.close()
    return 0


def profile_write_ceiling(ctx, leg, n_loc, M, kern, steps):
    """The profile's write rate against this device's own ceiling for the same
    buffer, measured in this process: hipMemsetAsync of the N x M x 8 bytes
    (karma_memset_timed, HIP events).  The profile is write-bound (its counting
    hides under the row writes), so memset is the bar."""
    import ctypes

    from karma_amd import _lib

    nbytes = 8 * n_loc * M
    if not nbytes or "kmer_profile" not in kern:
        return None
    buf = _lib.DevBuf(ctx, (nbytes,), np.uint8)
    ms = ctypes.c_double(0)
    try:
        _lib.call("karma_memset_timed", ctx.h, ctypes.c_void_p(buf.ptr), nbytes, 10, ctypes.byref(ms))
    finally:
        buf.close()
    prof_ms = kern["kmer_profile"][0] / kern["kmer_profile"][1]
    ceil = nbytes / (ms.value / 1e3) / 1e9
    rate = nbytes / (prof_ms / 1e3) / 1e9
    return {"bytes": nbytes, "memset_ms": round(ms.value, 4), "write_ceiling_GBs": round(ceil, 1),
            "profile_ms": round(prof_ms, 4), "profile_write_GBs": round(rate, 1),
            "profile_vs_ceiling": round(rate / ceil, 3),
            "note": "profile time from the sequential per-kernel pass; memset of the same bytes, same process"}


def reference_measured(config):
    """The reference Python timed on this exact workload in the build container
    (tests/golden/time_reference.py -> tests/golden/reference_<config>.json,
    which ships to the GPU box): read_fasta_file + __calc_kmer_profile +
    from_equivalence_classes."""
    try:
        with open(os.path.join(REPO, "tests", "golden", f"reference_{config}.json")) as f:
            r = json.load(f)
    except (OSError, ValueError):
        return None
    if "units_per_s" not in r:
        return None
    return {"units_per_s": r["units_per_s"], "seconds": r["total_s"],
            "split_s": {k: r[k] for k in ("read_fasta_file_s", "calc_kmer_profile_s", "from_equivalence_classes_s")},
            "threads": r["threads"], "host": "build container (8 vCPU Xeon), not the GPU box",
            "source": f"tests/golden/reference_{config}.json"}


def pmc_traffic(args, world, kernel):
    """HBM bytes per launch of `kernel` from a rocprofv3 PMC run of THIS
    workload (profiles/pmc_traffic.json, written by tools/pmc_traffic.py and
    keyed by workload), else None."""
    ranks = world * max(1, args.emulate_ranks)
    # strong and weak are one workload on one rank (the table's config3_n1)
    key = f"{args.config}{'_strong' if args.strong and ranks > 1 else ''}" \
          f"{'_shuffled' if args.shuffle_contigs else ''}{'_pairs' if args.records == 'pairs' else ''}_n{ranks}"
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(key, {}).get(kernel)
    except (OSError, ValueError):
        return None


def end_to_end_legs(args, inp, ctx, build, store):
    """Host-resident inputs -> host-resident outputs, as the drop-in classes see
    them (kmer.py:264 returns a host ndarray; read_graph.py returns a graph):
      records leg  FASTA text -> karma_fasta_parse -> pack/H2D -> profile -> D2H,
                   and host records -> H2D -> graph -> edges D2H
      eq leg       the path karma.py:240 calls (read_graph.py:61-148): this
                   rank's fragments as salmon eq classes -> karma_graph_eq ->
                   edges D2H."""
    from karma_amd import _lib, engine, ingest

    out = {}
    n, blob, offs = inp["n_loc"], inp["blob"], inp["offs"]
    # FASTA text of the contigs (one sequence line each)
    names = [f">ctg{inp['c_lo'] + i}".encode() for i in range(n)]
    seqb = bytes(blob[: int(offs[-1])])
    parts = []
    for i in range(n):
        parts.append(names[i])
        parts.append(seqb[int(offs[i]):int(offs[i + 1])])
    fasta = b"\n".join(parts) + b"\n"
    rec = inp["rec"]
    kmode = engine.kmode_of(inp["kmer"])
    prof_host = np.empty((n, 1), np.float64)

    def e2e_once():
        nonlocal prof_host
        t0 = time.perf_counter()
        fr = ingest.parse_fasta(fasta)
        st = engine.ContigStore(ctx, fr.seq, fr.seq_off, fr.key_len)
        plan = engine.KmerPlan(ctx, st, kmode)
        M = plan.finalize()
        if prof_host.shape != (n, M):
            prof_host = np.empty((n, M), np.float64)
        _lib.call("karma_kmer_profile", plan.h, _lib.ptr(prof_host), M, 0)
        p = engine.Pairs.from_records(ctx, rec, inp["n_glob"])
        e = p.edges(_lib.KARMA_MODE_READS, inp["n_glob"])
        ea = e.get()
        for x in (e, p, plan, st):
            x.close()
        return time.perf_counter() - t0, len(fasta), len(ea.a)

    e2e_once()  # warm (allocator, pinned staging)
    ts = [e2e_once() for _ in range(3)]
    t = min(x[0] for x in ts)
    out["end_to_end"] = {
        "value": round((n + inp["f_loc"]) / t, 1), "unit": "(contigs+fragments)/s", "ms": round(t * 1e3, 2),
        "includes": "FASTA parse (C++, host) + H2D + pack + profile + D2H of the f64 profile; host records H2D + "
                    "graph + edge D2H",
        "fasta_bytes": ts[0][1], "profile_bytes_d2h": int(prof_host.nbytes)}
    # eq leg (read_graph.py:61-148)
    cls_off, members, counts = engine.synth_eq_classes(inp["seed"], inp["n_glob"], inp["f_lo"],
                                                       inp["f_lo"] + inp["f_loc"], inp["paired"], genes=inp["genes"])
    skip = (np.diff(cls_off) == 1).astype(np.uint8)  # eq_size token "1"
    # the form the drop-in's C++ parser hands over (ingest.parse_eq(compact=True):
    # sizes u8, counts u32, pinned host memory), built before the timed calls
    cq = engine.eq_compact(cls_off, counts, skip)
    if cq is not None:
        c_sz, c_mem, c_cnt = (_lib.pinned_empty(len(x), x.dtype) for x in (cq[0], members, cq[1]))
        c_sz[:], c_mem[:], c_cnt[:] = cq[0], members, cq[1]

    def eq_once():
        t0 = time.perf_counter()
        if cq is not None:
            a, _, _ = engine.graph_from_eq_compact_ordered(c_sz, c_mem, c_cnt, inp["n_glob"], ctx=ctx)
        else:
            a, _, _ = engine.graph_from_eq_ordered(cls_off, members, counts, skip, inp["n_glob"], ctx=ctx)
        return time.perf_counter() - t0, len(a)

    eq_once()
    te = [eq_once() for _ in range(5)]
    ctx.timing(True)  # one more call with every launch timed (outside the best-of-5)
    ctx.timing_reset()
    eq_once()
    eq_k = {k: round(ms, 4) for k, (ms, nl) in sorted(ctx.timing_read().items())}
    ctx.timing(False)
    out["eq_path"] = {"ms": round(min(x[0] for x in te) * 1e3, 3), "classes": int(len(counts)),
                      "members": int(len(members)), "edges": te[0][1],
                      "includes": "host eq arrays as the C++ parser emits them (sizes u8, members u32, counts "
                                  "u32, pinned) -> H2D -> size and pair-count scans, eq_rank, eq_place, "
                                  "seg_reduce, eq_totals (csrc/eq.hip) -> weights -> eq_order (the reference's "
                                  "insertion order, as the drop-in reads it) -> (a, b, w) D2H",
                      "compact": cq is not None,
                      "kernels_ms": eq_k,
                      "value": round((n + inp["f_loc"]) / min(x[0] for x in te), 1)}
    out["dropin"] = dropin_leg(inp)
    return out


def dropin_files(inp, fasta_path, eq_path):
    """The workload as the files karma.py reads (karma.py:190, :236): a FASTA
    with one sequence line per contig (keys ">ctg<i>") and the fragments as a
    salmon eq_classes.txt (read_graph.py:75-82 format: n_txp, n_eq, n_txp
    names, then "size<TAB>ids...<TAB>count" lines).  Also written by
    tests/golden/time_reference.py, which times the reference on the same bytes."""
    from karma_amd import engine

    n, blob, offs, c_lo = inp["n_loc"], inp["blob"], inp["offs"], inp["c_lo"]
    seqb = bytes(blob[: int(offs[-1])])
    with open(fasta_path, "wb") as f:
        f.write(b"".join(b">ctg%d\n%s\n" % (c_lo + i, seqb[int(offs[i]):int(offs[i + 1])]) for i in range(n)))
    cls_off, mem, cnt = engine.synth_eq_classes(inp["seed"], inp["n_glob"], inp["f_lo"], inp["f_lo"] + inp["f_loc"],
                                                inp["paired"], genes=inp["genes"])
    ids = [str(x) for x in range(inp["n_glob"])]
    memb = [ids[x] for x in mem.tolist()]
    offl = cls_off.tolist()
    lines = [f"{inp['n_glob']}\n{len(cnt)}\n"] + [f"ctg{i}\n" for i in range(inp["n_glob"])]
    for c, k in enumerate(cnt.tolist()):
        lo, hi = offl[c], offl[c + 1]
        lines.append(f"{hi - lo}\t" + "\t".join(memb[lo:hi]) + f"\t{k}\n")
    with open(eq_path, "w") as f:
        f.write("".join(lines))
    return len(cnt)


def dropin_leg(inp, reps=2):
    """The drop-in exactly as karma.py calls it, on files (karma.py:190, :197-210,
    :240): karma_amd.fasta.read_fasta_file -> KmerClustering(...).
    _KmerClustering__calc_kmer_profile() (a host float64 ndarray, kmer.py:199-264)
    and ReadGraph.from_equivalence_classes(eq file, sequences) (an nx.Graph,
    read_graph.py:61-148).  Best of `reps` after one warm call."""
    import shutil
    import tempfile

    from karma_amd.fasta import read_fasta_file
    from karma_amd.kmer import KmerClustering
    from karma_amd.read_graph import ReadGraph

    d = tempfile.mkdtemp(prefix="karma_dropin_")
    try:
        fa, eq = os.path.join(d, "contigs.fa"), os.path.join(d, "eq_classes.txt")
        n_cls = dropin_files(inp, fa, eq)
        best = None
        for it in range(reps + 1):
            t0 = time.perf_counter()
            seqs = read_fasta_file(fa)
            t1 = time.perf_counter()
            prof = KmerClustering(seqs, d, inp["kmer"], 16)._KmerClustering__calc_kmer_profile()
            t2 = time.perf_counter()
            g = ReadGraph.from_equivalence_classes(eq, seqs)
            t3 = time.perf_counter()
            cur = (t3 - t0, t1 - t0, t2 - t1, t3 - t2, prof.shape, g.number_of_nodes(), g.number_of_edges())
            del prof, g, seqs
            if it and (best is None or cur[0] < best[0]):
                best = cur
    finally:
        shutil.rmtree(d, ignore_errors=True)
    units = inp["n_loc"] + inp["f_loc"]
    out = {"value": round(units / best[0], 1), "unit": "(contigs+fragments)/s", "seconds": round(best[0], 4),
           "split_s": {"read_fasta_file": round(best[1], 4), "calc_kmer_profile": round(best[2], 4),
                       "from_equivalence_classes": round(best[3], 4)},
           "profile_shape": list(best[4]), "graph_nodes": best[5], "graph_edges": best[6], "eq_classes": n_cls,
           "includes": "files on local disk -> FASTA parse -> profile as a host ndarray (H2D, kernels, D2H of "
                       "8*N*M bytes) -> eq parse -> GPU graph -> nx.Graph in the reference's layout"}
    ref = reference_measured("config3") if (inp["n_loc"], inp["f_loc"]) == (200_000, 100_000_000) else None
    if ref:
        out["reference_seconds"] = ref["seconds"]
        out["speedup_vs_reference"] = round(ref["seconds"] / best[0], 1)
        out["reference_split_s"] = ref["split_s"]
    return out


def cpu_baseline(inp):
    """The oracle's OpenMP twin (oracle/oracle.c, same arithmetic as the scalar
    restatement) on the FULL per-GPU workload: profile of every contig + the
    readset graph of every fragment, on all host cores."""
    try:
        from oracle import oracle
    except Exception as e:  # oracle not built on this box
        return {"error": f"oracle unavailable: {e}"}
    n, f = inp["n_loc"], inp["f_loc"]
    blob, offs = inp["blob"], inp["offs"]
    key_len = inp["key_len"].astype(np.int64)
    t0 = time.perf_counter()
    raw, M = oracle.omp_kmer_columns_packed(blob, offs, inp["kmer"])
    tc = time.perf_counter()
    oracle.omp_kmer_profile_packed(blob, offs, key_len, inp["kmer"], raw, M)
    t1 = time.perf_counter()
    rec = inp["rec"]
    starts = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    off = np.r_[starts, len(rec)].astype(np.int64)
    t2 = time.perf_counter()
    oracle.omp_graph_reads(off, rec[:, 1], inp["n_glob"])
    t3 = time.perf_counter()
    secs = (t1 - t0) + (t3 - t2)
    return {"value": round((n + f) / secs, 1), "unit": "(contigs+fragments)/s", "cores": oracle.threads(),
            "kind": "port",
            "split_s": {"columns": round(tc - t0, 3), "profile": round(t1 - tc, 3), "graph": round(t3 - t2, 3)},
            "sample": f"full per-GPU workload: {n} contigs k={inp['kmer']} column table ({tc - t0:.2f}s) + profile "
                      f"({t1 - tc:.2f}s) + readset graph of {f} fragments / {len(rec)} records ({t3 - t2:.2f}s); "
                      f"oracle/ C restatement, OpenMP on every stage"}


if __name__ == "__main__":
    sys.exit(main())
