"""Multi-GPU (one process per GPU) sharded build — SURVEY.md §8(e).

Sharding: rank r owns a contiguous block of contig rows and a contiguous
range of fragments (read ids).  Two exchange steps exist in the path and only
those use collectives (RCCL over xGMI through torch.distributed "nccl"):

  k-mer profile  the column set is the GLOBAL sorted union of present k-mers
                 (kmer.py:172): the ACGT presence bytes are MAX-allreduced
                 (S <= 64 KiB) and the non-ACGT k-mer keys all-gathered; then
                 every rank derives the identical column table and writes its
                 own rows.
  shared graph   each rank reduces its fragments' pairs locally (HIP bucket
                 reduce), routes the pre-reduced (key, count) list to the owner
                 of contig a (all-to-all-v), the owner merges; its merged
                 diagonal counts are the readset sizes of the contigs it owns,
                 and those slices are all-gathered so every owner can weight
                 edges to contigs it does not own.
All arithmetic is integer until the one weight formula, so the result is
bit-identical to the single-GPU (and the reference) result.

The compute backend is injectable (`ops`): HipOps drives libkarma_hip.so on
the GPU; tests/test_distributed_cpu.py plugs an oracle-backed CPU backend into
the same driver to cover the exchange logic with gloo at world size 2.
"""

from __future__ import annotations

import os

import numpy as np


class Comm:
    """Thin torch.distributed wrapper; world size 1 needs no process group.

    With backend "gloo", device tensors are staged through host memory (used
    to run several GPU ranks on one device in tests; production multi-GPU runs
    use "nccl" = RCCL over xGMI on the device tensors directly)."""

    def __init__(self, world, rank, dist=None, device=None, backend=None):
        self.world, self.rank, self.dist, self.device, self.backend = world, rank, dist, device, backend

    def _h(self, t):
        return t.cpu() if self.backend == "gloo" and t.device.type != "cpu" else t

    def _back(self, h, like):
        if h is like:
            return like
        like.copy_(h)
        return like

    @classmethod
    def create(cls, world, rank, local_rank=0, backend=None):
        if world == 1:
            return cls(1, 0)
        import torch
        import torch.distributed as dist

        if backend is None:
            # KARMA_DIST_BACKEND=gloo: rehearse several GPU ranks on one device
            backend = os.environ.get("KARMA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            device = torch.device(f"cuda:{local_rank}")
        else:
            device = torch.device("cpu")
        if not dist.is_initialized():
            dist.init_process_group(backend, rank=rank, world_size=world)
        return cls(world, rank, dist, device, backend)

    # scalar helpers (host values)
    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def _scalar(self, x, dtype, op):
        import torch

        t = torch.tensor([x], dtype=dtype, device=self.device)
        self.dist.all_reduce(t, op=op)
        return t.item()

    def max_float(self, x):
        return x if not self.dist else self._scalar(float(x), __import__("torch").float64, self.dist.ReduceOp.MAX)

    def sum_int(self, x):
        return x if not self.dist else int(self._scalar(int(x), __import__("torch").int64, self.dist.ReduceOp.SUM))

    # tensor collectives (in place / returning)
    def allreduce_max_(self, t):
        if self.dist:
            h = self._h(t)
            self.dist.all_reduce(h, op=self.dist.ReduceOp.MAX)
            self._back(h, t)
        return t

    def allreduce_sum_(self, t):
        if self.dist:
            h = self._h(t)
            self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM)
            self._back(h, t)
        return t

    def all_gather_var(self, t):
        """Concatenation of every rank's 1-D tensor (sizes may differ)."""
        if not self.dist:
            return t
        import torch

        dev = t.device
        t = self._h(t)
        n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        if mx == 0:
            return t[:0].to(dev)
        pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
        pad[: t.numel()] = t
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(outs, pad)
        return torch.cat([o[:s] for o, s in zip(outs, sizes)]).to(dev)

    def allgather_slices_(self, t, bounds):
        """t[bounds[r]:bounds[r+1]] of rank r into every rank's t (in place):
        each rank contributes only its own slice (bounds are known everywhere,
        so no size exchange; slices padded to the largest)."""
        if not self.dist:
            return t
        import torch

        lo, hi = int(bounds[self.rank]), int(bounds[self.rank + 1])
        sizes = [int(bounds[r + 1] - bounds[r]) for r in range(self.world)]
        mx = max(sizes)
        h = self._h(t)
        mine = torch.zeros(mx, dtype=h.dtype, device=h.device)
        mine[: hi - lo] = h[lo:hi]
        outs = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(outs, mine)
        for r in range(self.world):
            h[int(bounds[r]):int(bounds[r + 1])] = outs[r][: sizes[r]]
        self._back(h, t)
        return t

    def alltoallv(self, t, send_counts):
        """1-D all-to-all-v: send_counts[r] consecutive elements go to rank r.
        Returns (received, recv_counts): recv_counts[r] elements came from rank r."""
        if not self.dist:
            return t, [int(x) for x in send_counts]
        import torch

        dev = t.device
        t = self._h(t)
        sc = torch.tensor(list(send_counts), dtype=torch.int64, device=t.device)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc)
        recv_counts = [int(x) for x in rc.tolist()]
        out = torch.empty(sum(recv_counts), dtype=t.dtype, device=t.device)
        self.dist.all_to_all_single(out, t, output_split_sizes=recv_counts,
                                    input_split_sizes=[int(x) for x in send_counts])
        return out.to(dev), recv_counts

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()
            self.dist = None


class HipOps:
    """Compute backend on libkarma_hip.so; exchange buffers are torch CUDA tensors."""

    def __init__(self, ctx, device_index=None, make_current=True):
        import torch

        from . import engine

        self.torch, self.engine = torch, engine
        self.dev = torch.device(f"cuda:{torch.cuda.current_device() if device_index is None else device_index}")
        # one stream shared by torch (collectives, buffers) and the HIP kernels;
        # a second ops object (concurrent graph build) keeps its own stream and
        # leaves torch's current stream alone
        # the main stream runs the k-mer kernels (short prologue, then the
        # profile): high priority, so its blocks dispatch first when CUs free up
        self.stream = torch.cuda.Stream(device=self.dev, priority=-1 if make_current else 0)
        if make_current:
            torch.cuda.set_stream(self.stream)
        ctx.set_stream(self.stream.cuda_stream)
        self.ctx = ctx
        # the k-mer profile runs here, beside the graph's tail and exchange
        # (ShardedBuild.run); the main stream keeps the higher priority
        self.side = torch.cuda.Stream(device=self.dev, priority=0)

    # -- k-mer --
    def kmer_plan(self, store, kmode):
        return self.engine.KmerPlan(self.ctx, store, kmode)

    def presence_bytes(self, plan):
        t = self.torch
        nw = plan.presence_words()
        words = t.empty(nw, dtype=t.int32, device=self.dev)
        plan.presence_get(words.data_ptr())
        bits = t.arange(32, device=self.dev, dtype=t.int64)
        return ((words.to(t.int64).unsqueeze(1) >> bits) & 1).to(t.uint8).reshape(-1)

    def set_presence_bytes(self, plan, pres):
        t = self.torch
        bits = t.arange(32, device=self.dev, dtype=t.int64)
        w = (pres.reshape(-1, 32).to(t.int64) << bits).sum(1)
        w = w - ((w >> 31) & 1) * (1 << 32)  # to signed 32-bit without overflow
        words = w.to(t.int32).contiguous()
        plan.presence_set(words.data_ptr())
        self._keep = words

    def exceptions(self, plan):
        t = self.torch
        n = plan.exceptions_count()
        keys = t.empty(max(n, 1), dtype=t.int64, device=self.dev)
        plan.exceptions_get(keys.data_ptr() if n else None)
        return keys[:n]

    def set_exceptions(self, plan, keys):
        keys = keys.contiguous()
        plan.exceptions_set(keys.data_ptr() if keys.numel() else None, keys.numel())
        self._keep_exc = keys

    def finalize(self, plan):
        return plan.finalize()

    def finalize_async(self, plan):
        plan.finalize_async()

    def finalize_wait(self, plan):
        return plan.finalize_wait()

    def columns(self, plan):
        return plan.columns()

    def profile(self, plan, out):
        if out.numel():
            plan.profile_device(out.data_ptr(), out.shape[1])

    def profile_side(self, plan, out):
        """The profile on the side stream, after everything enqueued so far."""
        if out.numel():
            plan.profile_side(out.data_ptr(), self.side.cuda_stream, out.shape[1])

    def join(self):
        """The main stream waits for the side stream (before the plan or profile are used)."""
        self.ctx.join(self.side.cuda_stream)

    def profile_buffer(self, n, M):
        return self.torch.empty((n, M), dtype=self.torch.float64, device=self.dev)

    # -- graph --
    def adopt(self, pairs):
        """Continue work on a pair list built by another HipOps on this stream."""
        pairs.rebind(self.ctx)
        return pairs

    def graph_begin(self, records, n_records, n_contigs):
        return self.engine.Pairs.from_records_begin(self.ctx, n_contigs, records, n_records)

    def graph_end(self, job):
        return job.end()

    def graph_local(self, records, n_records, n_contigs):
        return self.engine.Pairs.from_records(self.ctx, None, n_contigs, grouped=True, device_ptr=records,
                                              n_records=n_records)

    def pairs_kc_split(self, pairs, bounds):
        """The list as interleaved (key, count) int64 pairs [n, 2] (the exchange's
        wire format, written on the device) and the owners' start offsets."""
        t = self.torch
        starts = pairs.split(bounds)
        n = pairs.count()
        kc = t.empty((max(n, 1), 2), dtype=t.int64, device=self.dev)
        pairs.get_kc(kc.data_ptr() if n else None)
        return kc[:n], starts

    def merge_kc(self, kc, runs):
        """The owner's list from the senders' slices of interleaved pairs (runs: their lengths, each sorted)."""
        kc = kc.contiguous()
        return self.engine.Pairs.merge_runs_kc(self.ctx, kc.data_ptr() if kc.numel() else None, runs)

    def totals(self, pairs, n_contigs):
        tot = self.torch.zeros(n_contigs, dtype=self.torch.int64, device=self.dev)
        pairs.totals_device(tot.data_ptr(), n_contigs)
        return tot

    def edges(self, pairs, n_contigs, totals=None):
        from ._lib import KARMA_MODE_READS
        return pairs.edges(KARMA_MODE_READS, n_contigs, totals.data_ptr() if totals is not None else None)

    def edge_count(self, edges):
        return edges.E

    def edge_arrays(self, edges):
        return edges.get()

    def pair_count(self, pairs):
        return pairs.count()

    def entries(self, pairs):
        _, counts, _ = pairs.get()
        return int(counts.sum())

    def close(self, *objs):
        for o in objs:
            if o is not None:
                o.close()


class ShardedBuild:
    """k-mer profile + shared-read graph over contig/fragment shards."""

    def __init__(self, ctx, comm: Comm, kmode, n_glob, c_lo, n_loc, ops=None, overlap=None, emulate_ranks=1):
        self.comm, self.kmode, self.n_glob, self.c_lo, self.n_loc = comm, kmode, n_glob, c_lo, n_loc
        # one process standing in for a rank of a W-rank job (bench.py
        # --emulate-ranks W): the exchange's local work runs -- split at the W
        # owners' bounds, merge of W sorted slices, totals -- its collectives do not
        self.emulate = emulate_ranks if comm.world == 1 and emulate_ranks > 1 else 0
        self.ops = ops if ops is not None else HipOps(ctx)
        self._prof = None
        # The local graph build (records -> pair list) shares nothing with the
        # k-mer profile: with overlap it runs from a worker thread on a second
        # context/stream while this thread drives the profile; every collective
        # stays on this thread, in the same order on every rank.
        # Off by default: sharing the chip stretches both kernels, which blurs
        # per-kernel measurement for ~2.5 % of step time.
        if overlap is None:
            overlap = ops is None and os.environ.get("KARMA_OVERLAP", "0") == "1"
        self.gctx = self.gops = self._pool = None
        if overlap:
            from concurrent.futures import ThreadPoolExecutor

            from . import _lib
            self.gctx = _lib.Context(ctx.device)
            self.gops = HipOps(self.gctx, ctx.device, make_current=False)
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="karma-graph")
        bounds = np.zeros(comm.world + 1, np.int64)
        if comm.world > 1:
            import torch
            dev = comm.device
            t = torch.tensor([c_lo, c_lo + n_loc], dtype=torch.int64, device=dev)
            allb = [torch.zeros_like(t) for _ in range(comm.world)]
            comm.dist.all_gather(allb, t)
            allb = [b.tolist() for b in allb]
            for r in range(comm.world):
                assert allb[r][0] == (allb[r - 1][1] if r else 0), "contig shards must be contiguous, in rank order"
                bounds[r + 1] = allb[r][1]
            assert bounds[-1] == n_glob
        else:
            bounds[1] = n_glob
        self.bounds = bounds

    def contexts(self):
        """The karma contexts this build launches on (per-kernel timing)."""
        return [c for c in (self.ops.ctx if hasattr(self.ops, "ctx") else None, self.gctx) if c is not None]

    def run(self, store, records, n_records, keep=False):
        ops = self.ops
        # Default order (one stream pair): k-mer columns, then the graph's
        # kernels alone on the chip (classify .. final), then the profile on
        # the side stream beside the graph's host-synchronised assembly,
        # exchange and weights on the main stream.  The side stream is joined
        # before anything uses the plan or the profile.
        side = self._pool is None and hasattr(ops, "graph_begin")
        if side:
            # one GPU: nothing but short kernels share the chip with the profile,
            # which then takes all of it (1.35 vs 1.36-1.39 ms/step); with an
            # exchange, a block slot per CU stays free for its collectives
            ops.ctx.set_side_headroom(1 if self.comm.world > 1 or self.emulate else 0)
        try:
            return self._run(store, records, n_records, keep, side)
        finally:
            if side:
                ops.join()

    def _run(self, store, records, n_records, keep, side):
        ops, comm = self.ops, self.comm
        fut = None
        if self._pool is not None:  # ---- shared-read graph, concurrent (read_graph.py:19-50) ----
            fut = self._pool.submit(self.gops.graph_local, records, n_records, self.n_glob)
        local = None
        try:
            # ---- k-mer profile (kmer.py:199-233) ----
            plan = ops.kmer_plan(store, self.kmode)
            if comm.world > 1:
                pres = comm.allreduce_max_(ops.presence_bytes(plan))
                ops.set_presence_bytes(plan, pres)
                ops.set_exceptions(plan, comm.all_gather_var(ops.exceptions(plan)))
            if side:
                # the column table, then the graph's kernels behind it on the
                # main stream; M is read back without waiting for the graph,
                # and the profile (side stream) starts after the graph's kernels
                ops.finalize_async(plan)
                job = ops.graph_begin(records, n_records, self.n_glob)  # ---- read_graph.py:19-50 ----
                try:
                    M = ops.finalize_wait(plan)
                    if self._prof is None or tuple(self._prof.shape) != (self.n_loc, M):
                        self._prof = ops.profile_buffer(self.n_loc, M)
                    ops.profile_side(plan, self._prof)
                finally:
                    local = ops.graph_end(job)
            else:
                M = ops.finalize(plan)
                if self._prof is None or tuple(self._prof.shape) != (self.n_loc, M):
                    self._prof = ops.profile_buffer(self.n_loc, M)
                ops.profile(plan, self._prof)
        finally:
            if fut is not None:
                local = fut.result()  # joined on every path
        if fut is not None:
            local = ops.adopt(local)
        elif local is None:  # ---- shared-read graph (read_graph.py:19-50) ----
            local = ops.graph_local(records, n_records, self.n_glob)
        stats = {"M": M}
        if keep:
            stats["entries"] = ops.entries(local)
            stats["pairs_local"] = ops.pair_count(local)
        if comm.world > 1 or self.emulate:
            if comm.world > 1:
                # one all-to-all-v of interleaved (key, count) int64 pairs; the
                # owner receives one sorted slice per sender and merges them
                kc, starts = ops.pairs_kc_split(local, self.bounds)
                recv_kc, recv = comm.alltoallv(kc.reshape(-1), 2 * np.diff(starts))
                merged = ops.merge_kc(recv_kc, [r // 2 for r in recv])
            else:  # emulation: this rank's own W slices stand in for the W received ones
                kc, starts = ops.pairs_kc_split(local, np.linspace(0, self.n_glob, self.emulate + 1).astype(np.int64))
                merged = ops.merge_kc(kc.reshape(-1), np.diff(starts).tolist())
            # the owner's merged list holds the diagonal (a, a) of every a it owns:
            # complete readset sizes for its slice, gathered to every rank
            tot = comm.allgather_slices_(ops.totals(merged, self.n_glob), self.bounds)
            edges = ops.edges(merged, self.n_glob, tot)
            ops.close(local)
            final_pairs = merged
        else:
            edges = ops.edges(local, self.n_glob)
            final_pairs = local
        stats["E_local"] = ops.edge_count(edges)
        if keep:
            stats["profile"] = self._prof
            stats["edges"] = ops.edge_arrays(edges)
            stats["columns"] = ops.columns(plan)
        ops.close(edges, final_pairs, plan)
        return stats

    def close(self):
        self._prof = None
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        if self.gctx is not None:
            self.gops = None
            self.gctx.close()
            self.gctx = None
