"""Multi-GPU (one process per GPU) sharded build — SURVEY.md §8(e).

Sharding: rank r owns a contiguous block of contig rows and a contiguous
range of fragments (read ids).  Two exchange steps exist in the path and only
those use collectives (the library's own RCCL communicator over xGMI,
karma_amd/comm.py; no PyTorch anywhere on this path):

  k-mer profile  the column set is the GLOBAL sorted union of present k-mers
                 (kmer.py:172): the ACGT presence bitmaps are all-gathered and
                 OR-merged on the device (<= 8 KiB per rank) and the non-ACGT
                 k-mer keys all-gathered; then
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
the same driver to cover the exchange logic with the host-staged transport
(karma_amd/comm.py HostComm) at world sizes 2 to 8.
"""

from __future__ import annotations

import os

import numpy as np

import ctypes

from . import _lib
from ._lib import DevBuf, Stream, call, ptr
from .comm import RcclComm, SoloComm


class HipOps:
    """Compute backend on libkarma_hip.so; every buffer is library device memory (DevBuf)."""

    def __init__(self, ctx, make_current=True):
        from . import engine

        self.engine, self.ctx = engine, ctx
        # the main stream runs the k-mer kernels (short prologue, then the
        # graph and the exchange): high priority, so its blocks dispatch first
        # when CUs free up; a second ops object (concurrent graph build) keeps
        # normal priority.  The k-mer profile runs on the side stream, beside
        # the graph's tail and exchange (ShardedBuild.run).
        self.stream = Stream(ctx, -1 if make_current else 0)
        ctx.set_stream(self.stream)
        self.side = Stream(ctx, 0)

    # -- k-mer --
    def kmer_plan(self, store, kmode):
        return self.engine.KmerPlan(self.ctx, store, kmode)

    def kmer_plan_side(self, store, kmode, comm=None):
        """The presence pass and the column table enqueued on the side stream,
        so that the graph's kernels on the main stream start at once, beside
        them; finalize_wait() waits for the column table alone.  With a
        communicator of several ranks the column set's exchange runs there too
        (presence all-gather and OR-merge, exception keys all-gather; their
        host synchronisations wait for the side stream only), issued in the
        same order on every rank."""
        self.ctx.set_stream(self.side)
        try:
            plan = self.engine.KmerPlan(self.ctx, store, kmode)
            if comm is not None and comm.world > 1:
                # the side stream's own communicator (RcclComm.side) when there
                # is one.  RcclComm defaults to one communicator (comm.side is
                # comm): the side stream then waits for everything enqueued on
                # the main stream first (a previous step's totals all-gather may
                # still be in flight there), so the communicator's operations
                # never run on two streams at once
                sc = getattr(comm, "side", comm)
                if sc is comm:
                    self.ctx.join(self.stream)
                self.presence_merge(plan, sc.allgather_fixed(self.presence_words(plan)), comm.world)
                self.set_exceptions(plan, sc.allgather_var(self.exceptions(plan)))
            plan.finalize_async()
        finally:
            self.ctx.set_stream(self.stream)
        return plan

    def presence_words(self, plan):
        words = DevBuf(self.ctx, (plan.presence_words(),), np.uint32)
        plan.presence_get(words.ptr)
        return words

    def presence_merge(self, plan, all_words, n_sets):
        plan.presence_merge(all_words.ptr, n_sets)
        self._keep = all_words  # read by the merge kernel, stream-ordered

    def exceptions(self, plan):
        n = plan.exceptions_count()
        keys = DevBuf(self.ctx, (n,), np.uint64)
        plan.exceptions_get(keys.ptr if n else None)
        return keys

    def set_exceptions(self, plan, keys):
        plan.exceptions_set(keys.ptr if keys.size else None, keys.size)
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
        if out.size:
            plan.profile_device(out.ptr, out.shape[1])

    def profile_side(self, plan, out):
        """The profile on the side stream, after everything enqueued so far."""
        if out.size:
            plan.profile_side(out.ptr, self.side.ptr, out.shape[1])

    def join(self):
        """The main stream waits for the side stream (before the plan or profile are used)."""
        self.ctx.join(self.side)

    def profile_buffer(self, n, M):
        return DevBuf(self.ctx, (n, M), np.float64)

    # -- graph --
    def adopt(self, pairs):
        """Continue work on a pair list built by another HipOps on this stream."""
        pairs.rebind(self.ctx)
        return pairs

    def graph_begin(self, records, n_records, n_contigs, split_bounds=None, flagged=False):
        return self.engine.Pairs.from_records_begin(self.ctx, n_contigs, records, n_records,
                                                    split_bounds=split_bounds, flagged=flagged)

    def graph_end(self, job):
        return job.end()

    def graph_local(self, records, n_records, n_contigs, flagged=False):
        return self.engine.Pairs.from_records(self.ctx, None, n_contigs, grouped=True, device_ptr=records,
                                              n_records=n_records, flagged=flagged)

    def pairs_kc_split(self, pairs, bounds):
        """The list as interleaved (key, count) int64 pairs (2n, the exchange's
        wire format, written on the device) and the owners' start offsets: one
        launch (karma_pairs_split_kc)."""
        n = pairs.count()
        kc = DevBuf(self.ctx, (2 * n,), np.int64)
        starts = pairs.split_kc(bounds, kc.ptr if n else None)
        return kc, starts

    def pairs_kv(self, pairs, bounds):
        """The owners' start offsets (karma_pairs_split: device searches) and the
        list's own key and count arrays as device buffers (no copy): the
        exchange sends each owner's slice of both (RcclComm.alltoallv_kv)."""
        starts = pairs.split(bounds)
        k, c = pairs.device_ptrs()
        n = pairs.count()
        return (DevBuf(self.ctx, (n,), np.uint64, _ptr=k, _owner=pairs),
                DevBuf(self.ctx, (n,), np.int64, _ptr=c, _owner=pairs), starts)

    def merge_kv(self, keys, counts, runs):
        """The owner's list from received runs of keys and counts (each sorted):
        one ranking pass, no host synchronisation (karma_pairs_merge_runs)."""
        return self.engine.Pairs.merge(self.ctx, keys.ptr if keys.size else None,
                                       counts.ptr if counts.size else None, device=True, n=keys.size, runs=runs)

    def merge_kc(self, kc, runs):
        """The owner's list from the senders' slices of interleaved pairs (runs: their lengths, each sorted)."""
        return self.engine.Pairs.merge_runs_kc(self.ctx, kc.ptr if kc.size else None, runs)

    def totals(self, pairs, n_contigs):
        tot = DevBuf(self.ctx, (n_contigs,), np.int64)
        pairs.totals_device(tot.ptr, n_contigs)  # zeroes, then the diagonal
        return tot

    def edges(self, pairs, n_contigs, totals=None):
        return pairs.edges(_lib.KARMA_MODE_READS, n_contigs, totals.ptr if totals is not None else None)

    def edges_begin(self, pairs, n_contigs):
        """The edge stage's first half (karma_edges_begin): the list's diagonal
        counts land in the returned totals buffer (a view owned by the edges),
        which the caller all-gathers before edges_end."""
        e, tp = pairs.edges_begin(_lib.KARMA_MODE_READS, n_contigs)
        return e, DevBuf(self.ctx, (n_contigs,), np.int64, _ptr=tp, _owner=e)

    def edges_end(self, e, count=True):
        """count=False: the weights launched, the edge count read when first
        used (no synchronisation in the step)."""
        return e.end(count)

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

    def shutdown(self):
        """Release the streams (after the last step)."""
        self.ctx.set_stream(None)
        self.side.close()
        self.stream.close()


class NativeStep:
    """One step as one C ABI call (karma_step, csrc/step.hip): the sequence
    ShardedBuild._run drives from Python, natively, with the library's RCCL
    communicators (main and side) or none.  A step whose outputs are not read
    (count=False) in one process returns without waiting for anything."""

    def __init__(self, ctx, comm, kmode, n_glob, bounds, rank, n_loc):
        self.ctx, self.n_glob = ctx, n_glob
        b = np.ascontiguousarray(bounds, np.int64)
        assert int(b[rank + 1] - b[rank]) == n_loc, "the owner bounds disagree with this rank's contig shard"
        multi = comm.world > 1
        # a distinct side communicator only (one that is the main one is none:
        # its operations would go on two streams at once)
        side = comm.side.h if multi and comm.side is not comm else None
        h = ctypes.c_void_p()
        call("karma_step_create", ctx.h, comm.h if multi else None, side, int(kmode),
             int(n_glob), ptr(b), len(b) - 1, int(rank), ctypes.byref(h))
        self.h = h
        self._info = np.zeros(4, np.int64)

    def run(self, store, records, n_records, keep=False, sequential=False, count=True, flagged=False):
        flags = (_lib.KARMA_STEP_KEEP if keep else 0) | (_lib.KARMA_STEP_SEQUENTIAL if sequential else 0) | \
            (_lib.KARMA_STEP_DEFER if not count and not keep else 0) | (_lib.KARMA_STEP_FLAGGED if flagged else 0)
        info = self._info
        call("karma_step_run", self.h, store.h, ctypes.c_void_p(records), int(n_records), flags, ptr(info))
        M, E = int(info[0]), int(info[1])
        stats = {"M": M if M >= 0 else None, "E_local": E if E >= 0 else None}
        if keep:
            from .engine import EdgeArrays

            stats["pairs_local"], stats["entries"] = int(info[2]), int(info[3])
            dev, rows = ctypes.c_void_p(), ctypes.c_int64()
            call("karma_step_profile", self.h, ctypes.byref(dev), ctypes.byref(rows), None)
            stats["profile"] = DevBuf(self.ctx, (rows.value, M), np.float64, _ptr=dev.value or 0, _owner=self)
            keys = np.zeros(max(M, 1), np.uint64)
            call("karma_step_columns", self.h, ptr(keys))
            stats["columns"] = keys[:M]
            eh = ctypes.c_void_p()
            call("karma_step_edges", self.h, ctypes.byref(eh))
            a, b = np.zeros(max(E, 1), np.uint32), np.zeros(max(E, 1), np.uint32)
            s, w = np.zeros(max(E, 1), np.int64), np.zeros(max(E, 1), np.float64)
            call("karma_edges_get", eh, ptr(a), ptr(b), ptr(s), ptr(w), None, 0)
            tot = np.zeros(max(self.n_glob, 1), np.int64)
            call("karma_edges_totals", eh, ptr(tot), 0)
            stats["edges"] = EdgeArrays(a[:E], b[:E], s[:E], w[:E], np.zeros(E, np.uint64), tot[:self.n_glob])
        return stats

    def sync(self):
        call("karma_step_sync", self.h)

    def profile(self):
        """The newest step's profile (device, rows x M) after sync(): deferred steps included."""
        dev, rows, M = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        call("karma_step_profile", self.h, ctypes.byref(dev), ctypes.byref(rows), ctypes.byref(M))
        return DevBuf(self.ctx, (rows.value, M.value), np.float64, _ptr=dev.value or 0, _owner=self)

    def newest_edges(self):
        """The newest step's edges after sync() (karma_step_newest_edges): a
        deferred step's from the arrays its own tail kernels wrote.  Returns
        (EdgeArrays, deferred)."""
        from .engine import EdgeArrays

        E, dfr = ctypes.c_int64(), ctypes.c_int()
        call("karma_step_newest_edges", self.h, None, None, None, None, None, 0, 0, ctypes.byref(E), None)
        n = E.value
        a, b = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint32)
        s, w = np.zeros(max(n, 1), np.int64), np.zeros(max(n, 1), np.float64)
        tot = np.zeros(max(self.n_glob, 1), np.int64)
        call("karma_step_newest_edges", self.h, ptr(a), ptr(b), ptr(s), ptr(w), ptr(tot), n, 0, ctypes.byref(E),
             ctypes.byref(dfr))
        return EdgeArrays(a[:n], b[:n], s[:n], w[:n], np.zeros(n, np.uint64), tot[:self.n_glob]), bool(dfr.value)

    def info(self):
        """[M, E, pairs, entries, synchronous steps, deferred steps, re-run steps, pending,
        host ns inside karma_step_run, of which ns waiting for deferred statuses, deferred steps on
        two main streams, deferred tails on the exchange stream, mode bits, ranks]."""
        v = np.zeros(15, np.int64)
        call("karma_step_info", self.h, ptr(v), 15)
        return v

    def mode(self):
        """How the steps ran (the bench line's step_driver.mode)."""
        v = self.info()
        bits, ranks = int(v[12]), int(v[13])
        return {"ranks": ranks, "one_communicator": bool(bits & 1), "exchange_stream": bool(bits & 2),
                "defer_across_ranks": bool(bits & 4), "deferred_two_main_streams": int(v[10]),
                "deferred_tail_on_exchange_stream": int(v[11]), "synchronous": int(v[4]), "deferred": int(v[5]),
                "rerun": int(v[6]), "deferred_on_own_control_block": int(v[14])}

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_step_destroy(self.h)
            self.h = None


def native_step_on(comm, ops, overlap):
    """The native step runs the production path (the library's own kernels and
    RCCL communicators); the Python driver stays for an injected compute backend
    (tests/test_distributed_cpu.py), the host-staged rehearsal transport
    (HostComm) and the opt-in concurrent graph build."""
    if ops is not None or overlap or os.environ.get("KARMA_NATIVE_STEP", "1") == "0":
        return False
    return isinstance(comm, (SoloComm, RcclComm))


class ShardedBuild:
    """k-mer profile + shared-read graph over contig/fragment shards."""

    def __init__(self, ctx, comm, kmode, n_glob, c_lo, n_loc, ops=None, overlap=None, emulate_ranks=1, flagged=False):
        self.comm, self.kmode, self.n_glob, self.c_lo, self.n_loc = comm, kmode, n_glob, c_lo, n_loc
        # the records this build's steps take: (read, contig) pairs, or
        # KARMA_REC_FLAGGED words (engine.flag_records: 4 bytes per record)
        self.flagged = bool(flagged)
        # one process standing in for a rank of a W-rank job (bench.py
        # --emulate-ranks W): the exchange's local work runs -- split at the W
        # owners' bounds, merge of W sorted slices, totals -- its collectives do not
        self.emulate = emulate_ranks if comm.world == 1 and emulate_ranks > 1 else 0
        if overlap is None:
            overlap = ops is None and os.environ.get("KARMA_OVERLAP", "0") == "1"
        self.native = None
        native = native_step_on(comm, ops, overlap)
        self.ops = ops if ops is not None else (None if native else HipOps(ctx))
        self._prof = None
        # The local graph build (records -> pair list) shares nothing with the
        # k-mer profile: with overlap it runs from a worker thread on a second
        # context/stream while this thread drives the profile; every collective
        # stays on this thread, in the same order on every rank.
        # Off by default: sharing the chip stretches both kernels, which blurs
        # per-kernel measurement for ~2.5 % of step time.
        self.gctx = self.gops = self._pool = None
        if overlap:
            from concurrent.futures import ThreadPoolExecutor

            from . import _lib
            self.gctx = _lib.Context(ctx.device)
            self.gops = HipOps(self.gctx, make_current=False)
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="karma-graph")
        bounds = np.zeros(comm.world + 1, np.int64)
        self.split_bounds = None  # the exchange's owner bounds (None: no exchange)
        if comm.world > 1:
            allb = [b.tolist() for b in comm.allgather_host(np.array([c_lo, c_lo + n_loc], np.int64))]
            for r in range(comm.world):
                assert allb[r][0] == (allb[r - 1][1] if r else 0), "contig shards must be contiguous, in rank order"
                bounds[r + 1] = allb[r][1]
            assert bounds[-1] == n_glob
        else:
            bounds[1] = n_glob
        self.bounds = bounds
        if comm.world > 1:
            self.split_bounds = bounds
        elif self.emulate:
            # the W owners' contig ranges, rank 0's first (bench.py shard())
            self.split_bounds = np.array([n_glob * r // self.emulate for r in range(self.emulate + 1)], np.int64)
        if native:
            own = self.split_bounds if self.split_bounds is not None else np.array([c_lo, c_lo + n_loc], np.int64)
            self.native = NativeStep(ctx, comm, kmode, n_glob, own, comm.rank if comm.world > 1 else 0, n_loc)
        self._ctx = ctx

    def contexts(self):
        """The karma contexts this build launches on (per-kernel timing)."""
        if self.native is not None:
            return [self._ctx]
        return [c for c in (self.ops.ctx if hasattr(self.ops, "ctx") else None, self.gctx) if c is not None]

    def sync(self):
        """Wait for every step enqueued so far (and check deferred ones)."""
        if self.native is not None:
            self.native.sync()
        for c in self.contexts():
            c.sync()

    def run(self, store, records, n_records, keep=False, sequential=False, count=True):
        """One step.  sequential=True keeps the profile on the main stream (no
        side stream): slower, but every kernel has the chip to itself, which is
        what a per-kernel timing pass wants.  count=False (a step of a stream
        of identical steps; with an exchange only): the owner's edge count is
        not read back, so the step ends without waiting for its last kernels,
        and stats["E_local"] is None."""
        if self.native is not None:
            return self.native.run(store, records, n_records, keep=keep, sequential=sequential, count=count,
                                   flagged=self.flagged)
        ops = self.ops
        # Default order (one stream pair): k-mer columns, then the graph's
        # kernels alone on the chip (classify .. final), then the profile on
        # the side stream beside the graph's host-synchronised assembly,
        # exchange and weights on the main stream.  The side stream is joined
        # before anything uses the plan or the profile.
        side = self._pool is None and hasattr(ops, "graph_begin") and not sequential
        if side:
            # the profile's one-round grid takes the whole chip (3 blocks per
            # CU at 6 waves per SIMD); the exchange's kernels and collectives
            # queue behind its blocks.  Leaving a block slot free for them
            # (round 2's default with an exchange) halves the profile's blocks
            # now: 8-rank strong preview 0.244 (none free) vs 0.256 ms, weak
            # 1.35-1.37 vs 1.40-1.42 ms (profiles/r03/measurements.md (ab_headroom))
            hr = os.environ.get("KARMA_SIDE_HEADROOM")  # measurement override (blocks per CU)
            ops.ctx.set_side_headroom(int(hr) if hr else 0)
        try:
            return self._run(store, records, n_records, keep, side, count or keep)
        finally:
            if side:
                ops.join()

    def _graph_begin(self, records, n_records):
        """The records job, told the exchange's owner bounds when there is one."""
        kw = {"flagged": True} if self.flagged else {}
        if self.split_bounds is not None:
            return self.ops.graph_begin(records, n_records, self.n_glob, split_bounds=self.split_bounds, **kw)
        return self.ops.graph_begin(records, n_records, self.n_glob, **kw)

    def _run(self, store, records, n_records, keep, side, count=True):
        ops, comm = self.ops, self.comm
        fut = None
        if self._pool is not None:  # ---- shared-read graph, concurrent (read_graph.py:19-50) ----
            fut = self._pool.submit(self.gops.graph_local, records, n_records, self.n_glob,
                                    **({"flagged": True} if self.flagged else {}))
        local = None
        try:
            # ---- k-mer profile (kmer.py:199-233) ----
            # with a side stream: the graph's kernels are enqueued first, then
            # the presence pass, the column set's exchange (several ranks) and
            # the column table on the side stream, beside them
            early = side and hasattr(ops, "kmer_plan_side")
            job = None
            if early:
                job = self._graph_begin(records, n_records)  # ---- read_graph.py:19-50 ----
                try:
                    plan = ops.kmer_plan_side(store, self.kmode, comm)
                except BaseException:
                    ops.graph_end(job)
                    raise
            else:
                plan = ops.kmer_plan(store, self.kmode)
            if comm.world > 1 and not early:
                # column set = global union: OR of every rank's presence bitmap,
                # union of every rank's exception keys (kmer.py:146-179)
                ops.presence_merge(plan, comm.allgather_fixed(ops.presence_words(plan)), comm.world)
                ops.set_exceptions(plan, comm.allgather_var(ops.exceptions(plan)))
            if side:
                # the column table, then the graph's kernels behind it on the
                # main stream; M is read back without waiting for the graph,
                # and the profile (side stream) starts after the graph's kernels
                if not early:
                    ops.finalize_async(plan)
                    job = self._graph_begin(records, n_records)  # ---- read_graph.py:19-50 ----
                try:
                    M = ops.finalize_wait(plan)
                    if self._prof is None or tuple(self._prof.shape) != (self.n_loc, M):
                        self._prof = ops.profile_buffer(self.n_loc, M)
                    # queued behind the graph's kernels while the host waits, so
                    # it starts the moment they end (taking the graph's list
                    # first, with an exchange to follow, measured slower: strong
                    # 8-rank preview 0.396 against 0.315 ms)
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
            local = ops.graph_local(records, n_records, self.n_glob, **({"flagged": True} if self.flagged else {}))
        stats = {"M": M}
        if keep:
            stats["entries"] = ops.entries(local)
            stats["pairs_local"] = ops.pair_count(local)
        if comm.world > 1 or self.emulate:
            bounds = self.split_bounds
            if hasattr(ops, "pairs_kv"):
                # the list's keys and counts, each owner's slice of both in one
                # grouped all-to-all-v; the owner merges one sorted run per sender
                keys, counts, starts = ops.pairs_kv(local, bounds)
                if comm.world > 1:
                    rk, rc, recv = comm.alltoallv_kv(keys, counts, np.diff(starts))
                    merged = ops.merge_kv(rk, rc, recv)
                else:  # emulation: this rank's own W slices stand in for the W received ones
                    st = starts.tolist()
                    merged = ops.merge_kv(keys, counts, [b - a for a, b in zip(st, st[1:])])
            elif comm.world > 1:
                # one all-to-all-v of interleaved (key, count) int64 pairs; the
                # owner receives one sorted slice per sender and merges them
                kc, starts = ops.pairs_kc_split(local, self.bounds)
                recv_kc, recv = comm.alltoallv(kc, 2 * np.diff(starts))
                merged = ops.merge_kc(recv_kc, [r // 2 for r in recv])
            else:  # emulation: this rank's own W slices stand in for the W received ones
                kc, starts = ops.pairs_kc_split(local, bounds)
                merged = ops.merge_kc(kc, np.diff(starts).tolist())
            # the owner's merged list holds the diagonal (a, a) of every a it owns:
            # complete readset sizes for its slice, gathered to every rank
            if hasattr(ops, "edges_begin"):
                # two halves around the all-gather: the edge count kernel writes
                # the diagonal into the edges' own totals, gathered in place
                eh, tot = ops.edges_begin(merged, self.n_glob)
                comm.allgather_slices_(tot, self.bounds)
                edges = ops.edges_end(eh) if count else ops.edges_end(eh, count=False)
            else:
                tot = comm.allgather_slices_(ops.totals(merged, self.n_glob), self.bounds)
                edges = ops.edges(merged, self.n_glob, tot)
            ops.close(local)
            final_pairs = merged
        else:
            edges = ops.edges(local, self.n_glob)
            final_pairs = local
        stats["E_local"] = ops.edge_count(edges) if count else None
        if keep:
            stats["profile"] = self._prof
            stats["edges"] = ops.edge_arrays(edges)
            stats["columns"] = ops.columns(plan)
        ops.close(edges, final_pairs, plan)
        return stats

    def close(self):
        self._prof = None
        if self.native is not None:
            self.native.close()
            self.native = None
        if hasattr(self.ops, "shutdown"):
            self.ops.shutdown()
        if self.gops is not None:
            self.gops.shutdown()
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        if self.gctx is not None:
            self.gops = None
            self.gctx.close()
            self.gctx = None
