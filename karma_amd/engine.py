"""Host-side driver of the HIP hot path (thin layer over karma_amd._lib).

Everything here moves host arrays to/from libkarma_hip.so; all compute is in
the HIP kernels (karma_amd/csrc/*.hip).  The drop-in classes (kmer.py,
read_graph.py, contig.py) call these functions.
"""

from __future__ import annotations

import ctypes
import itertools
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import call, ptr

KMODE_5P6 = _lib.KARMA_KMER_5P6


def kmode_of(kmer_size) -> int:
    """kmer.py:69 tests `kmer_size == "5p6"`; anything else is an int k
    (cmd_parser.py:234-235 casts with int())."""
    if kmer_size == "5p6":
        return KMODE_5P6
    return int(kmer_size)


def encode_sequences(sequences):
    """OrderedDict[str, str] -> (bytes blob, offsets int64[N+1], key_len int32[N]).

    Sequences are compared/sliced as Python str; for code points < 256 latin-1
    bytes preserve both length and ordering, so the byte kernels are exact.
    """
    vals = []
    for v in sequences.values():
        try:
            vals.append(v.encode("latin-1"))
        except UnicodeEncodeError as e:
            raise ValueError("sequence contains a code point >= 256; libkarma_hip handles byte sequences "
                             "(latin-1) only") from e
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    if vals:
        np.cumsum([len(v) for v in vals], out=offs[1:])
    blob = np.frombuffer(b"".join(vals) + b"\0" * 16, dtype=np.uint8)
    key_len = np.array([len(k) for k in sequences.keys()], dtype=np.int32)
    return blob, offs, key_len


def decode_keys(keys: np.ndarray, kmode: int):
    """u64 column keys (karma.h encoding) -> list[str] (latin-1)."""
    out = []
    for k in keys.tolist():
        if kmode == 8:
            ln = 8
        else:
            ln = k & 0xFF
        b = k.to_bytes(8, "big")[:ln]
        out.append(b.decode("latin-1"))
    return out


class ContigStore:
    """Device-resident contigs (karma_contigs): 2-bit packed + exception mask."""

    def __init__(self, ctx, blob, offsets, key_len, device_pointers=False, n=None):
        self.ctx = ctx
        h = ctypes.c_void_p()
        if device_pointers:
            call("karma_contigs_create", ctx.h, ctypes.c_void_p(blob), ctypes.c_void_p(offsets),
                 ctypes.c_void_p(key_len), n, 1, ctypes.byref(h))
        else:
            self._keep = (blob, offsets, key_len)
            n = len(key_len)
            call("karma_contigs_create", ctx.h, ptr(blob), ptr(offsets), ptr(key_len) if n else ptr(
                np.zeros(1, np.int32)), n, 0, ctypes.byref(h))
        self.h = h
        self.n = n

    def info(self):
        v = [ctypes.c_int64() for _ in range(4)]
        call("karma_contigs_info", self.h, *[ctypes.byref(x) for x in v])
        return dict(n=v[0].value, total_bases=v[1].value, exception_bases=v[2].value, packed_bytes=v[3].value)

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_contigs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class KmerPlan:
    """Presence pass + column table + dense profile (karma_kmer_plan)."""

    def __init__(self, ctx, store: ContigStore, kmode: int):
        self.ctx, self.store, self.kmode = ctx, store, kmode
        h = ctypes.c_void_p()
        call("karma_kmer_plan_create", ctx.h, store.h, kmode, ctypes.byref(h))
        self.h = h
        self.M = None

    # -- exchange points (multi-rank) --
    def presence_words(self):
        n = ctypes.c_int64()
        call("karma_kmer_presence_words", self.h, ctypes.byref(n))
        return n.value

    def presence_get(self, dst_dev_ptr):
        call("karma_kmer_presence_get", self.h, ctypes.c_void_p(dst_dev_ptr))

    def presence_set(self, src_dev_ptr):
        call("karma_kmer_presence_set", self.h, ctypes.c_void_p(src_dev_ptr))

    def presence_merge(self, all_dev_ptr, n_sets):
        """Presence = OR of n_sets bitmaps back to back in device memory."""
        call("karma_kmer_presence_merge", self.h, ctypes.c_void_p(all_dev_ptr), int(n_sets))

    def exceptions_count(self):
        n = ctypes.c_int64()
        call("karma_kmer_exceptions_count", self.h, ctypes.byref(n))
        return n.value

    def exceptions_get(self, dst_dev_ptr):
        call("karma_kmer_exceptions_get", self.h, ctypes.c_void_p(dst_dev_ptr) if dst_dev_ptr else None)

    def exceptions_set(self, src_dev_ptr, n):
        call("karma_kmer_exceptions_set", self.h, ctypes.c_void_p(src_dev_ptr) if src_dev_ptr else None, n)

    def finalize(self):
        m = ctypes.c_int64()
        call("karma_kmer_plan_finalize", self.h, ctypes.byref(m))
        self.M = m.value
        return self.M

    def finalize_async(self):
        """Enqueue the column table; finalize_wait() returns M."""
        call("karma_kmer_plan_finalize_async", self.h)

    def finalize_wait(self):
        m = ctypes.c_int64()
        call("karma_kmer_plan_finalize_wait", self.h, ctypes.byref(m))
        self.M = m.value
        return self.M

    def columns(self):
        keys = np.zeros(max(self.M, 1), dtype=np.uint64)
        call("karma_kmer_columns", self.h, ptr(keys))
        return keys[: self.M]

    def row_totals(self):
        out = np.zeros(max(self.store.n, 1), dtype=np.int64)
        call("karma_kmer_row_totals", self.h, ptr(out))
        return out[: self.store.n]

    def profile_host(self):
        out = np.zeros((self.store.n, self.M), dtype=np.float64)
        if out.size:
            call("karma_kmer_profile", self.h, ptr(out), self.M, 0)
        return out

    def profile_rows(self, lo, hi, out):
        """Rows [lo, hi) into a host float64 array of hi - lo rows (C order,
        row stride = its second dimension >= M)."""
        assert out.dtype == np.float64 and out.flags.c_contiguous and out.shape[0] == hi - lo
        if hi > lo:
            call("karma_kmer_profile_rows", self.h, lo, hi, ptr(out), out.shape[1], 0)

    def profile_device(self, dst_dev_ptr, ld=None):
        call("karma_kmer_profile", self.h, ctypes.c_void_p(dst_dev_ptr), ld or self.M, 1)

    def profile_side(self, dst_dev_ptr, side_stream_ptr, ld=None):
        """profile_device on a side stream, after the work already enqueued on the
        context's stream; the context joins it with Context.join(side)."""
        call("karma_kmer_profile_side", self.h, ctypes.c_void_p(dst_dev_ptr), ld or self.M,
             ctypes.c_void_p(side_stream_ptr))

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_kmer_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


BLOCK_BYTES = 4 << 30  # row blocks of a streamed profile (device buffer and D2H unit)


def kmer_profile(sequences, kmer_size, ctx=None, out=None, block_bytes=None):
    """Full single-device k-mer profile of an OrderedDict (kmer.py:199-233).

    out: None (a new array), or a caller float64[N, M] C-order array -- a
    numpy.memmap for a profile larger than host memory -- that is filled one
    row block (~block_bytes) at a time (SURVEY.md §8(e) streaming).  Its shape
    must be (N, M); M is the column count the sequences give (kmer_columns).
    Returns (profile, columns list[str], row_totals int64[N])."""
    ctx = ctx or _lib.default_context()
    kmode = kmode_of(kmer_size)
    packed = getattr(sequences, "karma_packed", None)  # fasta.FastaDict straight from the C++ reader
    blob, offs, key_len = packed if packed is not None else encode_sequences(sequences)
    store = ContigStore(ctx, blob, offs, key_len)
    try:
        plan = KmerPlan(ctx, store, kmode)
        try:
            M = plan.finalize()
            cols = decode_keys(plan.columns(), kmode)
            n = store.n
            big = n * M * 8 > (block_bytes or BLOCK_BYTES)
            if out is None and not big:
                prof = plan.profile_host()
            else:
                if out is None:
                    out = np.empty((n, M), np.float64)
                if out.shape != (n, M) or out.dtype != np.float64 or not out.flags.c_contiguous:
                    raise ValueError(f"out must be a C-order float64 array of shape {(n, M)}")
                for lo, hi, blk in _row_blocks(plan, n, M, block_bytes):
                    out[lo:hi] = blk
                prof = out
            tot = plan.row_totals()
        finally:
            plan.close()
    finally:
        store.close()
    return prof, cols, tot


def _row_blocks(plan, n, M, block_bytes=None, ring=1):
    """(lo, hi, block) over the profile's rows; blocks are host arrays reused
    round-robin from a ring of `ring` (a consumer may hold ring - 1 of them)."""
    rows = max(1, min(n, (block_bytes or BLOCK_BYTES) // max(1, 8 * M)))
    bufs = [np.empty((rows, M), np.float64) for _ in range(max(1, ring))]
    for i, lo in enumerate(range(0, n, rows)):
        hi = min(n, lo + rows)
        blk = bufs[i % len(bufs)][: hi - lo]
        plan.profile_rows(lo, hi, blk)  # M == 0: the row totals only
        yield lo, hi, blk


def kmer_profile_blocks(sequences, kmer_size, block_rows, ctx=None, ring=1):
    """The profile as a stream of (lo, hi, rows float64[hi - lo, M]) row blocks
    and the column list: (columns, generator).  Block arrays are reused from a
    ring of `ring` buffers: a consumer may keep the last ring - 1 blocks while
    it advances (e.g. hash them on a thread pool).  Nothing of size N x M
    exists on the host or the device at once (SURVEY.md §8(e) C5 streaming)."""
    ctx = ctx or _lib.default_context()
    kmode = kmode_of(kmer_size)
    packed = getattr(sequences, "karma_packed", None)
    blob, offs, key_len = packed if packed is not None else encode_sequences(sequences)
    store = ContigStore(ctx, blob, offs, key_len)
    plan = KmerPlan(ctx, store, kmode)
    M = plan.finalize()
    cols = decode_keys(plan.columns(), kmode)

    def gen():
        try:
            yield from _row_blocks(plan, store.n, M, block_rows * max(1, 8 * M), ring)
        finally:
            plan.close()
            store.close()

    return cols, gen()


def kmer_columns_count(sequences, kmer_size, ctx=None):
    """M: the number of columns (present k-mers) of the sequences' profile."""
    ctx = ctx or _lib.default_context()
    kmode = kmode_of(kmer_size)
    packed = getattr(sequences, "karma_packed", None)
    blob, offs, key_len = packed if packed is not None else encode_sequences(sequences)
    store = ContigStore(ctx, blob, offs, key_len)
    try:
        plan = KmerPlan(ctx, store, kmode)
        try:
            return plan.finalize()
        finally:
            plan.close()
    finally:
        store.close()


def kmer_profile_device(sequences, kmer_size, ctx=None):
    """kmer_profile with the profile left in HBM:
    returns (DeviceProfile, columns list[str], row_totals int64[N]); nothing of
    size N x M crosses PCIe."""
    from .device_profile import profile_to_device

    ctx = ctx or _lib.default_context()
    kmode = kmode_of(kmer_size)
    packed = getattr(sequences, "karma_packed", None)
    blob, offs, key_len = packed if packed is not None else encode_sequences(sequences)
    store = ContigStore(ctx, blob, offs, key_len)
    try:
        plan = KmerPlan(ctx, store, kmode)
        try:
            plan.finalize()
            cols = decode_keys(plan.columns(), kmode)
            dev = profile_to_device(ctx, plan, cols)
            tot = plan.row_totals()
        finally:
            plan.close()
    finally:
        store.close()
    return dev, cols, tot


# ---------------------------------------------------------------------------
# Graph
# ---------------------------------------------------------------------------

class GraphJob:
    """An open karma_graph_records_begin call (one per context)."""

    def __init__(self, pairs_cls, ctx, h):
        self.pairs_cls, self.ctx, self.h = pairs_cls, ctx, h

    def end(self):
        h, self.h = self.h, None
        out = ctypes.c_void_p()
        call("karma_graph_records_end", h, ctypes.byref(out))
        return self.pairs_cls(self.ctx, out)

    def __del__(self):
        if getattr(self, "h", None):  # never ended: end it (frees the job and its list)
            try:
                self.end().close()
            except Exception:
                pass


class Pairs:
    """Sorted unique (a << 32 | b, count) list (karma_pairs)."""

    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, h

    @classmethod
    def from_records(cls, ctx, records, n_contigs, grouped=True, device_ptr=None, n_records=None, flagged=False):
        """flagged: the records are KARMA_REC_FLAGGED words (flag_records), one u32 each."""
        h = ctypes.c_void_p()
        flags = _lib.KARMA_REC_FLAGGED if flagged else _lib.KARMA_REC_SORTED if grouped else _lib.KARMA_REC_UNSORTED
        if device_ptr is not None:
            call("karma_graph_records", ctx.h, ctypes.c_void_p(device_ptr), n_records, n_contigs, flags, 1,
                 ctypes.byref(h))
        else:
            rec = np.ascontiguousarray(records, dtype=np.uint32)
            rec = rec.reshape(-1) if flagged else rec.reshape(-1, 2)
            call("karma_graph_records", ctx.h, ptr(rec) if len(rec) else None, len(rec), n_contigs, flags, 0,
                 ctypes.byref(h))
        return cls(ctx, h)

    @classmethod
    def from_records_begin(cls, ctx, n_contigs, device_ptr, n_records, grouped=True, split_bounds=None,
                           flagged=False):
        """First half of from_records on device records (karma_graph_records_begin):
        the pipeline is enqueued up to its host synchronisation; .end() finishes.
        split_bounds: owner bounds the list will be split at (karma_graph_split_hint)."""
        if split_bounds is not None:
            b = np.ascontiguousarray(split_bounds, np.int64)
            call("karma_graph_split_hint", ctx.h, ptr(b), len(b) - 1)
        h = ctypes.c_void_p()
        flags = _lib.KARMA_REC_FLAGGED if flagged else _lib.KARMA_REC_SORTED if grouped else _lib.KARMA_REC_UNSORTED
        call("karma_graph_records_begin", ctx.h, ctypes.c_void_p(device_ptr), n_records, n_contigs, flags, 1,
             ctypes.byref(h))
        return GraphJob(cls, ctx, h)

    @classmethod
    def from_eq(cls, ctx, cls_off, members, counts, pair_skip, n_contigs):
        h = ctypes.c_void_p()
        cls_off = np.ascontiguousarray(cls_off, np.int64)
        members = np.ascontiguousarray(members, np.uint32)
        counts = np.ascontiguousarray(counts, np.int64)
        skip = np.ascontiguousarray(pair_skip, np.uint8)
        call("karma_graph_eq", ctx.h, ptr(cls_off), ptr(members) if len(members) else None,
             ptr(counts) if len(counts) else None, ptr(skip) if len(skip) else None, len(cls_off) - 1, n_contigs, 0,
             ctypes.byref(h))
        return cls(ctx, h)

    @classmethod
    def from_eq_compact(cls, ctx, sizes, members, counts32, n_contigs):
        """karma_graph_eq_compact: sizes uint8[C] (member count | 0x80 for the
        size token "1"), members uint32, counts uint32[C]."""
        h = ctypes.c_void_p()
        sizes = np.ascontiguousarray(sizes, np.uint8)
        members = np.ascontiguousarray(members, np.uint32)
        counts32 = np.ascontiguousarray(counts32, np.uint32)
        call("karma_graph_eq_compact", ctx.h, ptr(sizes) if len(sizes) else None,
             ptr(members) if len(members) else None, len(members), ptr(counts32) if len(counts32) else None,
             len(sizes), n_contigs, ctypes.byref(h))
        return cls(ctx, h)

    @classmethod
    def merge_runs_kc(cls, ctx, kc_dev_ptr, runs):
        """Merge received runs of interleaved (key, count) int64 pairs in device memory."""
        off = np.zeros(len(runs) + 1, np.int64)
        np.cumsum(np.asarray(runs, np.int64), out=off[1:])
        h = ctypes.c_void_p()
        call("karma_pairs_merge_runs_kc", ctx.h, ctypes.c_void_p(kc_dev_ptr) if kc_dev_ptr else None, ptr(off),
             len(runs), ctypes.byref(h))
        return cls(ctx, h)

    def get_kc(self, kc_dev_ptr):
        """Interleaved (key, count) int64 pairs into device memory (stream-ordered)."""
        call("karma_pairs_get_kc", self.h, ctypes.c_void_p(kc_dev_ptr) if kc_dev_ptr else None)

    @classmethod
    def merge(cls, ctx, keys, counts, device=False, n=None, runs=None):
        """Sorted unique (key, count) list.  runs = lengths of consecutive runs that
        are each sorted by key (an exchange owner's received slices): merged by a
        merge tree instead of a full sort."""
        h = ctypes.c_void_p()
        if runs is not None:
            if device:
                # the run offsets as a ctypes array (no numpy on this per-step path)
                off = (ctypes.c_int64 * (len(runs) + 1))(0, *itertools.accumulate(int(r) for r in runs))
                assert n is None or n == off[len(runs)], "run lengths do not add up to n"
                call("karma_pairs_merge_runs", ctx.h, ctypes.c_void_p(keys) if keys else None,
                     ctypes.c_void_p(counts) if counts else None, off, len(runs), 1, ctypes.byref(h))
                return cls(ctx, h)
            off = np.zeros(len(runs) + 1, np.int64)
            np.cumsum(np.asarray(runs, np.int64), out=off[1:])
            keys = np.ascontiguousarray(keys, np.uint64)
            counts = np.ascontiguousarray(counts, np.int64)
            call("karma_pairs_merge_runs", ctx.h, ptr(keys) if len(keys) else None,
                 ptr(counts) if len(counts) else None, ptr(off), len(runs), 0, ctypes.byref(h))
            return cls(ctx, h)
        if device:
            call("karma_pairs_merge", ctx.h, ctypes.c_void_p(keys) if keys else None,
                 ctypes.c_void_p(counts) if counts else None, n, 1, ctypes.byref(h))
        else:
            keys = np.ascontiguousarray(keys, np.uint64)
            counts = np.ascontiguousarray(counts, np.int64)
            call("karma_pairs_merge", ctx.h, ptr(keys) if len(keys) else None, ptr(counts) if len(counts) else None,
                 len(keys), 0, ctypes.byref(h))
        return cls(ctx, h)

    def count(self):
        n = ctypes.c_int64()
        call("karma_pairs_count", self.h, ctypes.byref(n))
        return n.value

    def device_ptrs(self):
        k, c = ctypes.c_void_p(), ctypes.c_void_p()
        call("karma_pairs_device", self.h, ctypes.byref(k), ctypes.byref(c))
        return k.value, c.value

    def get(self):
        n = self.count()
        keys = np.zeros(max(n, 1), np.uint64)
        counts = np.zeros(max(n, 1), np.int64)
        first = np.zeros(max(n, 1), np.uint64)
        call("karma_pairs_get", self.h, ptr(keys), ptr(counts), ptr(first), 0)
        return keys[:n], counts[:n], first[:n]

    def split(self, bounds):
        bounds = np.ascontiguousarray(bounds, np.int64)
        starts = np.zeros(len(bounds), np.int64)
        call("karma_pairs_split", self.h, ptr(bounds), len(bounds) - 1, ptr(starts))
        return starts

    def split_kc(self, bounds, kc_dev_ptr):
        """split(bounds) and get_kc(kc_dev_ptr) in one launch (karma_pairs_split_kc)."""
        bounds = np.ascontiguousarray(bounds, np.int64)
        starts = np.zeros(len(bounds), np.int64)
        call("karma_pairs_split_kc", self.h, ptr(bounds), len(bounds) - 1, ptr(starts),
             ctypes.c_void_p(kc_dev_ptr) if kc_dev_ptr else None)
        return starts

    def edges_begin(self, mode, n_contigs):
        """First half of edges() (karma_edges_begin): returns the open Edges and the
        device address of its int64[n_contigs] totals, for an all-gather before
        Edges.end() computes the weights."""
        h = ctypes.c_void_p()
        tp = ctypes.c_void_p()
        call("karma_edges_begin", self.ctx.h, self.h, mode, n_contigs, ctypes.byref(h), ctypes.byref(tp))
        e = Edges(self.ctx, h, -1, n_contigs)
        e._pairs = self  # the list stays alive until end()
        return e, tp.value

    def totals_device(self, dst_dev_ptr, n_contigs):
        call("karma_pairs_totals", self.h, ctypes.c_void_p(dst_dev_ptr), n_contigs)

    def edges(self, mode, n_contigs, totals_dev_ptr=None):
        h = ctypes.c_void_p()
        E = ctypes.c_int64()
        call("karma_edges_from_pairs", self.ctx.h, self.h, mode,
             ctypes.c_void_p(totals_dev_ptr) if totals_dev_ptr else None, n_contigs, ctypes.byref(h),
             ctypes.byref(E))
        return Edges(self.ctx, h, E.value, n_contigs)

    def rebind(self, ctx):
        """Run later kernels on this list on ``ctx``'s stream (karma_pairs_rebind)."""
        call("karma_pairs_rebind", self.h, ctx.h)
        self.ctx = ctx

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_pairs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


@dataclass
class EdgeArrays:
    a: np.ndarray
    b: np.ndarray
    shared: np.ndarray
    weight: np.ndarray
    first: np.ndarray
    totals: np.ndarray


class Edges:
    def __init__(self, ctx, h, E, n_contigs):
        self.ctx, self.h, self._E, self.n_contigs = ctx, h, E, n_contigs

    @property
    def E(self):
        """Edge count; after end(count=False) its first read synchronises and
        reports the edge stage's errors (karma_edges_count)."""
        if self._E is None:
            E = ctypes.c_int64()
            call("karma_edges_count", self.h, ctypes.byref(E))
            self._E = E.value
        return self._E

    def end(self, count=True):
        """Second half of Pairs.edges_begin (karma_edges_end): weights, and the
        edge count (count=False: launched only; E is read when first used)."""
        if count:
            E = ctypes.c_int64()
            call("karma_edges_end", self.h, ctypes.byref(E))
            self._E = E.value
        else:
            call("karma_edges_end", self.h, None)
            self._E = None
        self._pairs = None
        return self

    def get(self) -> EdgeArrays:
        """The edges in host arrays (pinned host memory: the copies run at the
        full PCIe rate; the blocks return to the library's cache with the arrays)."""
        E = self.E
        e1, n1 = max(E, 1), max(self.n_contigs, 1)
        # one pinned block: s, w, f, totals (8-byte items) then a, b (4-byte)
        blk = _lib.pinned_empty(8 * (3 * e1 + n1) + 4 * (2 * e1 + 1), np.uint8)
        o = [0]

        def take(n, dt):
            dt = np.dtype(dt)
            v = blk[o[0]:o[0] + n * dt.itemsize].view(dt)
            o[0] += n * dt.itemsize
            return v
        s, w, f, t = take(e1, np.int64), take(e1, np.float64), take(e1, np.uint64), take(n1, np.int64)
        a, b = take(e1, np.uint32), take(e1, np.uint32)
        call("karma_edges_get_all", self.h, ptr(a), ptr(b), ptr(s), ptr(w), ptr(f), ptr(t), 0)
        return EdgeArrays(a[:E], b[:E], s[:E], w[:E], f[:E], t[: self.n_contigs])

    def get_ordered(self):
        """Eq edge stages: (a, b, w) in the reference's insertion order -- by a,
        then by the pair's first emission (read_graph.py:96-131), ordered on the
        device (karma_edges_get_ordered); one pinned block."""
        E = self.E
        e1 = max(E, 1)
        blk = _lib.pinned_empty(16 * e1, np.uint8)
        w = blk[: 8 * e1].view(np.float64)
        a = blk[8 * e1: 12 * e1].view(np.uint32)
        b = blk[12 * e1:].view(np.uint32)
        call("karma_edges_get_ordered", self.h, ptr(a), ptr(b), ptr(w), 0)
        return a[:E], b[:E], w[:E]

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_edges_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def graph_from_records(records, n_contigs, grouped=True, ctx=None, flagged=False) -> EdgeArrays:
    """Shared-read edges from (read, contig) records (read_graph.py:19-50 semantics);
    flagged: records given as flag_records words."""
    ctx = ctx or _lib.default_context()
    p = Pairs.from_records(ctx, records, n_contigs, grouped=grouped, flagged=flagged)
    try:
        e = p.edges(_lib.KARMA_MODE_READS, n_contigs)
        try:
            return e.get()
        finally:
            e.close()
    finally:
        p.close()


def graph_from_eq(cls_off, members, counts, pair_skip, n_contigs, ctx=None) -> EdgeArrays:
    """Eq-class edges (read_graph.py:86-131 semantics), with first-emission order."""
    ctx = ctx or _lib.default_context()
    p = Pairs.from_eq(ctx, cls_off, members, counts, pair_skip, n_contigs)
    try:
        e = p.edges(_lib.KARMA_MODE_EQ, n_contigs)
        try:
            return e.get()
        finally:
            e.close()
    finally:
        p.close()


def graph_from_eq_ordered(cls_off, members, counts, pair_skip, n_contigs, ctx=None):
    """Eq-class edges as the drop-in needs them: (a, b, w) in the reference's
    insertion order (read_graph.py:96-131), ordered on the device."""
    ctx = ctx or _lib.default_context()
    p = Pairs.from_eq(ctx, cls_off, members, counts, pair_skip, n_contigs)
    try:
        e = p.edges(_lib.KARMA_MODE_EQ, n_contigs)
        try:
            return e.get_ordered()
        finally:
            e.close()
    finally:
        p.close()


def eq_compact(cls_off, counts, pair_skip):
    """(sizes uint8, counts uint32) of wide eq arrays for karma_graph_eq_compact,
    or None when a class has > 127 members or a count past 2^32 - 1 (the form
    the C++ parser emits directly, ingest.parse_eq(compact=True))."""
    m = np.diff(np.asarray(cls_off, np.int64))
    counts = np.asarray(counts, np.int64)
    if len(m) and (m.max() > 127 or counts.min() < 0 or counts.max() > 0xFFFFFFFF):
        return None
    sizes = m.astype(np.uint8)
    if pair_skip is not None and len(pair_skip):
        sizes |= (np.asarray(pair_skip, np.uint8) != 0).astype(np.uint8) << 7
    return sizes, counts.astype(np.uint32)


def graph_from_eq_compact_ordered(sizes, members, counts32, n_contigs, ctx=None):
    """graph_from_eq_ordered from the compact inputs (karma_graph_eq_compact)."""
    ctx = ctx or _lib.default_context()
    p = Pairs.from_eq_compact(ctx, sizes, members, counts32, n_contigs)
    try:
        e = p.edges(_lib.KARMA_MODE_EQ, n_contigs)
        try:
            return e.get_ordered()
        finally:
            e.close()
    finally:
        p.close()


# ---------------------------------------------------------------------------
# Synthetic inputs through the native generator (twin of synth.py)
# ---------------------------------------------------------------------------

def synth_contigs(seed, n, len_min=400, len_span=800, n_rate=0, first=0):
    """(blob uint8, offsets int64[n+1], key_len int32[n]) of contigs ">ctg<i>",
    i in [first, first + n) of the global synthetic set (counter-based, so a
    shard generates only its own rows)."""
    lens = np.zeros(first + n, np.int64)
    call("karma_synth_contig_lengths", seed, first + n, len_min, len_span, ptr(lens))
    goffs = np.zeros(first + n + 1, np.int64)
    np.cumsum(lens, out=goffs[1:])
    gslice = np.ascontiguousarray(goffs[first:])
    blob = np.zeros(int(gslice[-1] - gslice[0]) + 16, np.uint8)
    call("karma_synth_contig_bases", seed, ptr(gslice), n, n_rate, ptr(blob))
    offs = gslice - gslice[0]
    key_len = _key_lens(first + n)[first:].copy()
    return blob, offs, key_len


def _key_lens(n):
    i = np.arange(n)
    digits = np.ones(n, np.int32)
    p = 10
    while p <= n:
        digits += (i >= p)
        p *= 10
    return (4 + digits).astype(np.int32)


def synth_genes(seed, n_contigs, gene_max=4):
    ng = ctypes.c_int64()
    call("karma_synth_n_genes", seed, n_contigs, gene_max, ctypes.byref(ng))
    gf = np.zeros(ng.value, np.int64)
    gs = np.zeros(ng.value, np.int32)
    call("karma_synth_genes", seed, n_contigs, gene_max, ptr(gf), ptr(gs))
    return gf, gs


def flag_records(records):
    """(read, contig) records grouped by read -> KARMA_REC_FLAGGED words (the
    read ids replaced by read-start flags): contig | (first record of its read) << 31.
    The graph depends only on which records share a read, so the two formats
    give the same graph."""
    rec = np.asarray(records, np.uint32).reshape(-1, 2)
    if len(rec) and int(rec[:, 1].max()) >= 1 << 31:
        raise ValueError("flagged records hold contig ids < 2^31")
    out = rec[:, 1].copy()
    if len(rec):
        start = np.empty(len(rec), np.uint32)
        start[0] = 1
        np.not_equal(rec[1:, 0], rec[:-1, 0], out=start[1:], casting="unsafe")
        out |= start << np.uint32(31)
    return out


def synth_records(seed, n_contigs, frag_lo, frag_hi, paired, gene_max=4, genes=None):
    """records uint32[A, 2] (read, contig) for fragments [frag_lo, frag_hi)."""
    gf, gs = genes if genes is not None else synth_genes(seed, n_contigs, gene_max)
    nf = frag_hi - frag_lo
    cnt = np.zeros(max(nf, 1), np.int32)
    call("karma_synth_read_counts", seed, ptr(gf), ptr(gs), len(gf), frag_lo, frag_hi, int(paired), ptr(cnt))
    off = np.zeros(nf + 1, np.int64)
    np.cumsum(cnt[:nf], out=off[1:])
    rec = np.zeros((max(int(off[-1]), 1), 2), np.uint32)
    call("karma_synth_read_records", seed, ptr(gf), ptr(gs), len(gf), frag_lo, frag_hi, int(paired), ptr(off),
         ptr(rec))
    return rec[: int(off[-1])]


def synth_eq_classes(seed, n_contigs, frag_lo, frag_hi, paired, gene_max=4, genes=None):
    """(cls_off int64[C+1], members uint32[], counts int64[C]) of the fragments'
    eq classes, first-seen order (native twin of synth.eq_classes)."""
    gf, gs = genes if genes is not None else synth_genes(seed, n_contigs, gene_max)
    nc, nm = ctypes.c_int64(), ctypes.c_int64()
    call("karma_synth_eq_classes", seed, ptr(gf), ptr(gs), len(gf), frag_lo, frag_hi, int(paired), ctypes.byref(nc),
         ctypes.byref(nm), None, None, None)
    off = np.zeros(nc.value + 1, np.int64)
    mem = np.zeros(max(nm.value, 1), np.uint32)
    cnt = np.zeros(max(nc.value, 1), np.int64)
    call("karma_synth_eq_classes", seed, ptr(gf), ptr(gs), len(gf), frag_lo, frag_hi, int(paired), ctypes.byref(nc),
         ctypes.byref(nm), ptr(off), ptr(mem), ptr(cnt))
    return off, mem[: nm.value], cnt[: nc.value]
