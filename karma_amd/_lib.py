"""ctypes binding of libkarma_hip.so (C ABI in include/karma.h).

This is the ONLY way the package reaches the compute path: there is no CPU
fallback.  If the library is missing or no gfx950 device is visible, every
entry point raises KarmaError — loudly — instead of computing something else.
"""

from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# KARMA_LIB: an alternative build of the same library (tools/build_variant.sh A/B timing)
LIB_PATH = os.environ.get("KARMA_LIB") or os.path.join(HERE, "libkarma_hip.so")

KARMA_OK = 0
KARMA_ERR_ARG = -1
KARMA_ERR_KMER = -2
KARMA_ERR_HIP = -3
KARMA_ERR_OOM = -4
KARMA_ERR_ZERO_DIV = -5
KARMA_ERR_UNSORTED = -6
KARMA_ERR_STATE = -7
KARMA_ERR_PARSE = -8
KARMA_ERR_COMM = -9
KARMA_ERR_STALL = -10

KARMA_DT_U8, KARMA_DT_I32, KARMA_DT_I64, KARMA_DT_U64, KARMA_DT_F64 = 0, 1, 2, 3, 4
KARMA_OP_SUM, KARMA_OP_MAX, KARMA_OP_MIN = 0, 1, 2
KARMA_COMM_SIDE = 1
_DTYPE_CODE = {np.dtype(np.uint8): KARMA_DT_U8, np.dtype(np.int32): KARMA_DT_I32, np.dtype(np.int64): KARMA_DT_I64,
               np.dtype(np.uint64): KARMA_DT_U64, np.dtype(np.float64): KARMA_DT_F64}

KARMA_KMER_5P6 = -1
KARMA_REC_SORTED = 0
KARMA_REC_UNSORTED = 1
KARMA_REC_FLAGGED = 2
KARMA_STEP_FLAGGED = 8
KARMA_MODE_READS = 0
KARMA_MODE_EQ = 1
KARMA_STEP_KEEP, KARMA_STEP_SEQUENTIAL, KARMA_STEP_DEFER = 1, 2, 4

_c_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_u64 = ctypes.c_uint64
_PP = ctypes.POINTER(ctypes.c_void_p)
_I64P = ctypes.POINTER(ctypes.c_int64)

# name -> (restype is int status, argtypes)
_SIGS = {
    "karma_version": [],
    "karma_device_count": [ctypes.POINTER(ctypes.c_int)],
    "karma_ctx_create": [_i32, _PP],
    "karma_ctx_destroy": [_c_p],
    "karma_ctx_set_stream": [_c_p, _c_p],
    "karma_ctx_sync": [_c_p],
    "karma_timing_enable": [_c_p, _i32],
    "karma_timing_only": [_c_p, ctypes.c_char_p],
    "karma_timing_reset": [_c_p],
    "karma_timing_read": [_c_p, ctypes.c_char_p, _c_p, _c_p, _i32, ctypes.POINTER(ctypes.c_int)],
    "karma_dev_alloc": [_c_p, ctypes.c_size_t, _PP],
    "karma_dev_free": [_c_p, _c_p],
    "karma_memcpy": [_c_p, _c_p, _c_p, ctypes.c_size_t, _i32],
    "karma_memcpy_async": [_c_p, _c_p, _c_p, ctypes.c_size_t, _i32],
    "karma_memset_async": [_c_p, _c_p, _i32, ctypes.c_size_t],
    "karma_host_alloc": [ctypes.c_size_t, _PP],
    "karma_host_free": [_c_p],
    "karma_memset_timed": [_c_p, _c_p, ctypes.c_size_t, _i32, ctypes.POINTER(ctypes.c_double)],
    "karma_stream_create": [_c_p, _i32, _PP],
    "karma_stream_destroy": [_c_p, _c_p],
    "karma_stream_sync": [_c_p, _c_p],
    "karma_comm_unique_id": [_c_p],
    "karma_comm_create": [_c_p, _c_p, _i32, _i32, _PP],
    "karma_comm_create_ex": [_c_p, _c_p, _i32, _i32, _i32, _PP],
    "karma_mapped_slots": [_c_p, _c_p, _i32, ctypes.POINTER(ctypes.c_int)],
    "karma_comm_destroy": [_c_p],
    "karma_comm_info": [_c_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    "karma_comm_allreduce": [_c_p, _c_p, _i64, _i32, _i32],
    "karma_comm_allreduce_host": [_c_p, _c_p, _i64, _i32, _i32],
    "karma_comm_barrier": [_c_p],
    "karma_comm_allgather": [_c_p, _c_p, _c_p, _i64],
    "karma_comm_exchange_counts": [_c_p, _c_p, _c_p],
    "karma_comm_alltoallv": [_c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_comm_alltoallv_kv": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_contigs_create": [_c_p, _c_p, _c_p, _c_p, _i64, _i32, _PP],
    "karma_contigs_destroy": [_c_p],
    "karma_contigs_info": [_c_p, _I64P, _I64P, _I64P, _I64P],
    "karma_kmer_plan_create": [_c_p, _c_p, _i32, _PP],
    "karma_kmer_plan_destroy": [_c_p],
    "karma_kmer_presence_words": [_c_p, _I64P],
    "karma_kmer_presence_get": [_c_p, _c_p],
    "karma_kmer_presence_set": [_c_p, _c_p],
    "karma_kmer_presence_merge": [_c_p, _c_p, _i32],
    "karma_kmer_exceptions_count": [_c_p, _I64P],
    "karma_kmer_exceptions_get": [_c_p, _c_p],
    "karma_kmer_exceptions_set": [_c_p, _c_p, _i64],
    "karma_kmer_plan_finalize": [_c_p, _I64P],
    "karma_kmer_plan_finalize_async": [_c_p],
    "karma_kmer_plan_finalize_wait": [_c_p, _I64P],
    "karma_kmer_columns": [_c_p, _c_p],
    "karma_kmer_profile": [_c_p, _c_p, _i64, _i32],
    "karma_kmer_profile_rows": [_c_p, _i64, _i64, _c_p, _i64, _i32],
    "karma_kmer_profile_side": [_c_p, _c_p, _i64, _c_p],
    "karma_ctx_join": [_c_p, _c_p],
    "karma_ctx_set_side_headroom": [_c_p, _i32],
    "karma_kmer_row_totals": [_c_p, _c_p],
    "karma_graph_records": [_c_p, _c_p, _i64, _i64, _i32, _i32, _PP],
    "karma_graph_records_begin": [_c_p, _c_p, _i64, _i64, _i32, _i32, _PP],
    "karma_graph_records_end": [_c_p, _PP],
    "karma_graph_split_hint": [_c_p, _c_p, _i32],
    "karma_graph_eq": [_c_p, _c_p, _c_p, _c_p, _c_p, _i64, _i64, _i32, _PP],
    "karma_graph_eq_compact": [_c_p, _c_p, _c_p, _i64, _c_p, _i64, _i64, _PP],
    "karma_pairs_merge": [_c_p, _c_p, _c_p, _i64, _i32, _PP],
    "karma_pairs_merge_runs": [_c_p, _c_p, _c_p, _c_p, _i32, _i32, _PP],
    "karma_pairs_merge_runs_kc": [_c_p, _c_p, _c_p, _i32, _PP],
    "karma_pairs_get_kc": [_c_p, _c_p],
    "karma_pairs_destroy": [_c_p],
    "karma_pairs_rebind": [_c_p, _c_p],
    "karma_pairs_count": [_c_p, _I64P],
    "karma_pairs_device": [_c_p, _PP, _PP],
    "karma_pairs_get": [_c_p, _c_p, _c_p, _c_p, _i32],
    "karma_pairs_split": [_c_p, _c_p, _i32, _c_p],
    "karma_pairs_totals": [_c_p, _c_p, _i64],
    "karma_edges_from_pairs": [_c_p, _c_p, _i32, _c_p, _i64, _PP, _I64P],
    "karma_edges_begin": [_c_p, _c_p, _i32, _i64, _PP, _PP],
    "karma_edges_end": [_c_p, _I64P],
    "karma_edges_count": [_c_p, _I64P],
    "karma_pairs_split_kc": [_c_p, _c_p, _i32, _c_p, _c_p],
    "karma_edges_destroy": [_c_p],
    "karma_edges_get": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _i32],
    "karma_edges_totals": [_c_p, _c_p, _i32],
    "karma_edges_get_all": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _i32],
    "karma_edges_get_ordered": [_c_p, _c_p, _c_p, _c_p, _i32],
    "karma_api_calls": [_c_p],
    "karma_step_create": [_c_p, _c_p, _c_p, _i32, _i64, _c_p, _i32, _i32, _PP],
    "karma_step_run": [_c_p, _c_p, _c_p, _i64, _i32, _c_p],
    "karma_step_sync": [_c_p],
    "karma_step_info": [_c_p, _c_p, _i32],
    "karma_step_profile": [_c_p, _PP, _I64P, _I64P],
    "karma_step_columns": [_c_p, _c_p],
    "karma_step_edges": [_c_p, _PP],
    "karma_step_newest_edges": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _i64, _i32, _I64P, _c_p],
    "karma_step_destroy": [_c_p],
    "karma_synth_contig_lengths": [_u64, _i64, _i32, _i32, _c_p],
    "karma_synth_contig_bases": [_u64, _c_p, _i64, _i32, _c_p],
    "karma_synth_n_genes": [_u64, _i64, _i32, _I64P],
    "karma_synth_genes": [_u64, _i64, _i32, _c_p, _c_p],
    "karma_synth_read_counts": [_u64, _c_p, _c_p, _i64, _i64, _i64, _i32, _c_p],
    "karma_synth_read_records": [_u64, _c_p, _c_p, _i64, _i64, _i64, _i32, _c_p, _c_p],
    "karma_synth_eq_classes": [_u64, _c_p, _c_p, _i64, _i64, _i64, _i32, _I64P, _I64P, _c_p, _c_p, _c_p],
    "karma_fasta_parse": [_c_p, ctypes.c_size_t, _i32, _PP],
    "karma_fasta_info": [_c_p, _I64P, _I64P, _I64P, ctypes.POINTER(ctypes.c_int)],
    "karma_fasta_get": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_fasta_view": [_c_p, _PP, _PP, _PP, _PP, _PP],
    "karma_fasta_destroy": [_c_p],
    "karma_eq_parse": [_c_p, ctypes.c_size_t, _i32, _PP],
    "karma_eq_info": [_c_p, _I64P, _I64P, _I64P, _I64P],
    "karma_eq_get": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_eq_get_compact": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_eq_destroy": [_c_p],
    "karma_sam_parse": [_c_p, ctypes.c_size_t, _i32, _i32, _PP],
    "karma_sam_info": [_c_p, _I64P, _I64P, _I64P, _I64P, _I64P],
    "karma_sam_get": [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_sam_destroy": [_c_p],
    "karma_adj_from_edges": [_c_p, _i64, _c_p, _c_p, _c_p, _c_p, _i64, _i32, _PP],
    "karma_adj_from_lists": [_c_p, _i64, _c_p, _c_p, _c_p, _c_p, _i32, _PP],
    "karma_adj_view": [_c_p, _c_p, _i64, _PP],
    "karma_adj_keep": [_c_p, _c_p, _i64, _PP],
    "karma_adj_view_summary": [_c_p, _c_p, _i64, _c_p, _c_p, _i32, _c_p, _c_p, _c_p, _i64, _I64P,
                               ctypes.POINTER(ctypes.c_int)],
    "karma_adj_node_stats": [_c_p, _c_p, _c_p],
    "karma_adj_info": [_c_p, _I64P, _I64P],
    "karma_adj_get": [_c_p, _c_p, _c_p, _c_p, _c_p],
    "karma_adj_degrees": [_c_p, _c_p],
    "karma_adj_node_weights": [_c_p, _c_p],
    "karma_adj_edge_list": [_c_p, _c_p, _c_p, _i64, _i32, _c_p, _i64, _I64P],
    "karma_adj_cross_sums": [_c_p, _c_p, _c_p, ctypes.c_double, _c_p, _c_p, _c_p, _c_p, _i64, _I64P],
    "karma_adj_destroy": [_c_p],
    "karma_repr_f64_host": [_c_p, _i64, _c_p, _i64, _I64P],
}

EXPORTED = tuple(_SIGS) + ("karma_last_error", "karma_comm_id_bytes", "karma_build_info")


class KarmaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libkarma_hip error {code}: {msg}")
        self.code = code


_LIB = None


def load():
    """Load libkarma_hip.so (no GPU needed to load; compute calls need one)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise KarmaError(KARMA_ERR_HIP, f"{LIB_PATH} not built — run `make -C karma_amd/csrc` "
                                        "(or __graft_entry__.build()); there is no CPU fallback")
    # No PyTorch on this path: device memory, streams and the RCCL
    # communicator all come from the library itself, so the process holds one
    # HIP runtime (ROCm's, /opt/rocm/lib) by construction.
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    lib.karma_last_error.argtypes = []
    lib.karma_last_error.restype = ctypes.c_char_p
    lib.karma_comm_id_bytes.argtypes = []
    lib.karma_comm_id_bytes.restype = ctypes.c_int
    lib.karma_build_info.argtypes = []
    lib.karma_build_info.restype = ctypes.c_char_p
    _LIB = lib
    return lib


def build_info():
    """The loaded library's build identity (karma_build_info): arch, extra -D
    defines of a variant build ("" for the shipped library), source hash."""
    import json

    info = json.loads(load().karma_build_info().decode())
    info["library"] = os.path.relpath(LIB_PATH, os.path.dirname(HERE))
    return info


def check(rc):
    if rc != KARMA_OK:
        msg = load().karma_last_error().decode(errors="replace")
        raise KarmaError(rc, msg)
    return rc


# diagnostic: per-entry-point host time (KARMA_CALL_TIMES=1; tools/host_profile.py),
# and with KARMA_CALL_TIMES=seq every call's (name, start, end) in CALL_SEQ
# (tools/host_timeline.py)
CALL_TIMES = {} if os.environ.get("KARMA_CALL_TIMES") in ("1", "seq") else None
CALL_SEQ = [] if os.environ.get("KARMA_CALL_TIMES") == "seq" else None


def call(name, *args):
    if CALL_TIMES is None:
        return check(getattr(load(), name)(*args))
    import time

    t0 = time.perf_counter()
    try:
        return check(getattr(load(), name)(*args))
    finally:
        t1 = time.perf_counter()
        n, tot = CALL_TIMES.get(name, (0, 0.0))
        CALL_TIMES[name] = (n + 1, tot + t1 - t0)
        if CALL_SEQ is not None:
            CALL_SEQ.append((name, t0, t1))


def ptr(a):
    """Host numpy array -> c_void_p (None for None)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


class Context:
    """One HIP device + stream (karma_ctx).  Objects created from it must be
    destroyed before it (they are, through their own close())."""

    def __init__(self, device=0):
        lib = load()
        n = ctypes.c_int(0)
        rc = lib.karma_device_count(ctypes.byref(n))
        if rc != KARMA_OK or n.value == 0:
            raise KarmaError(KARMA_ERR_HIP, "no HIP device visible: libkarma_hip needs an MI355X (gfx950); "
                                            "there is no CPU fallback")
        h = ctypes.c_void_p()
        call("karma_ctx_create", device, ctypes.byref(h))
        self.h = h
        self.device = device

    def set_stream(self, stream):
        """Launch on `stream` (a Stream or a raw hipStream_t; None: the context's own)."""
        raw = stream.ptr if isinstance(stream, Stream) else stream
        call("karma_ctx_set_stream", self.h, ctypes.c_void_p(raw) if raw else None)

    def sync(self):
        call("karma_ctx_sync", self.h)

    def set_side_headroom(self, blocks_per_cu):
        call("karma_ctx_set_side_headroom", self.h, int(blocks_per_cu))

    def join(self, side):
        """This context's stream waits (on the device) for work on a side stream."""
        raw = side.ptr if isinstance(side, Stream) else side
        call("karma_ctx_join", self.h, ctypes.c_void_p(raw))

    def timing(self, on=True, only=None):
        """Per-kernel HIP-event timing; `only` restricts it to one kernel name."""
        call("karma_timing_only", self.h, (only or "").encode())
        call("karma_timing_enable", self.h, 1 if on else 0)

    def timing_reset(self):
        call("karma_timing_reset", self.h)

    def timing_read(self, cap=64):
        names = ctypes.create_string_buffer(64 * cap)
        ms = np.zeros(cap, np.float64)
        cnt = np.zeros(cap, np.int64)
        n = ctypes.c_int(0)
        call("karma_timing_read", self.h, names, ptr(ms), ptr(cnt), cap, ctypes.byref(n))
        out = {}
        raw = names.raw
        for i in range(min(n.value, cap)):
            nm = raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode()
            out[nm] = (float(ms[i]), int(cnt[i]))
        return out

    def close(self):
        if getattr(self, "h", None):
            load().karma_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Stream:
    """A HIP stream owned by the library (karma_stream_create)."""

    def __init__(self, ctx, priority=0):
        h = ctypes.c_void_p()
        call("karma_stream_create", ctx.h, int(priority), ctypes.byref(h))
        self.ctx, self.ptr = ctx, h.value

    def sync(self):
        call("karma_stream_sync", self.ctx.h, ctypes.c_void_p(self.ptr))

    def close(self):
        if getattr(self, "ptr", None) and self.ctx.h:
            load().karma_stream_destroy(self.ctx.h, ctypes.c_void_p(self.ptr))
        self.ptr = None


class DevBuf:
    """Device memory from the context's caching allocator (karma_dev_alloc),
    typed like a 1-D/2-D numpy array.  Copies in and out go through the
    context's stream; `numpy()` and `copy_from()` wait for it."""

    def __init__(self, ctx, shape, dtype, _ptr=None, _owner=None):
        self.ctx = ctx
        # plain Python arithmetic: a buffer is made per exchange step, where
        # numpy's scalar helpers cost microseconds each
        self.shape = tuple(int(x) for x in shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        size = 1
        for x in self.shape:
            size *= x
        self.size = size
        self.nbytes = size * self.dtype.itemsize
        self._owner = _owner
        if _ptr is not None:
            self.ptr = _ptr
            return
        h = ctypes.c_void_p()
        call("karma_dev_alloc", ctx.h, max(self.nbytes, 1), ctypes.byref(h))
        self.ptr = h.value

    @classmethod
    def from_numpy(cls, ctx, arr):
        arr = np.ascontiguousarray(arr)
        b = cls(ctx, arr.shape, arr.dtype)
        b.copy_from(arr)
        return b

    def view(self, start, n, shape=None):
        """Elements [start, start + n) as a buffer that does not own its memory."""
        assert 0 <= start and start + n <= self.size, "view out of range"
        return DevBuf(self.ctx, shape or (n,), self.dtype, _ptr=self.ptr + start * self.dtype.itemsize,
                      _owner=self)

    def reshape(self, *shape):
        shape = shape[0] if len(shape) == 1 and not np.isscalar(shape[0]) else shape
        out = DevBuf(self.ctx, shape, self.dtype, _ptr=self.ptr, _owner=self)
        assert out.size == self.size, "reshape changes the size"
        return out

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            call("karma_memcpy", self.ctx.h, ptr(out), ctypes.c_void_p(self.ptr), self.nbytes, 1)
        return out

    def copy_from(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self.dtype)
        assert arr.nbytes <= self.nbytes, "host array larger than the buffer"
        if arr.nbytes:
            call("karma_memcpy", self.ctx.h, ctypes.c_void_p(self.ptr), ptr(arr), arr.nbytes, 0)

    def copy_from_device(self, src, nbytes=None, dst_offset=0, src_offset=0):
        """Stream-ordered device-to-device copy (bytes)."""
        n = src.nbytes if nbytes is None else nbytes
        if n:
            call("karma_memcpy_async", self.ctx.h, ctypes.c_void_p(self.ptr + dst_offset),
                 ctypes.c_void_p(src.ptr + src_offset), n, 2)

    def close(self):
        if self._owner is None and getattr(self, "ptr", None) and self.ctx.h:
            load().karma_dev_free(self.ctx.h, ctypes.c_void_p(self.ptr))
        self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pinned_empty(n, dtype):
    """An uninitialised numpy array of n items in pinned host memory
    (karma_host_alloc): device -> host copies into it run at the full PCIe
    rate.  The block returns to the library's cache when the last array or
    view over it is collected."""
    dtype = np.dtype(dtype)
    nbytes = max(int(n), 1) * dtype.itemsize
    p = ctypes.c_void_p()
    call("karma_host_alloc", nbytes, ctypes.byref(p))
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    weakref.finalize(buf, _host_free, p.value)
    return np.frombuffer(buf, dtype=dtype, count=int(n))


def _host_free(addr):
    lib = _LIB
    if lib is not None:
        lib.karma_host_free(ctypes.c_void_p(addr))


def api_calls():
    """HIP runtime (and RCCL) calls this thread has made through the library (karma_api_calls)."""
    n = ctypes.c_uint64(0)
    call("karma_api_calls", ctypes.byref(n))
    return n.value


def dtype_code(dtype):
    return _DTYPE_CODE[np.dtype(dtype)]


_DEFAULT_CTX = {}


def default_context(device=0):
    ctx = _DEFAULT_CTX.get(device)
    if ctx is None:
        ctx = _DEFAULT_CTX[device] = Context(device)
    return ctx
