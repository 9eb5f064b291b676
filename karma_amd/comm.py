"""Communicators of the sharded build.

The multi-GPU build needs five collectives, all in its two exchange steps:
  allgather_fixed   the ranks' presence bitmaps (OR-merged on the device: the
                    column set is the global sorted union, kmer.py:146-179)
  allgather_var     the ranks' non-ACGT k-mer keys
  alltoallv         pre-reduced (key, count) pairs to the owner of contig a
  allgather_slices_ the owners' readset totals
  max_float / sum_int / barrier / allgather_host   host scalars and bounds

RcclComm  production: the library's own RCCL communicator (karma_comm_*,
          csrc/comm.hip) on device buffers, enqueued on the context's stream;
          RCCL runs over xGMI between the GPUs of a node.
HostComm  host-staged transport over a hostgroup (threads or a TCP star), for
          rehearsals RCCL cannot run: several ranks sharing ONE GPU (RCCL
          refuses duplicate devices) and CPU-only tests of the sharding logic.
          It moves bytes only; the compute stays on the device (or, in the CPU
          tests, in the test's oracle backend).
SoloComm  world size 1: no collectives.

Buffers are karma_amd._lib.DevBuf (device) or numpy arrays (CPU test backend).
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import DevBuf, call, ptr


class SoloComm:
    world, rank = 1, 0

    def barrier(self):
        pass

    def max_float(self, x):
        return x

    def sum_int(self, x):
        return x

    def allgather_host(self, arr):
        return [np.asarray(arr).reshape(-1)]

    def allgather_fixed(self, buf):
        return buf

    def allgather_var(self, buf):
        return buf

    def allgather_slices_(self, buf, bounds):
        return buf

    def alltoallv(self, buf, send_counts):
        return buf, [int(x) for x in send_counts]

    def alltoallv_kv(self, a, b, send_counts):
        return a, b, [int(x) for x in send_counts]

    def close(self):
        pass


def _to_host(b):
    return b if isinstance(b, np.ndarray) else b.numpy()


def _like(b, arr):
    return arr if isinstance(b, np.ndarray) else DevBuf.from_numpy(b.ctx, arr)


def _write(b, arr):
    if isinstance(b, np.ndarray):
        b.reshape(-1)[:] = arr.reshape(-1)
    else:
        b.copy_from(arr)


class HostComm:
    """Collectives staged through host memory over a hostgroup (see module doc)."""

    def __init__(self, group):
        self.group, self.world, self.rank = group, group.world, group.rank

    def barrier(self):
        self.group.barrier()

    def max_float(self, x):
        return float(max(a[0] for a in self.group.allgather(np.array([x], np.float64))))

    def sum_int(self, x):
        return int(sum(int(a[0]) for a in self.group.allgather(np.array([x], np.int64))))

    def allgather_host(self, arr):
        return self.group.allgather(np.asarray(arr))

    def allgather_fixed(self, buf):
        parts = self.group.allgather(_to_host(buf).reshape(-1))
        return _like(buf, np.concatenate(parts))

    def allgather_var(self, buf):
        return self.allgather_fixed(buf)

    def allgather_slices_(self, buf, bounds):
        h = _to_host(buf).reshape(-1)
        lo, hi = int(bounds[self.rank]), int(bounds[self.rank + 1])
        parts = self.group.allgather(h[lo:hi])
        for r, p in enumerate(parts):
            h[int(bounds[r]):int(bounds[r + 1])] = p
        _write(buf, h)
        return buf

    def alltoallv(self, buf, send_counts):
        h = _to_host(buf).reshape(-1)
        counts = np.asarray(send_counts, np.int64)
        assert counts.sum() == h.size, "send counts do not cover the buffer"
        allc = self.group.allgather(counts)
        alld = self.group.allgather(h)
        me = self.rank
        pieces, recv = [], []
        for r in range(self.world):
            off = int(allc[r][:me].sum())
            n = int(allc[r][me])
            pieces.append(alld[r][off:off + n])
            recv.append(n)
        out = np.concatenate(pieces) if pieces else h[:0]
        return _like(buf, out.astype(h.dtype, copy=False)), recv

    def alltoallv_kv(self, a, b, send_counts):
        ra, recv = self.alltoallv(a, send_counts)
        rb, _ = self.alltoallv(b, send_counts)
        return ra, rb, recv

    def close(self):
        self.group.close()


class RcclComm:
    """The library's RCCL communicator on one device (karma_comm_*).

    One communicator by default: the native step (csrc/step.hip) issues every
    collective of a step on one stream in the same order on every rank, so no
    two collectives are ever in flight at once.  with_side=True (or
    KARMA_STEP_SIDE_COMM=1) adds a second communicator over the same ranks,
    `side` (KARMA_COMM_SIDE, its own unique id), for the column set's exchange
    on the side stream beside the main one's operations (round 4's mode)."""

    def __init__(self, group, ctx, with_side=None):
        if with_side is None:
            with_side = os.environ.get("KARMA_STEP_SIDE_COMM", "0") == "1"
        self.group, self.world, self.rank, self.ctx = group, group.world, group.rank, ctx
        lib = _lib.load()
        nb = lib.karma_comm_id_bytes()
        nid = 2 if with_side and self.world > 1 else 1
        uid = np.zeros(nid * nb, np.uint8)
        if self.rank == 0:
            for i in range(nid):
                call("karma_comm_unique_id", ctypes.c_void_p(uid.ctypes.data + i * nb))
        uid = np.ascontiguousarray(self.group.allgather(uid)[0])
        self.h = self._create(uid[:nb], 0)
        self.side, self._side_of = self, None
        if nid == 2:
            s = RcclComm.__new__(RcclComm)
            s.group, s.world, s.rank, s.ctx = group, self.world, self.rank, ctx
            s.h = self._create(uid[nb:], _lib.KARMA_COMM_SIDE)
            s.side, s._side_of = s, self
            self.side = s

    def _create(self, uid, flags):
        h = ctypes.c_void_p()
        call("karma_comm_create_ex", self.ctx.h, ptr(np.ascontiguousarray(uid)), self.world, self.rank, flags,
             ctypes.byref(h))
        return h

    def info(self):
        """(ranks, rank) as the RCCL communicator itself reports them."""
        w, r = ctypes.c_int(0), ctypes.c_int(0)
        call("karma_comm_info", self.h, ctypes.byref(w), ctypes.byref(r))
        return w.value, r.value

    # -- host scalars --
    def _reduce_host(self, arr, op):
        arr = np.ascontiguousarray(arr)
        call("karma_comm_allreduce_host", self.h, ptr(arr), arr.size, _lib.dtype_code(arr.dtype), op)
        return arr

    def barrier(self):
        call("karma_comm_barrier", self.h)

    def max_float(self, x):
        return float(self._reduce_host(np.array([x], np.float64), _lib.KARMA_OP_MAX)[0])

    def sum_int(self, x):
        return int(self._reduce_host(np.array([x], np.int64), _lib.KARMA_OP_SUM)[0])

    def allgather_host(self, arr):
        return self.group.allgather(np.asarray(arr))

    def _sizes(self, n):
        v = np.zeros(self.world, np.int64)
        v[self.rank] = n
        return self._reduce_host(v, _lib.KARMA_OP_SUM)

    # -- device buffers (stream-ordered on the context's stream) --
    def allgather_fixed(self, buf):
        out = DevBuf(self.ctx, (self.world * buf.size,), buf.dtype)
        call("karma_comm_allgather", self.h, ctypes.c_void_p(buf.ptr), ctypes.c_void_p(out.ptr), buf.nbytes)
        return out

    def _gather_padded(self, buf, sizes):
        """Every rank's first sizes[r] elements, padded to the largest, gathered."""
        isz = buf.dtype.itemsize
        mx = int(sizes.max())
        send = DevBuf(self.ctx, (max(mx, 1),), buf.dtype)
        send.copy_from_device(buf, int(sizes[self.rank]) * isz)
        allb = DevBuf(self.ctx, (self.world * max(mx, 1),), buf.dtype)
        call("karma_comm_allgather", self.h, ctypes.c_void_p(send.ptr), ctypes.c_void_p(allb.ptr), max(mx, 1) * isz)
        return allb, max(mx, 1)

    def allgather_var(self, buf):
        sizes = self._sizes(buf.size)
        allb, mx = self._gather_padded(buf, sizes)
        out = DevBuf(self.ctx, (int(sizes.sum()),), buf.dtype)
        isz, off = buf.dtype.itemsize, 0
        for r in range(self.world):
            out.copy_from_device(allb, int(sizes[r]) * isz, off * isz, r * mx * isz)
            off += int(sizes[r])
        return out

    def allgather_slices_(self, buf, bounds):
        bounds = np.asarray(bounds, np.int64)
        sizes = np.diff(bounds)
        isz = buf.dtype.itemsize
        if bounds[0] == 0 and np.all(sizes == sizes[0]) and sizes[0] > 0:
            # equal shards: in place (send = my slice of the receive buffer)
            n = int(sizes[0])
            call("karma_comm_allgather", self.h, ctypes.c_void_p(buf.ptr + self.rank * n * isz),
                 ctypes.c_void_p(buf.ptr), n * isz)
            return buf
        mine = buf.view(int(bounds[self.rank]), int(sizes[self.rank]))
        allb, mx = self._gather_padded(mine, sizes)
        for r in range(self.world):
            if r != self.rank:
                buf.copy_from_device(allb, int(sizes[r]) * isz, int(bounds[r]) * isz, r * mx * isz)
        return buf

    def alltoallv(self, buf, send_counts):
        isz = buf.dtype.itemsize
        sc = np.ascontiguousarray(send_counts, np.int64)
        rc = np.zeros(self.world, np.int64)
        call("karma_comm_exchange_counts", self.h, ptr(sc), ptr(rc))
        soff = np.zeros(self.world + 1, np.int64)
        roff = np.zeros(self.world + 1, np.int64)
        np.cumsum(sc * isz, out=soff[1:])
        np.cumsum(rc * isz, out=roff[1:])
        out = DevBuf(self.ctx, (int(rc.sum()),), buf.dtype)
        call("karma_comm_alltoallv", self.h, ctypes.c_void_p(buf.ptr), ptr(soff), ctypes.c_void_p(out.ptr), ptr(roff))
        return out, [int(x) for x in rc]

    def alltoallv_kv(self, a, b, send_counts):
        """alltoallv of a list held as two arrays of one element size (keys and
        counts): two grouped sends per peer, no interleaved copy."""
        assert a.dtype.itemsize == b.dtype.itemsize and a.size == b.size
        isz = a.dtype.itemsize
        sc = np.ascontiguousarray(send_counts, np.int64)
        rc = np.zeros(self.world, np.int64)
        call("karma_comm_exchange_counts", self.h, ptr(sc), ptr(rc))
        soff = np.zeros(self.world + 1, np.int64)
        roff = np.zeros(self.world + 1, np.int64)
        np.cumsum(sc * isz, out=soff[1:])
        np.cumsum(rc * isz, out=roff[1:])
        ra = DevBuf(self.ctx, (int(rc.sum()),), a.dtype)
        rb = DevBuf(self.ctx, (int(rc.sum()),), b.dtype)
        call("karma_comm_alltoallv_kv", self.h, ctypes.c_void_p(a.ptr), ctypes.c_void_p(b.ptr), ptr(soff),
             ctypes.c_void_p(ra.ptr), ctypes.c_void_p(rb.ptr), ptr(roff))
        return ra, rb, [int(x) for x in rc]

    def close(self):
        if self.side is not self:
            self.side.close()
            self.side = self
        if getattr(self, "h", None):
            _lib.load().karma_comm_destroy(self.h)
            self.h = None
        if self._side_of is None:  # the side communicator shares the main one's group
            self.group.close()


def create(ctx=None, world=None, rank=None, backend=None):
    """The communicator of a launcher-started rank (RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT, as torchrun sets them).

    backend: "rccl" (default: the library's RCCL communicator on ctx's device)
    or "host" (KARMA_DIST_BACKEND=host: host-staged, for several ranks on one
    GPU)."""
    from .hostgroup import SocketGroup

    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    if world == 1:
        return SoloComm()
    backend = backend or os.environ.get("KARMA_DIST_BACKEND", "rccl")
    group = SocketGroup.from_env(world, rank)
    if backend == "host":
        return HostComm(group)
    if backend != "rccl":
        raise ValueError(f"unknown KARMA_DIST_BACKEND {backend!r} (rccl | host)")
    return RcclComm(group, ctx)
