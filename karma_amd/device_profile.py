"""Device-resident k-mer profile hand-off.

The reference hands its dense profile to UMAP on the host
(karma/kmer.py:283-290: ``umap.UMAP(...).fit_transform(kmer_profile)``).  A GPU
consumer (a GPU UMAP or kNN) needs no host copy: ``DeviceProfile`` owns the
profile in HBM (float64, N x M, row-major = numpy C order, written by
``karma_kmer_profile(..., is_device=1)``) and exposes it through the two
zero-copy protocols device array libraries import from:

  * DLPack: ``__dlpack__`` / ``__dlpack_device__`` (device type kDLROCM = 10),
    e.g. ``torch.from_dlpack(profile)``;
  * ``__cuda_array_interface__`` (version 3; HIP's device pointers).

The profile kernel has finished when the object is handed out (its stream is
synchronised once), so consumers need no stream ordering.  The memory stays
alive while any consumer tensor refers to it.  ``numpy()`` copies it to the
host (the reference's return value).  This module is plain ctypes: no torch.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

KDL_ROCM = 10  # DLDeviceType kDLROCM
KDL_FLOAT = 2  # DLDataTypeCode kDLFloat


class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", _DELETER)]

# managed tensors handed out and not yet released: address -> (struct, shape, owner)
_LIVE = {}


def _release(addr):
    entry = _LIVE.pop(addr, None)
    if entry is not None:
        entry[2]._maybe_free()


@_DELETER
def _dl_deleter(mt):
    _release(ctypes.addressof(mt.contents))


# the destructor gets the dying capsule as a raw PyObject* (no new reference)
_CAPSULE_DTOR = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, _CAPSULE_DTOR]
_PyCapsule_IsValid = ctypes.pythonapi.PyCapsule_IsValid
_PyCapsule_IsValid.restype = ctypes.c_int
_PyCapsule_IsValid.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
_PyCapsule_GetPointer = ctypes.pythonapi.PyCapsule_GetPointer
_PyCapsule_GetPointer.restype = ctypes.c_void_p
_PyCapsule_GetPointer.argtypes = [ctypes.c_void_p, ctypes.c_char_p]


@_CAPSULE_DTOR
def _capsule_dtor(cap):
    # never consumed (a consumer renames the capsule to "used_dltensor" and
    # calls the deleter itself): release it here
    if _PyCapsule_IsValid(cap, b"dltensor"):
        _release(_PyCapsule_GetPointer(cap, b"dltensor"))


class DeviceProfile:
    """The dense float64 profile (N x M) resident on one device."""

    def __init__(self, ctx, buf, n, M, columns):
        self.ctx, self._buf, self._closed = ctx, buf, False
        self.shape = (int(n), int(M))
        self.dtype = np.dtype(np.float64)
        self.columns = columns

    @property
    def ptr(self) -> int:
        return int(self._buf.ptr or 0)

    @property
    def device(self) -> int:
        return self.ctx.device

    @property
    def nbytes(self) -> int:
        return self.shape[0] * self.shape[1] * 8

    def numpy(self) -> np.ndarray:
        """Host copy (what kmer.py:264 returns)."""
        if self._buf is None:
            raise ValueError("DeviceProfile is closed")
        return self._buf.numpy().reshape(self.shape)

    @property
    def __cuda_array_interface__(self):
        return {"shape": self.shape, "typestr": "<f8", "data": (self.ptr, False), "strides": None,
                "version": 3, "stream": None}

    def __dlpack_device__(self):
        return (KDL_ROCM, self.device)

    def __dlpack__(self, stream=None, max_version=None, dl_device=None, copy=None):
        if copy:
            raise BufferError("DeviceProfile exports its device memory without copies")
        if self._buf is None:
            raise BufferError("DeviceProfile is closed")
        mt = _DLManagedTensor()
        shape = (ctypes.c_int64 * 2)(*self.shape)
        mt.dl_tensor.data = self.ptr if self.nbytes else None
        mt.dl_tensor.device = _DLDevice(KDL_ROCM, self.device)
        mt.dl_tensor.ndim = 2
        mt.dl_tensor.dtype = _DLDataType(KDL_FLOAT, 64, 1)
        mt.dl_tensor.shape = shape
        mt.dl_tensor.strides = None  # compact row-major
        mt.dl_tensor.byte_offset = 0
        mt.manager_ctx = None
        mt.deleter = _dl_deleter
        addr = ctypes.addressof(mt)
        _LIVE[addr] = (mt, shape, self)  # keeps the device buffer alive until the consumer releases it
        return _PyCapsule_New(addr, b"dltensor", _capsule_dtor)

    def close(self):
        """Drop this handle; the memory is freed now, or when the last consumer
        tensor exported from it is released."""
        self._closed = True
        self._maybe_free()

    def _maybe_free(self):
        if self._closed and self._buf is not None and not any(v[2] is self for v in _LIVE.values()):
            self._buf.close()
            self._buf = None

    def __del__(self):  # unreachable while an export is live (_LIVE holds self)
        if getattr(self, "_buf", None) is not None:
            self._buf.close()
            self._buf = None


def profile_to_device(ctx, plan, columns) -> DeviceProfile:
    """Run a finalised KmerPlan's profile into a new device buffer and hand it
    over once written (one stream synchronisation, no host copy)."""
    n, M = plan.store.n, plan.M
    buf = _lib.DevBuf(ctx, (n, M), np.float64)
    if n:  # also with M == 0: the call zeroes the row totals (kmer.py:250-258 check)
        plan.profile_device(buf.ptr)
    ctx.sync()
    return DeviceProfile(ctx, buf, n, M, list(columns))
