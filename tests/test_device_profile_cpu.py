"""DLPack capsule bookkeeping of karma_amd.device_profile (CPU; no device
memory is touched: a stand-in buffer records when it would be freed)."""
import ctypes

from karma_amd import device_profile as dp


class _Buf:
    def __init__(self):
        self.ptr, self.freed = 0x10000, 0

    def close(self):
        self.freed += 1


class _Ctx:
    device = 3


def test_capsule_released_when_unconsumed():
    b = _Buf()
    p = dp.DeviceProfile(_Ctx(), b, 5, 7, ["AAAAA"])
    cap = p.__dlpack__()
    assert len(dp._LIVE) == 1
    (struct, shape, owner), = dp._LIVE.values()
    t = struct.dl_tensor
    assert t.data == 0x10000 and t.ndim == 2 and list(shape) == [5, 7]
    assert (t.device.device_type, t.device.device_id) == (10, 3)
    assert (t.dtype.code, t.dtype.bits, t.dtype.lanes) == (2, 64, 1) and not t.strides
    del cap
    assert not dp._LIVE and b.freed == 0
    p.close()
    assert b.freed == 1


def test_close_waits_for_live_export():
    b = _Buf()
    p = dp.DeviceProfile(_Ctx(), b, 2, 2, [])
    cap = p.__dlpack__()
    p.close()
    assert b.freed == 0  # a consumer may still hold it
    del cap  # never consumed: the capsule's destructor releases it
    assert b.freed == 1 and not dp._LIVE


def test_consumer_deleter_releases():
    b = _Buf()
    p = dp.DeviceProfile(_Ctx(), b, 2, 2, [])
    p.__dlpack__()  # capsule dropped at once: released
    cap = p.__dlpack__()
    (struct, _, _), = dp._LIVE.values()
    p.close()
    struct.deleter(ctypes.pointer(struct))  # what a consumer does when its tensor dies
    assert b.freed == 1 and not dp._LIVE
    del cap
