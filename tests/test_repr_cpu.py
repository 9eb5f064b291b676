"""CPU check of the device's repr(float) formatter (csrc/repr.h, Ryu shortest
digits + CPython's float_repr_style layout), through its host build
(karma_repr_f64_host).  The oracle is CPython's own repr(), which
ReadGraph.edge_list's f-string uses (karma/read_graph.py:356).  No GPU calls."""
import ctypes

import numpy as np

from karma_amd import _lib


def host_repr(x):
    x = np.ascontiguousarray(x, np.float64)
    n = _lib._i64(0)
    _lib.call("karma_repr_f64_host", _lib.ptr(x), len(x), None, 0, ctypes.byref(n))
    buf = ctypes.create_string_buffer(max(1, n.value))
    _lib.call("karma_repr_f64_host", _lib.ptr(x), len(x), buf, n.value, ctypes.byref(n))
    return buf.raw[:n.value].decode().split("\n")[:-1]


def check(x):
    got = host_repr(x)
    want = [repr(float(v)) for v in np.asarray(x, np.float64).tolist()]
    bad = [(w, g) for w, g in zip(want, got) if w != g]
    assert len(got) == len(want) and not bad, bad[:5]


def test_special_values_and_layout_boundaries():
    check([0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 0.2, 0.3, 2.0 / 3, 1e16, 1e15, 9999999999999998.0, 1e-4, 9.999e-5,
           1e-5, 0.0001234, 5e-324, 2.2250738585072014e-308, 2.225073858507201e-308, 1.7976931348623157e308,
           float("inf"), -float("inf"), float("nan"), 9007199254740993.0, 123456789012345678.0, 1e22, 1e23,
           1e100, 1e-100, 1e-7, 1234.5, 0.1 + 0.2])


def test_powers_of_two_and_ten():
    check(2.0 ** np.arange(-1074, 1024, dtype=np.float64))
    check(np.array([float(f"1e{e}") for e in range(-323, 309)]))


def test_random_bit_patterns():
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2**63, 300_000, dtype=np.int64).view(np.uint64)
    check(bits.view(np.float64))
    check(-bits.view(np.float64)[:1000])


def test_weight_shaped_values():
    # the read graph's weights: (s/a + s/b) / 2 of integer counts (read_graph.py:39-42, :128-130)
    rng = np.random.default_rng(8)
    a = rng.integers(1, 10**7, 200_000)
    b = rng.integers(1, 10**7, 200_000)
    s = np.minimum(np.minimum(a, b), rng.integers(1, 10**7, 200_000))
    check((s / a + s / b) / 2)
    small = np.arange(1, 60)
    check([(x / y + x / z) / 2 for x in small for y in small[::7] for z in small[::5]])
