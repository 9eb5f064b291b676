"""CPU checks of the C ABI: the library loads, exports every function that
include/karma.h declares, and its host-only entry points (the synthetic
generator) match the Python specification byte for byte.  No GPU calls."""
import ctypes
import os
import re

import numpy as np

from karma_amd import _lib, engine, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "karma.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(karma_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) > 40
    for name in declared:
        assert hasattr(lib, name), name
    # the Python binding covers the whole header
    assert set(declared) == set(_lib.EXPORTED)


def test_version_and_error_string():
    lib = _lib.load()
    assert lib.karma_version() == 1
    assert isinstance(lib.karma_last_error(), bytes)


def test_synth_contigs_match_spec():
    for seed, n, lmin, lspan, nrate in [(1, 40, 400, 800, 0), (11, 64, 5, 300, 40), (14, 32, 1, 60, 7)]:
        ref = synth.contig_sequences(seed, n, lmin, lspan, nrate)
        blob, offs, key_len = engine.synth_contigs(seed, n, lmin, lspan, nrate)
        got = [bytes(blob[offs[i]:offs[i + 1]]).decode() for i in range(n)]
        assert got == list(ref.values())
        assert key_len.tolist() == [len(k) for k in ref.keys()]


def test_synth_records_match_spec():
    for seed, n, nf, paired in [(1, 1000, 3000, False), (21, 300, 2000, True), (3, 7, 500, True)]:
        ref = synth.read_records(seed, n, nf, paired)
        got = engine.synth_records(seed, n, 0, nf, paired)
        assert got.tolist() == [list(r) for r in ref]
        # ranges compose (per-rank generation)
        a = engine.synth_records(seed, n, 0, nf // 3, paired)
        b = engine.synth_records(seed, n, nf // 3, nf, paired)
        assert np.concatenate([a, b]).tolist() == got.tolist()


def test_key_lens_vectorised():
    n = 12345
    assert engine._key_lens(n).tolist() == [len(f">ctg{i}") for i in range(n)]


def test_no_cpu_fallback_without_device():
    # On a machine without a GPU the product path must refuse, not compute.
    n = ctypes.c_int(-1)
    rc = _lib.load().karma_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        return  # GPU box: covered by the gpu tests
    import pytest
    with pytest.raises(_lib.KarmaError):
        engine.kmer_profile({">a": "ACGTACGT"}, 5)


def test_default_build_is_auditable():
    # the shipped library adds no -D flags (a variant from tools/build_variant.sh
    # records its flags and bench.py refuses it), and its source hash is the
    # hash of the sources in the tree
    import hashlib
    import glob

    info = _lib.build_info()
    assert info["arch"] == "gfx950"
    assert info["defines"] == ""
    csrc = os.path.join(REPO, "karma_amd", "csrc")
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))
                  + glob.glob(os.path.join(csrc, "*.cpp")) + [os.path.join(REPO, "include", "karma.h")],
                  key=lambda p: os.path.relpath(p, csrc))
    h = hashlib.sha256()
    for p in srcs:
        h.update(open(p, "rb").read())
    assert info["src_sha256_16"] == h.hexdigest()[:16], "libkarma_hip.so is stale: rebuild (make -C karma_amd/csrc)"
    # no work-removing diagnostic switches in the product kernels
    for p in srcs:
        assert "ABLATE" not in open(p).read(), p


def test_mapped_slots_are_distinct():
    """A context's mapped host region is cut into fixed per-user slots (the
    comm scalars, the count exchange, the split, the merge and edge status
    words, the consumers, the step status): none overlaps another, every one is
    aligned, and the region never has to grow (core.hip ctx_mapped)."""
    n = ctypes.c_int(0)
    off = np.zeros(32, np.int64)
    nb = np.zeros(32, np.int64)
    _lib.call("karma_mapped_slots", _lib.ptr(off), _lib.ptr(nb), 32, ctypes.byref(n))
    k = n.value
    assert k >= 7
    spans = sorted((int(o), int(o + b)) for o, b in zip(off[:k], nb[:k]))
    assert all(b > 0 for b in nb[:k])
    assert all(o % 256 == 0 for o in off[:k])
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0, "mapped slots overlap"
    # the users that may run on different streams at once have their own slots
    assert len(set(off[:k].tolist())) == k
