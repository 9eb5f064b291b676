"""Host ingestion through the C++ parsers of libkarma_hip.so (csrc/ingest.cpp).

  parse_fasta  read_fasta_file's records (karma/karma.py:40-61)
  parse_eq     the eq_classes.txt parse (karma/read_graph.py:75-92)
  parse_sam    per-line (read, contig) records from SAM text (karma/contig.py:24,34)

Each returns plain numpy arrays.  The parsers accept exactly the input whose
reference result they reproduce and raise ``ParseDeferred`` for anything else.
The callers in fasta.py, read_graph.py and contig.py then run the reference's
own Python reading of that file, so a malformed file raises the reference's
exception (ValueError, KeyError, AssertionError, UnicodeDecodeError).
"""
import ctypes
import locale
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import KARMA_ERR_PARSE, KarmaError, call


class ParseDeferred(Exception):
    """The C++ parser declined; the reference-semantics reader decides."""


def _utf8_locale():
    # text-mode open() decodes with the locale's preferred encoding
    return locale.getpreferredencoding(False).lower().replace("-", "") in ("utf8",)


def _read(path):
    with open(path, "rb") as fh:
        return fh.read()


def _parse(fn, data, *args):
    h = ctypes.c_void_p()
    try:
        call(fn, ctypes.c_char_p(data), len(data), *args, ctypes.byref(h))
    except KarmaError as e:
        if e.code == KARMA_ERR_PARSE:
            raise ParseDeferred(str(e)) from None
        raise
    return h


def _buf(n, dtype):
    return np.empty(max(int(n), 1), dtype)


@dataclass
class FastaRecords:
    seq: np.ndarray       # uint8, UTF-8 (latin-1 == ASCII when ascii), + 16 bytes padding
    seq_off: np.ndarray   # int64[N + 1]
    keys: bytes           # UTF-8 key bytes
    key_off: np.ndarray   # int64[N + 1]
    key_len: np.ndarray   # int32[N], code points
    ascii: bool

    def __len__(self):
        return len(self.key_len)

    def names(self):
        return self._strs(memoryview(self.keys), self.key_off)

    def sequences(self):
        return self._strs(memoryview(self.seq), self.seq_off)

    def _strs(self, mv, off):
        o = off.tolist()
        if self.ascii:  # one decode, then str slices (code point offsets == byte offsets)
            whole = str(mv[:o[-1]], "ascii")
            return [whole[o[i]:o[i + 1]] for i in range(len(o) - 1)]
        return [str(mv[o[i]:o[i + 1]], "utf-8") for i in range(len(o) - 1)]


class _Handle:
    """Owns a parser handle; numpy views of its arrays keep it alive."""

    def __init__(self, h, destroy):
        self.h, self._destroy = h, destroy

    def __del__(self):
        if self.h:
            getattr(_lib.load(), self._destroy)(self.h)
            self.h = None


def _view(owner, addr, n, dtype):
    """numpy array over n items at addr; its base keeps `owner` alive."""
    if n == 0 or not addr:
        return np.zeros(0, dtype)
    raw = (ctypes.c_uint8 * (n * np.dtype(dtype).itemsize)).from_address(addr)
    raw._owner = owner
    return np.frombuffer(raw, dtype)


def parse_fasta(data: bytes, threads=0) -> FastaRecords:
    if not _utf8_locale():
        raise ParseDeferred("locale encoding is not UTF-8")
    own = _Handle(_parse("karma_fasta_parse", data, threads), "karma_fasta_destroy")
    n, sb, kb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    asc = ctypes.c_int()
    call("karma_fasta_info", own.h, ctypes.byref(n), ctypes.byref(sb), ctypes.byref(kb), ctypes.byref(asc))
    p = [ctypes.c_void_p() for _ in range(5)]
    call("karma_fasta_view", own.h, *[ctypes.byref(x) for x in p])
    N = n.value
    seq = _view(own, p[0].value, sb.value + 16, np.uint8)
    keys = ctypes.string_at(p[2].value, kb.value) if kb.value else b""
    return FastaRecords(seq, _view(own, p[1].value, N + 1, np.int64), keys, _view(own, p[3].value, N + 1, np.int64),
                        _view(own, p[4].value, N, np.int32), bool(asc.value))


@dataclass
class EqClasses:
    names: list
    cls_off: np.ndarray   # int64[C + 1]            (None in the compact form)
    members: np.ndarray   # uint32
    counts: np.ndarray    # int64[C]                (None in the compact form)
    pair_skip: np.ndarray  # uint8[C], eq_size token == "1" (None in the compact form)
    sizes: np.ndarray = None     # compact: uint8[C] member count | 0x80 for the token "1"
    counts32: np.ndarray = None  # compact: uint32[C]


def parse_eq(data: bytes, threads=0, compact=False) -> EqClasses:
    """compact=True: the karma_graph_eq_compact form when every class fits it
    (<= 127 members, counts < 2^32), in pinned host memory (the device copies
    run at the full PCIe rate); otherwise the wide form."""
    if not _utf8_locale():
        raise ParseDeferred("locale encoding is not UTF-8")
    h = _parse("karma_eq_parse", data, threads)
    try:
        v = [ctypes.c_int64() for _ in range(4)]
        call("karma_eq_info", h, *[ctypes.byref(x) for x in v])
        n, C, nm, nb = (x.value for x in v)
        names = ctypes.create_string_buffer(max(nb, 1))
        name_off = np.empty(n + 1, np.int64)
        if compact:
            try:
                sizes, mem, c32 = _lib.pinned_empty(C, np.uint8), _lib.pinned_empty(nm, np.uint32), \
                    _lib.pinned_empty(C, np.uint32)
            except KarmaError:  # no device to pin for (the parse itself is host code)
                sizes, mem, c32 = _buf(C, np.uint8), _buf(nm, np.uint32), _buf(C, np.uint32)
            rc = _lib.load().karma_eq_get_compact(h, names, _lib.ptr(name_off), _lib.ptr(sizes), _lib.ptr(mem),
                                                  _lib.ptr(c32))
            if rc == 0:
                raw, o = names.raw[:nb], name_off.tolist()
                return EqClasses([raw[o[i]:o[i + 1]].decode("utf-8") for i in range(n)], None, mem[:nm], None, None,
                                 sizes[:C], c32[:C])
        cls_off = np.empty(C + 1, np.int64)
        members = _buf(nm, np.uint32)
        counts = _buf(C, np.int64)
        skip = _buf(C, np.uint8)
        call("karma_eq_get", h, names, _lib.ptr(name_off), _lib.ptr(cls_off), _lib.ptr(members),
             _lib.ptr(counts), _lib.ptr(skip))
        raw, o = names.raw[:nb], name_off.tolist()
        return EqClasses([raw[o[i]:o[i + 1]].decode("utf-8") for i in range(n)], cls_off, members[:nm],
                         counts[:C], skip[:C])
    finally:
        _lib.load().karma_eq_destroy(h)


@dataclass
class SamRecords:
    records: np.ndarray   # uint32[L, 2]: read id, contig id (file order)
    rnames: list          # contig id -> RNAME, in order of first appearance
    q_start: np.ndarray   # int64[L]: QNAME byte range in the parsed buffer
    q_len: np.ndarray     # int32[L]
    n_reads: int
    read_id_bound: int


def parse_sam(data: bytes, skip_headers=True, threads=0) -> SamRecords:
    if not _utf8_locale():
        raise ParseDeferred("locale encoding is not UTF-8")
    h = _parse("karma_sam_parse", data, 1 if skip_headers else 0, threads)
    try:
        v = [ctypes.c_int64() for _ in range(5)]
        call("karma_sam_info", h, *[ctypes.byref(x) for x in v])
        L, nr, nc, rb, bound = (x.value for x in v)
        rec = np.empty((max(L, 1), 2), np.uint32)
        rn = ctypes.create_string_buffer(max(rb, 1))
        rn_off = np.empty(nc + 1, np.int64)
        qs = _buf(L, np.int64)
        ql = _buf(L, np.int32)
        call("karma_sam_get", h, _lib.ptr(rec), rn, _lib.ptr(rn_off), _lib.ptr(qs), _lib.ptr(ql))
        raw, o = rn.raw[:rb], rn_off.tolist()
        return SamRecords(rec[:L], [raw[o[i]:o[i + 1]].decode("utf-8") for i in range(nc)], qs[:L], ql[:L], nr,
                          bound)
    finally:
        _lib.load().karma_sam_destroy(h)
