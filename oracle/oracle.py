"""ctypes front-end of the CPU oracle (oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker (or as the timed CPU baseline).  The
product package ``karma_amd`` never imports it.

Each function restates the reference behaviour it names (file:line under
/root/reference) on top of the plain-C kernels in oracle.c.  Parity of the
oracle itself is pinned by tests/test_oracle_golden.py against
tests/golden/golden.json, which tests/golden/make_golden.py captured by running
the reference.
"""

from __future__ import annotations

import ctypes
import os
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

KEY_BYTES = 16  # {len, bytes[15]} records, see oracle.c okey_t

_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_f64p = ctypes.POINTER(ctypes.c_double)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        L.oracle_is_palindrome.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.oracle_is_palindrome.restype = ctypes.c_int
        L.oracle_kmer_columns.argtypes = [ctypes.c_void_p, _i64p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int64]
        L.oracle_kmer_columns.restype = ctypes.c_int64
        L.oracle_omp_kmer_columns.argtypes = L.oracle_kmer_columns.argtypes
        L.oracle_omp_kmer_columns.restype = ctypes.c_int64
        L.oracle_kmer_profile.argtypes = [ctypes.c_void_p, _i64p, _i64p, ctypes.c_int64, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int64, _f64p, ctypes.c_void_p]
        L.oracle_kmer_profile.restype = ctypes.c_int
        L.oracle_graph_groups.argtypes = [_i64p, _u32p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, _i64p, _u32p, _u32p, _i64p, _u64p, _f64p,
                                          ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
        L.oracle_graph_groups.restype = ctypes.c_int64
        for fn in (L.oracle_readset_pairs,):
            fn.argtypes = [_i64p, _u32p, ctypes.c_int64, _u32p, _u32p, _i64p, _f64p, ctypes.c_int64]
            fn.restype = ctypes.c_int64
        L.oracle_update_pairs.argtypes = [_i64p, _u32p, ctypes.c_int64, _i64p, _u32p, ctypes.c_int64, _u32p, _u32p,
                                          _i64p, _f64p, ctypes.c_int64]
        L.oracle_update_pairs.restype = ctypes.c_int64
        L.oracle_threads.argtypes = []
        L.oracle_threads.restype = ctypes.c_int
        L.oracle_omp_kmer_profile.argtypes = [ctypes.c_void_p, _i64p, _i64p, ctypes.c_int64, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_int64, _f64p]
        L.oracle_omp_kmer_profile.restype = ctypes.c_int
        L.oracle_omp_graph_reads.argtypes = [_i64p, _u32p, ctypes.c_int64, ctypes.c_int64, _i64p, _u32p, _u32p,
                                             _i64p, _f64p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
        L.oracle_omp_graph_reads.restype = ctypes.c_int64
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def is_palindrome(s: str) -> bool:
    """kmer.py:46-54."""
    b = s.encode("latin-1")
    return bool(lib().oracle_is_palindrome(b, len(b)))


def kmode_of(kmer_size) -> int:
    """kmer.py:69 compares with the string "5p6"; otherwise an int k (cmd_parser.py:234-235)."""
    return -1 if kmer_size == "5p6" else int(kmer_size)


def pack_sequences(sequences):
    """Concatenate values (latin-1) + offsets; key lengths (kmer.py:213 uses len(key))."""
    vals = [v.encode("latin-1") for v in sequences.values()]
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    if vals:
        offs[1:] = np.cumsum([len(v) for v in vals])
    blob = np.frombuffer(b"".join(vals) or b"\0", dtype=np.uint8).copy()
    key_len = np.array([len(k) for k in sequences.keys()], dtype=np.int64)
    return blob, offs, key_len


def decode_keys(raw: np.ndarray, M: int):
    recs = raw[: M * KEY_BYTES].reshape(M, KEY_BYTES)
    return [bytes(r[1:1 + r[0]]).decode("latin-1") for r in recs]


def kmer_columns(sequences, kmer_size):
    blob, offs, _ = pack_sequences(sequences)
    L = lib()
    km = kmode_of(kmer_size)
    cap = 1 << 16
    while True:
        raw = np.zeros(cap * KEY_BYTES, dtype=np.uint8)
        M = L.oracle_kmer_columns(_p(blob, ctypes.c_void_p), _p(offs, _i64p), len(sequences), km,
                                  _p(raw, ctypes.c_void_p), cap)
        if M == -(1 << 63):
            raise ValueError(f"oracle supports 1 <= k <= 15 or '5p6', got {kmer_size!r}")
        if M >= 0:
            return raw, M
        cap = -M


def omp_kmer_columns_packed(blob, offs, kmer_size):
    """kmer_columns of packed sequences on all host cores (oracle_omp_kmer_columns)."""
    L = lib()
    km = kmode_of(kmer_size)
    offs = np.ascontiguousarray(offs, np.int64)
    cap = 1 << 16
    while True:
        raw = np.zeros(cap * KEY_BYTES, dtype=np.uint8)
        M = L.oracle_omp_kmer_columns(_p(blob, ctypes.c_void_p), _p(offs, _i64p), len(offs) - 1, km,
                                      _p(raw, ctypes.c_void_p), cap)
        if M == -(1 << 63):
            raise ValueError(f"oracle supports 1 <= k <= 15 or '5p6', got {kmer_size!r}")
        if M >= 0:
            return raw, M
        cap = -M


def calc_kmer_profile(sequences, kmer_size, logger=None):
    """Restates KmerClustering.__calc_kmer_profile (kmer.py:199-264).

    Returns (profile float64[N, M], columns list[str], counts int64[N, M]).
    Raises SystemExit(1) for an all-zero column/row (kmer.py:236-258) and
    ZeroDivisionError for a zero-length key with a non-zero count (kmer.py:120).
    """
    blob, offs, key_len = pack_sequences(sequences)
    raw, M = kmer_columns(sequences, kmer_size)
    N = len(sequences)
    prof = np.zeros((N, M), dtype=np.float64)
    counts = np.zeros((N, M), dtype=np.int64)
    rc = lib().oracle_kmer_profile(_p(blob, ctypes.c_void_p), _p(offs, _i64p), _p(key_len, _i64p), N,
                                   kmode_of(kmer_size), _p(raw, ctypes.c_void_p), M, _p(prof, _f64p),
                                   _p(counts, ctypes.c_void_p))
    if rc == 1:
        raise AssertionError("oracle: k-mer missing from column set")
    if rc == 2:
        raise ZeroDivisionError("division by zero")
    cols = decode_keys(raw, M)
    for n in range(M):  # kmer.py:236-248
        if not counts[:, n].any():
            if logger:
                logger.error(f"Values of column {n} are all zero, which should not be the case.")
            raise SystemExit(1)
    for n in range(N):  # kmer.py:250-258
        if not counts[n, :].any():
            if logger:
                logger.error(f"Values of row {n} are all zero, which should not be the case.")
            raise SystemExit(1)
    return prof, cols, counts


# ---------------------------------------------------------------------------
# Shared-read graph
# ---------------------------------------------------------------------------

def graph_groups(grp_off, members, mult, pair_skip, n_nodes, dedup):
    """Group-based pair counting (oracle.c oracle_graph_groups)."""
    grp_off = np.ascontiguousarray(grp_off, dtype=np.int64)
    members = np.ascontiguousarray(members, dtype=np.uint32)
    G = len(grp_off) - 1
    mult_a = None if mult is None else np.ascontiguousarray(mult, dtype=np.int64)
    skip_a = None if pair_skip is None else np.ascontiguousarray(pair_skip, dtype=np.uint8)
    totals = np.zeros(max(n_nodes, 1), dtype=np.int64)
    cap = 1 << 12
    L = lib()
    while True:
        ea = np.zeros(cap, np.uint32)
        eb = np.zeros(cap, np.uint32)
        es = np.zeros(cap, np.int64)
        ef = np.zeros(cap, np.uint64)
        ew = np.zeros(cap, np.float64)
        zd = ctypes.c_int(0)
        E = L.oracle_graph_groups(_p(grp_off, _i64p), _p(members if len(members) else np.zeros(1, np.uint32), _u32p),
                                  None if mult_a is None else _p(mult_a, ctypes.c_void_p),
                                  None if skip_a is None else _p(skip_a, ctypes.c_void_p), G, n_nodes, int(dedup),
                                  _p(totals, _i64p), _p(ea, _u32p), _p(eb, _u32p), _p(es, _i64p), _p(ef, _u64p),
                                  _p(ew, _f64p), cap, ctypes.byref(zd))
        if E >= 0:
            break
        cap = -E
    return dict(a=ea[:E], b=eb[:E], shared=es[:E], first=ef[:E], weight=ew[:E], totals=totals[:n_nodes],
                zero_div=bool(zd.value))


def parse_eq_file(path):
    """read_graph.py:75-92 parse: header, names, eq lines; int() semantics."""
    with open(path, "r") as reader:
        no_of_contigs = int(reader.readline())
        _ = reader.readline()
        contig_hash = {}
        for i in range(no_of_contigs):
            contig_hash[str(i)] = reader.readline().rstrip("\n")
        eq_classes = [line.rstrip("\n") for line in reader.readlines()]
    names = list(contig_hash.values())
    if len(set(names)) != no_of_contigs:  # read_graph.py:93
        raise AssertionError()
    off = [0]
    mem, mult, skip = [], [], []
    for line in eq_classes:
        eq_size, *ids, count = line.split("\t")
        count = int(count)
        for cid in ids:
            contig_hash[cid]  # KeyError like read_graph.py:91
            mem.append(int(cid))
        off.append(len(mem))
        mult.append(count)
        skip.append(1 if eq_size == "1" else 0)
    return names, np.array(off, np.int64), np.array(mem, np.uint32), np.array(mult, np.int64), np.array(skip, np.uint8)


def graph_from_eq_file(path, fasta_keys):
    """ReadGraph.from_equivalence_classes (read_graph.py:61-148) -> nx.Graph."""
    import networkx as nx

    names, off, mem, mult, skip = parse_eq_file(path)
    r = graph_groups(off, mem, mult, skip, len(names), dedup=False)
    if r["zero_div"]:
        raise ZeroDivisionError("division by zero")
    # intermediate graph yields edge (u, v) from the lower node u in first-insertion order
    order = np.lexsort((r["first"], r["a"]))
    wg = nx.Graph()
    wg.add_nodes_from(names)
    for i in order:
        wg.add_edge(names[r["a"][i]], names[r["b"][i]], weight=float(r["weight"][i]))
    original = set([k.lstrip(">") for k in fasta_keys])
    for missing in original.difference(set(wg.nodes())):
        wg.add_node(missing)
    if len(wg.nodes()) != len(fasta_keys):
        raise AssertionError("The read graph has not enough nodes.")
    return nx.Graph(wg)


def readsets_to_ids(readsets):
    """QNAME strings -> dense ids; per-contig sorted unique arrays (CSR)."""
    ids = {}
    off = [0]
    flat = []
    for rs in readsets:
        cur = sorted({ids.setdefault(q, len(ids)) for q in rs})
        flat += cur
        off.append(len(flat))
    return np.array(off, np.int64), np.array(flat or [0], np.uint32)


def graph_from_readsets(names, readsets):
    """ReadGraph.from_contigs (read_graph.py:19-50) -> nx.Graph (direct O(N^2))."""
    import networkx as nx

    off, flat = readsets_to_ids(readsets)
    N = len(names)
    cap = max(16, N * 4)
    L = lib()
    while True:
        ea, eb = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
        es, ew = np.zeros(cap, np.int64), np.zeros(cap, np.float64)
        E = L.oracle_readset_pairs(_p(off, _i64p), _p(flat, _u32p), N, _p(ea, _u32p), _p(eb, _u32p),
                                   _p(es, _i64p), _p(ew, _f64p), cap)
        if E >= 0:
            break
        cap = -E
    g = nx.Graph()
    if N >= 2:  # every name appears in the first row of combinations
        g.add_nodes_from(names)
    for i in range(E):
        g.add_edge(names[ea[i]], names[eb[i]], weight=float(ew[i]))
    return nx.Graph(g)


def update_graph(graph, orig_names, orig_sets, new_names, new_sets):
    """ReadGraph.update_graph (read_graph.py:192-221) applied to nx graph `graph`."""
    all_off, all_flat = readsets_to_ids(list(orig_sets) + list(new_sets))
    no = len(orig_names)
    o_off = all_off[: no + 1].copy()
    n_off = all_off[no:] - all_off[no]
    o_ids = all_flat[: max(int(o_off[-1]), 1)].copy() if o_off[-1] else np.zeros(1, np.uint32)
    n_ids = all_flat[int(all_off[no]):].copy() if n_off[-1] else np.zeros(1, np.uint32)
    nn = len(new_names)
    cap = max(16, no * nn)
    ea, eb = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    es, ew = np.zeros(cap, np.int64), np.zeros(cap, np.float64)
    E = lib().oracle_update_pairs(_p(o_off, _i64p), _p(o_ids, _u32p), no, _p(np.ascontiguousarray(n_off), _i64p),
                                  _p(n_ids, _u32p), nn, _p(ea, _u32p), _p(eb, _u32p), _p(es, _i64p), _p(ew, _f64p),
                                  cap)
    if no == 0:
        return graph
    by_o = {}
    for i in range(E):
        by_o.setdefault(int(ea[i]), []).append((int(eb[i]), float(ew[i])))
    row0 = dict(by_o.get(0, []))
    for j, nm in enumerate(new_names):  # first product row touches every new contig
        if j in row0:
            graph.add_edge(orig_names[0], nm, weight=row0[j])
        else:
            graph.add_node(nm)
    for oi in range(1, no):
        for j, w in by_o.get(oi, []):
            graph.add_edge(orig_names[oi], new_names[j], weight=w)
    return graph


def graph_dump(g):
    return {"nodes": [str(n) for n in g.nodes()],
            "edges": [[str(a), str(b), float(d["weight"])] for a, b, d in g.edges(data=True)]}


def sequences_from_pairs(pairs):
    return OrderedDict(pairs)


def read_fasta_file(path):
    """read_fasta_file (karma/karma.py:40-61): text-mode line loop, key =
    header.rstrip("\\n").split(" ")[0], sequence = concatenated stripped lines,
    OrderedDict assignment for repeated keys."""
    sequences = OrderedDict()
    with open(path, "r", encoding="utf-8") as reader:
        name = reader.readline().rstrip("\n").split(" ")[0]
        seq = ""
        for line in reader:
            if line.startswith(">"):
                sequences[name] = seq
                name = line.rstrip("\n").split(" ")[0]
                seq = ""
            else:
                seq += line.rstrip("\n")
        sequences[name] = seq
    return sequences


def sam_groups(text, skip_headers=True):
    """SAM text -> [(RNAME, set(QNAME))] in order of first RNAME appearance:
    contig.py:29-35's readset per RNAME group (universal newlines, hisat2.py:49-53
    header filter)."""
    import io

    groups = OrderedDict()
    for line in io.StringIO(text, newline=None):  # text-mode line iteration
        if skip_headers and line.startswith("@"):
            continue
        read, _, name, position, *_ = line.split("\t")
        groups.setdefault(name, set()).add(read)
    return list(groups.items())


# ---------------------------------------------------------------------------
# OpenMP twins: the on-node CPU baseline (bench.py cpu_baseline, SURVEY.md
# §8(d)(2)).  Same results as the scalar functions (tests/test_oracle_golden.py).
# ---------------------------------------------------------------------------

def threads() -> int:
    """OpenMP threads the twins use (OMP_NUM_THREADS, else all host cores)."""
    return int(lib().oracle_threads())


def omp_kmer_profile_packed(blob, offs, key_len, kmer_size, raw_keys, M):
    """Dense profile of packed sequences against a column table from kmer_columns."""
    N = len(offs) - 1
    key_len = np.ascontiguousarray(key_len, np.int64)
    prof = np.empty((N, M), dtype=np.float64)
    rc = lib().oracle_omp_kmer_profile(_p(blob, ctypes.c_void_p), _p(np.ascontiguousarray(offs, np.int64), _i64p),
                                       _p(key_len, _i64p), N, kmode_of(kmer_size), _p(raw_keys, ctypes.c_void_p), M,
                                       _p(prof, _f64p))
    if rc == 1:
        raise AssertionError("oracle: k-mer missing from column set")
    if rc == 2:
        raise ZeroDivisionError("division by zero")
    return prof


def omp_graph_reads(grp_off, members, n_nodes):
    """graph_groups(..., mult=None, pair_skip=None, dedup=True) on all host cores
    (no first-emission positions)."""
    grp_off = np.ascontiguousarray(grp_off, dtype=np.int64)
    members = np.ascontiguousarray(members, dtype=np.uint32)
    totals = np.zeros(max(n_nodes, 1), dtype=np.int64)
    cap = max(1024, len(grp_off))
    L = lib()
    while True:
        ea = np.zeros(cap, np.uint32)
        eb = np.zeros(cap, np.uint32)
        es = np.zeros(cap, np.int64)
        ew = np.zeros(cap, np.float64)
        zd = ctypes.c_int(0)
        E = L.oracle_omp_graph_reads(_p(grp_off, _i64p), _p(members if len(members) else np.zeros(1, np.uint32), _u32p),
                                     len(grp_off) - 1, n_nodes, _p(totals, _i64p), _p(ea, _u32p), _p(eb, _u32p),
                                     _p(es, _i64p), _p(ew, _f64p), cap, ctypes.byref(zd))
        if E >= 0:
            break
        cap = -E
    return dict(a=ea[:E], b=eb[:E], shared=es[:E], weight=ew[:E], totals=totals[:n_nodes], zero_div=bool(zd.value))


def calc_connections(a, b, w, sub, rank, weight_cutoff=0):
    """karma.py:103-118 (calc_connections_between_mcl_subclusters) restated for
    large graphs: instead of walking product(nodes_A, nodes_B) with has_edge for
    every pair of subclusters (O(N^2)), every edge (a, b, w) between two
    subclusters is placed at its position in that walk -- pair (i, j), i < j the
    subcluster indices in dict order, then (rank of the i-side node in nodes_A,
    rank of the j-side node in nodes_B) -- and each pair's running sum is
    accumulated left to right from 0 in Python floats, counting the edges after
    which it exceeds the cutoff (the reference appends [A, B] once per such
    edge).  sub[node] = subcluster index or -1, rank[node] = position in its
    subcluster.  Returns a list of (i, j, count) in combinations order."""
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    sa, sb = np.asarray(sub)[a], np.asarray(sub)[b]
    keep = (sa >= 0) & (sb >= 0) & (sa != sb)
    a, b, w, sa, sb = a[keep], b[keep], np.asarray(w, np.float64)[keep], sa[keep], sb[keep]
    lo_is_a = sa < sb
    i = np.where(lo_is_a, sa, sb)
    j = np.where(lo_is_a, sb, sa)
    ri = np.where(lo_is_a, np.asarray(rank)[a], np.asarray(rank)[b])
    rj = np.where(lo_is_a, np.asarray(rank)[b], np.asarray(rank)[a])
    o = np.lexsort((rj, ri, j, i))
    out = []
    cur, weight, over = None, 0, 0
    for x, y, wt in zip(i[o].tolist(), j[o].tolist(), w[o].tolist()):
        if (x, y) != cur:
            if cur is not None and over:
                out.append((cur[0], cur[1], over))
            cur, weight, over = (x, y), 0, 0
        weight += wt
        if weight > weight_cutoff:
            over += 1
    if cur is not None and over:
        out.append((cur[0], cur[1], over))
    return out
