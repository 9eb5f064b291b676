"""Read-graph consumers on the device.

karma.py:255-395 takes ReadGraph(full_graph.subgraph(cluster)), trims its
unconnected nodes (read_graph.py:150-160), pipes edge_list() to MCL
(read_graph.py:350-357) and picks representatives by node weight
(read_graph.py:174-190, :315-344).  Each of these is a function of how
networkx iterates the graph: node order, and per node the adjacency-dict order
of its neighbours.  `DeviceAdj` holds that layout on the MI355X
(csrc/consumers.hip) and computes degrees, node weights (f64, left to right in
adjacency order) and the edge_list bytes (names + Python repr(float) on the
device) bit for bit as the reference does.

`Mirror` ties a DeviceAdj to a networkx graph: the node objects by position and
the UTF-8 name table.  ReadGraph keeps one for the graphs its constructors
build and for nx.Graph(G.subgraph(...)) copies of them; node removals are
applied to the mirror, any other mutation drops it, and a graph without a
mirror is exported from its networkx dicts (Python walk) before the device
computes.
"""

from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import call, ptr


class NameTable:
    """UTF-8 names (str(node), as an f-string prints it) by id, resident on the device."""

    def __init__(self, nodes, ctx=None):
        self.ctx = ctx or _lib.default_context()
        enc = [str(n).encode("utf-8") for n in nodes]  # UnicodeEncodeError like edge_list's .encode()
        self.off = np.zeros(len(enc) + 1, np.int64)
        if enc:
            np.cumsum([len(e) for e in enc], out=self.off[1:])
        self.blob = np.frombuffer(b"".join(enc), np.uint8) if enc else np.zeros(0, np.uint8)
        self.n = len(enc)
        self._dev = None

    def device(self):
        """(names_ptr, off_ptr) of device copies, uploaded once."""
        if self._dev is None:
            lib = _lib.load()
            ps = []
            for a in (self.blob, self.off):
                nbytes = max(1, a.nbytes)
                p = ctypes.c_void_p()
                call("karma_dev_alloc", self.ctx.h, nbytes, ctypes.byref(p))
                ps.append(p)
                if a.nbytes:
                    call("karma_memcpy", self.ctx.h, p, ptr(a), a.nbytes, 0)
            self._dev = (ps[0], ps[1], lib)
        return self._dev[0], self._dev[1]

    def __del__(self):
        d = getattr(self, "_dev", None)
        if d is not None and getattr(self.ctx, "h", None):
            for p in d[:2]:
                d[2].karma_dev_free(self.ctx.h, p)
            self._dev = None


SMALL_VIEW = 1024  # nodes of a view copy served by one launch (karma_adj_view_summary)
_TEXT_BUF = np.empty(1 << 20, np.uint8)  # edge_list bytes of one-launch view summaries
# karma_adj_view_summary uses the context's one mapped host buffer (order,
# status word, results) and _TEXT_BUF: one call at a time per process, so that
# graphs on several threads (a ShardedBuild pool, a caller's workers) cannot
# overwrite each other's inputs or results
_SUMMARY_LOCK = threading.Lock()


class DeviceAdj:
    """A karma_adj: graph layout in networkx iteration order on the device."""

    def __init__(self, ctx, h, n):
        self.ctx, self.h, self.n = ctx, h, n

    @property
    def m(self):
        """Adjacency entries (reads the device-side count)."""
        m = _lib._i64(0)
        call("karma_adj_info", self.h, None, ctypes.byref(m))
        return m.value

    @classmethod
    def from_edges(cls, n, a, b, w, ids=None, ctx=None):
        """add_edge(a[e], b[e], weight=w[e]) in order on n pre-added nodes."""
        ctx = ctx or _lib.default_context()
        a = np.ascontiguousarray(a, np.uint32)
        b = np.ascontiguousarray(b, np.uint32)
        w = np.ascontiguousarray(w, np.float64)
        ids = None if ids is None else np.ascontiguousarray(ids, np.uint32)
        h = ctypes.c_void_p()
        call("karma_adj_from_edges", ctx.h, n, ptr(ids), ptr(a), ptr(b), ptr(w), len(a), 0, ctypes.byref(h))
        return cls(ctx, h, n)

    @classmethod
    def from_lists(cls, off, nbr, w, ids=None, ctx=None):
        ctx = ctx or _lib.default_context()
        off = np.ascontiguousarray(off, np.int64)
        nbr = np.ascontiguousarray(nbr, np.uint32)
        w = np.ascontiguousarray(w, np.float64)
        ids = None if ids is None else np.ascontiguousarray(ids, np.uint32)
        h = ctypes.c_void_p()
        call("karma_adj_from_lists", ctx.h, len(off) - 1, ptr(ids), ptr(off), ptr(nbr), ptr(w), 0, ctypes.byref(h))
        return cls(ctx, h, len(off) - 1)

    def view(self, order):
        """nx.Graph(G.subgraph(nodes)): order = positions in the view's node order."""
        order = np.ascontiguousarray(order, np.int64)
        h = ctypes.c_void_p()
        if len(order) and (order.min() < 0 or order.max() >= self.n or len(np.unique(order)) != len(order)):
            raise ValueError("view order: positions must be distinct and in range")
        call("karma_adj_view", self.h, ptr(order), len(order), ctypes.byref(h))
        return DeviceAdj(self.ctx, h, len(order))

    def view_summary(self, order, names: "NameTable", with_text: bool):
        """Degrees, node weights and (with_text) the edge_list bytes of
        nx.Graph(G.subgraph(nodes at `order`)) in one launch; None when the view
        is over the one-block limits (karma_adj_view_summary)."""
        order = np.ascontiguousarray(order, np.int64)
        k = len(order)
        deg = np.empty(k, np.int64)
        w = np.empty(k, np.float64)
        done = ctypes.c_int(0)
        tl = _lib._i64(0)
        dn, do = names.device() if with_text else (None, None)
        with _SUMMARY_LOCK:
            call("karma_adj_view_summary", self.h, ptr(order), k, dn, do, 1 if with_text else 0, ptr(deg), ptr(w),
                 ptr(_TEXT_BUF) if with_text else None, len(_TEXT_BUF), ctypes.byref(tl), ctypes.byref(done))
            if not done.value:
                return None
            return deg, w, (_TEXT_BUF[:tl.value].tobytes() if with_text else None)

    def keep(self, mask):
        """G.remove_nodes_from(nodes at positions where mask == 0)."""
        mask = np.ascontiguousarray(mask, np.uint8)
        k = int(np.count_nonzero(mask))
        h = ctypes.c_void_p()
        call("karma_adj_keep", self.h, ptr(mask), k, ctypes.byref(h))
        return DeviceAdj(self.ctx, h, k)

    def layout(self):
        m = self.m
        ids = np.zeros(self.n, np.uint32)
        off = np.zeros(self.n + 1, np.int64)
        nbr = np.zeros(m, np.uint32)
        w = np.zeros(m, np.float64)
        call("karma_adj_get", self.h, ptr(ids), ptr(off), ptr(nbr), ptr(w))
        return ids, off, nbr, w

    def degrees(self):
        d = np.zeros(self.n, np.int64)
        call("karma_adj_degrees", self.h, ptr(d))
        return d

    def node_weights(self):
        out = np.zeros(self.n, np.float64)
        call("karma_adj_node_weights", self.h, ptr(out))
        return out

    def node_stats(self):
        """(degrees, node weights) in one device pass."""
        d = np.zeros(self.n, np.int64)
        w = np.zeros(self.n, np.float64)
        call("karma_adj_node_stats", self.h, ptr(d), ptr(w))
        return d, w

    def cross_sums(self, sub, rank, cutoff):
        """karma_adj_cross_sums: (A, B, sum, n_edges, n_over) arrays of the
        subcluster pairs joined by edges, sorted by (A, B)."""
        sub = np.ascontiguousarray(sub, np.int32)
        rank = np.ascontiguousarray(rank, np.int32)
        P = _lib._i64(0)
        call("karma_adj_cross_sums", self.h, ptr(sub), ptr(rank), float(cutoff), None, None, None, None, 0,
             ctypes.byref(P))
        p = P.value
        pair = np.zeros(p, np.uint64)
        s = np.zeros(p, np.float64)
        ne = np.zeros(p, np.int64)
        no = np.zeros(p, np.int64)
        if p:
            call("karma_adj_cross_sums", self.h, ptr(sub), ptr(rank), float(cutoff), ptr(pair), ptr(s), ptr(ne),
                 ptr(no), p, ctypes.byref(P))
        return (pair >> np.uint64(32)).astype(np.int64), (pair & np.uint64(0xFFFFFFFF)).astype(np.int64), s, ne, no

    def edge_list(self, names: NameTable) -> bytes:
        dn, do = names.device()
        n = _lib._i64(0)
        call("karma_adj_edge_list", self.h, dn, do, names.n, 1, None, 0, ctypes.byref(n))
        buf = np.zeros(max(1, n.value), np.uint8)
        call("karma_adj_edge_list", self.h, dn, do, names.n, 1, ptr(buf), n.value, ctypes.byref(n))
        return buf[:n.value].tobytes()

    def close(self):
        if getattr(self, "h", None):
            _lib.load().karma_adj_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Mirror:
    """A DeviceAdj for one networkx graph: `nodes` = node objects by position,
    `names` = the name table the adjacency's ids index (shared by views)."""

    def __init__(self, adj: DeviceAdj, names: NameTable, nodes: list, root=None):
        self.adj, self.names, self.nodes = adj, names, nodes
        self.root = root if root is not None else self  # the mirror positions are taken from
        self._pos = None

    def pos(self):
        """node -> position (built once, for views of this graph)."""
        if self._pos is None:
            self._pos = {n: i for i, n in enumerate(self.nodes)}
        return self._pos

    def view(self, nodes: list) -> "Mirror":
        """Mirror of nx.Graph(view) whose node order is `nodes` (a subset of ours)."""
        p = self.pos()
        order = np.fromiter((p[n] for n in nodes), np.int64, len(nodes))
        return Mirror(self.adj.view(order), self.names, list(nodes), root=self.root)

    def sync(self, current_nodes: list) -> "Mirror":
        """Apply node removals: `current_nodes` must be our nodes minus some, in order."""
        if len(current_nodes) == len(self.nodes):
            return self
        alive = set(current_nodes)
        mask = np.fromiter((n in alive for n in self.nodes), np.uint8, len(self.nodes))
        kept = [n for n, k in zip(self.nodes, mask) if k]
        if kept != current_nodes:
            return None
        return Mirror(self.adj.keep(mask), self.names, kept, root=self.root)


def export(G) -> Mirror:
    """Mirror of any networkx graph from its dicts (node order, adjacency order,
    float weights).  KeyError for an edge without 'weight' (as the reference's
    data['weight']); TypeError for a weight that is not a float, whose repr
    and sums the device's f64 path would not reproduce."""
    nodes = list(G)
    pos = {n: i for i, n in enumerate(nodes)}
    off = np.zeros(len(nodes) + 1, np.int64)
    nbr, w = [], []
    adj = G._adj
    for i, u in enumerate(nodes):
        for v, d in adj[u].items():
            x = d["weight"]
            if type(x) is not float and not isinstance(x, np.floating):
                raise TypeError(f"edge ({u!r}, {v!r}) weight {x!r} is not a float")
            nbr.append(pos[v])
            w.append(float(x))
        off[i + 1] = len(nbr)
    adj_dev = DeviceAdj.from_lists(off, np.array(nbr, np.uint32), np.array(w, np.float64))
    return Mirror(adj_dev, NameTable(nodes), nodes)
