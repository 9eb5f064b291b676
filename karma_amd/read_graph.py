"""Shared-read contig graph — drop-in for karma/read_graph.py:10-467.

Graph construction (the hot path) runs on the MI355X through libkarma_hip.so:
  from_contigs / update_graph  -> (read, contig) records -> per-read pair
                                  emission, bucket partition, LDS hash reduce
  from_equivalence_classes     -> eq-class pair emission + sort/reduce
The resulting networkx graph has the reference's nodes, edges, weights (bit
for bit) and insertion order (tests/test_gpu_parity.py compares
G.edges(data=True) lists with the reference's own output).

The consumers karma.py runs on cluster graphs -- get_unconnected_nodes /
get_connected_nodes, the node weights behind calculate_representative_sequences
and edge_list (MCL's input) -- run on the device too (consumers.py,
csrc/consumers.hip): a graph keeps a device mirror of its networkx layout (node
order, adjacency-dict order, weights).  The constructors and
ReadGraph(G.subgraph(...)) copies of a mirrored graph get one without a Python
walk; node removals are applied to it; any other mutation drops it and the next
consumer call exports the graph's dicts (in-place edits of edge attribute dicts
are not seen: change weights through add_edge).
"""

import itertools
import logging
import os

import networkx as nx
import numpy as np

from . import consumers, engine, ingest
from ._lib import KARMA_ERR_ZERO_DIV, KarmaError
from .contig import contig_records, load_sam_records
from .logs import logger


def _edges_or_zero_div(fn, *args, **kw):
    try:
        return fn(*args, **kw)
    except KarmaError as e:
        if e.code == KARMA_ERR_ZERO_DIV:
            raise ZeroDivisionError("division by zero") from e
        raise


def parse_eq_classes(equivalence_class_file, threads=0):
    """Parse salmon eq_classes.txt exactly as read_graph.py:75-92 does, with the
    C++ parser (csrc/ingest.cpp, karma_eq_parse).  A file it declines goes
    through the reference's own reading (_parse_eq_text), which raises the
    reference's exception or, for exotic-but-valid text, returns its result.

    Returns (names, cls_off int64[C+1], members uint32, counts int64, pair_skip uint8)."""
    try:
        q = ingest.parse_eq(ingest._read(equivalence_class_file), threads)
    except ingest.ParseDeferred:
        return _parse_eq_text(equivalence_class_file)
    return q.names, q.cls_off, q.members, q.counts, q.pair_skip


def _parse_eq_text(equivalence_class_file):
    """read_graph.py:75-92 line by line (int(), str keys, the :93 assert)."""
    with open(equivalence_class_file, "r") as reader:
        no_of_contigs = int(reader.readline())
        _ = reader.readline()
        contig_hash = {}
        for i in range(no_of_contigs):
            contig_hash[str(i)] = reader.readline().rstrip("\n")
        eq_lines = [line.rstrip("\n") for line in reader.readlines()]
    assert no_of_contigs == len(contig_hash)
    names = list(contig_hash.values())
    # read_graph.py:86 keys the totals by NAME: duplicated names collapse and
    # the assert at :93 fails
    assert no_of_contigs == len(set(names))
    index = {str(i): i for i in range(no_of_contigs)}
    off = np.zeros(len(eq_lines) + 1, np.int64)
    counts = np.zeros(len(eq_lines), np.int64)
    skip = np.zeros(len(eq_lines), np.uint8)
    members = []
    for c, line in enumerate(eq_lines):
        eq_size, *contig_ids, count = line.split("\t")
        counts[c] = int(count)
        for cid in contig_ids:
            if cid not in index:
                raise KeyError(cid)  # contig_hash[contig_id], read_graph.py:91
            members.append(index[cid])
        off[c + 1] = len(members)
        skip[c] = 1 if eq_size == "1" else 0  # read_graph.py:102 compares the TOKEN
    return names, off, np.array(members, np.uint32), counts, skip


def _copied_graph(cls, nodes, a, b, w):
    """cls(incoming_graph_data=G) for the graph G the reference builds:
        G = nx.Graph(); G.add_nodes_from(nodes)
        for i: G.add_edge(nodes[a[i]], nodes[b[i]], weight=w[i])
    built directly, without G.  nodes must be distinct and (a[i], b[i]) pairs
    unique.  The copy is networkx's from_dict_of_dicts(G.adj): nodes in G's
    order, then add_edges_from over (u, v) for u in G, v in G.adj[u].  So the
    copy's adj[u] holds first the neighbours v placed before u (met while
    walking v's list), by position, then the rest in G.adj[u] order, which is
    add_edge order.  Every edge gets its own {"weight": w} dict, shared by both
    directions, and every node an empty attribute dict, as in the copy."""
    import gc

    enabled = gc.isenabled()
    gc.disable()  # ~2 x 200k new dicts: collector passes would cost ~30 %
    try:
        return _copied_graph_body(cls, nodes, a, b, w)
    finally:
        if enabled:
            gc.enable()


def _copied_graph_body(cls, nodes, a, b, w):
    n = len(nodes)
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    nm = np.empty(n, dtype=object)
    nm[:] = nodes
    adj = {x: {} for x in nodes}
    dds = [{"weight": x} for x in np.asarray(w).tolist()]
    # neighbours placed before u: per u, by position
    o = np.lexsort((lo, hi))
    o = o[lo[o] < hi[o]]
    for u, v, i in zip(nm[hi[o]].tolist(), nm[lo[o]].tolist(), o.tolist()):
        adj[u][v] = dds[i]
    # the rest (and self-loops), in add_edge order
    for u, v, d in zip(nm[lo].tolist(), nm[hi].tolist(), dds):
        adj[u][v] = d
    out = cls()
    out._node = {x: {} for x in nodes}
    out._adj = adj
    return out


def _invalidating(name):
    base = getattr(nx.Graph, name)

    def method(self, *args, **kw):
        self._mirror = None
        self._mirror_spec = None
        self._view_root = None
        self._summary = None
        return base(self, *args, **kw)

    method.__name__ = name
    method.__doc__ = base.__doc__
    return method


def _removing(name):
    base = getattr(nx.Graph, name)

    def method(self, *args, **kw):
        self._mirror_dirty = True
        return base(self, *args, **kw)

    method.__name__ = name
    method.__doc__ = base.__doc__
    return method


class ReadGraph(nx.Graph):
    """Read graph to find clusters (read_graph.py:10)."""

    def __init__(self, incoming_graph_data=None, **attr):
        super().__init__(incoming_graph_data, **attr)
        self.original_contigs = []
        self.mcl_cluster = []
        self._mirror = None        # consumers.Mirror of this graph's layout
        self._mirror_spec = None   # or how to build it on first use
        self._mirror_dirty = False  # nodes removed since the mirror was taken
        self._view_root = None      # mirror this graph is a (node-removed) view copy of
        self._summary = None        # one-launch consumer results of a small view copy
        src = incoming_graph_data
        # nx.Graph(G.subgraph(nodes)) / nx.Graph(G) of a mirrored ReadGraph: the
        # copy's layout is derived from G's on the device
        if isinstance(src, ReadGraph):
            base = src
            if hasattr(src, "_NODE_OK"):
                base = getattr(src, "_graph", None)
                if getattr(src, "_EDGE_OK", None) is not nx.filters.no_filter:
                    base = None
            if isinstance(base, ReadGraph) and (base._mirror is not None or base._mirror_spec is not None):
                root = base._device_mirror()
                self._mirror_spec = ("view", root, list(self))
                self._view_root = root

    for _name in ("add_node", "add_nodes_from", "add_edge", "add_edges_from", "add_weighted_edges_from",
                  "remove_edge", "remove_edges_from", "update", "clear", "clear_edges"):
        locals()[_name] = _invalidating(_name)
    for _name in ("remove_node", "remove_nodes_from"):
        locals()[_name] = _removing(_name)
    del _name

    def _device_mirror(self) -> consumers.Mirror:
        """The device mirror of this graph's current layout (built, synced or exported)."""
        m = self._mirror
        if m is None:
            spec = self._mirror_spec
            if spec is None:
                m = consumers.export(self)
            elif spec[0] == "edges":
                _, nodes, a, b, w = spec
                adj = consumers.DeviceAdj.from_edges(len(nodes), a, b, w)
                # cls(incoming_graph_data=graph) rebuilt the adjacency (from_dict_of_dicts)
                rebuilt = adj.view(np.arange(len(nodes), dtype=np.int64))
                m = consumers.Mirror(rebuilt, consumers.NameTable(nodes), nodes)
            else:  # ("view", base mirror, node order)
                m = spec[1].view(spec[2])
            self._mirror, self._mirror_spec = m, None
            self._mirror_dirty = False
        if self._mirror_dirty:
            cur = list(self)
            synced = m.sync(cur)
            m = synced if synced is not None else consumers.export(self)
            self._mirror, self._mirror_dirty = m, False
        return m

    # ------------------------------------------------------------ build ----
    @classmethod
    def from_contigs(cls, contigs: list) -> "ReadGraph":
        """read_graph.py:19-50: every pair of contigs sharing reads becomes an
        edge with weight (s/|A| + s/|B|) / 2; computed on the GPU from the
        (read, contig) incidence instead of the O(N^2) pair loop."""
        logger.debug("Initial graph calculation.")
        n = len(contigs)
        if n < 2:
            return cls(incoming_graph_data=nx.Graph())
        rec, _ = contig_records(contigs)
        e = _edges_or_zero_div(engine.graph_from_records, rec, n, grouped=False)
        names = [c.name for c in contigs]
        # combinations order: row 0 touches every contig, so nodes appear
        # in list order; edges are added in (i, j) order = sorted order
        return cls._from_edge_list(names, e.a, e.b, e.weight)

    @classmethod
    def _from_edge_list(cls, names, a, b, w):
        """The reference's add_nodes_from(names) + add_edge loop + cls(...) copy."""
        if len(set(names)) == len(names):  # distinct names: positions = list indices
            out = _copied_graph(cls, names, a, b, w)
            out._mirror_spec = ("edges", list(names), a, b, np.asarray(w, np.float64))
            return out
        graph = nx.Graph()
        graph.add_nodes_from(names)
        for x, y, wt in zip(np.asarray(a).tolist(), np.asarray(b).tolist(), np.asarray(w).tolist()):
            graph.add_edge(names[x], names[y], weight=wt)
        return cls(incoming_graph_data=graph)

    @classmethod
    def from_sam(cls, sam, skip_headers: bool = True, threads: int = 0) -> "ReadGraph":
        """from_contigs over the contigs of SAM lines (contig.py:24,34 readsets,
        grouped by RNAME in order of first appearance) without building Python
        readsets: the C++ reader's (read, contig) records go straight to the GPU."""
        rec, _ = load_sam_records(sam, skip_headers, threads)
        names = rec.rnames
        if len(names) < 2:
            return cls(incoming_graph_data=nx.Graph())
        e = _edges_or_zero_div(engine.graph_from_records, rec.records, len(names), grouped=False)
        return cls._from_edge_list(list(names), e.a, e.b, e.weight)

    def set_original_contigs(self, original_contigs: list) -> None:
        self.original_contigs = original_contigs

    @classmethod
    def from_equivalence_classes(cls, equivalence_class_file: str, sequences_from_fasta: dict) -> "ReadGraph":
        """read_graph.py:61-148 with the pair sums and weights on the GPU."""
        try:
            # the compact form (1 + 4 bytes per class instead of 17 over PCIe)
            # when every class fits it, straight from the C++ parser
            q = ingest.parse_eq(ingest._read(equivalence_class_file), 0, compact=True)
        except ingest.ParseDeferred:
            names, off, members, counts, skip = _parse_eq_text(equivalence_class_file)
            return cls._from_eq_arrays(names, off, members, counts, skip, sequences_from_fasta)
        if q.sizes is not None:
            return cls._from_eq_arrays(q.names, None, q.members, None, None, sequences_from_fasta,
                                       compact=(q.sizes, q.counts32))
        return cls._from_eq_arrays(q.names, q.cls_off, q.members, q.counts, q.pair_skip, sequences_from_fasta)

    @classmethod
    def _from_eq_arrays(cls, names, off, members, counts, skip, sequences_from_fasta, compact=None):
        """from_equivalence_classes after the parse (read_graph.py:86-148): eq
        names, class offsets/members/counts and the size-token-"1" flags (or
        compact = (sizes, counts32), karma_graph_eq_compact's form)."""
        n = len(names)
        ea = eb = np.zeros(0, np.uint32)
        ew = np.zeros(0, np.float64)
        if n:
            # the reference's intermediate graph (read_graph.py:96-131) gets edge
            # (u, v) from its lower-index endpoint u, in first-insertion order:
            # that order comes from the device
            if compact is not None:
                ea, eb, ew = _edges_or_zero_div(engine.graph_from_eq_compact_ordered, compact[0], members, compact[1],
                                                n)
            else:
                ea, eb, ew = _edges_or_zero_div(engine.graph_from_eq_ordered, off, members, counts, skip, n)
        # read_graph.py:136-143: FASTA names missing from the eq file become
        # isolated nodes, in the order of this set difference (hash seed
        # dependent, as in the reference); eq names are distinct (:93 assert)
        eq_names = set(names)
        original_sequence_names = set([name.lstrip(">") for name in sequences_from_fasta.keys()])
        nodes = list(names) + list(original_sequence_names.difference(eq_names))
        assert len(nodes) == len(sequences_from_fasta), (
            "The read graph has not enough nodes. Maybe Salmon could couldn't add all contigs to a equivalence class")
        # cls(incoming_graph_data=weighted_graph) (read_graph.py:148), built
        # directly in the layout that copy has
        out = _copied_graph(cls, nodes, ea, eb, ew)
        out._mirror_spec = ("edges", nodes, ea, eb, np.asarray(ew, np.float64))
        return out

    def update_graph(self, contigs: list) -> None:
        """read_graph.py:192-221: weights between every (original, new) pair,
        computed on the GPU as the cross block of one records pass."""
        logger.debug("Updating graph.")
        orig = list(self.original_contigs)
        no, nn = len(orig), len(contigs)
        if no == 0:
            return
        ids = {}
        r1, ids = contig_records(orig, 0, ids)
        r2, ids = contig_records(contigs, no, ids)
        rec = np.concatenate([r1, r2]) if len(r1) + len(r2) else np.zeros((0, 2), np.uint32)
        e = _edges_or_zero_div(engine.graph_from_records, rec, no + nn, grouped=False)
        cross = (e.a < no) & (e.b >= no)
        oa, nb, w = e.a[cross].tolist(), (e.b[cross] - no).tolist(), e.weight[cross].tolist()
        i = 0
        # product row 0 visits every new contig: edge or add_node, in order
        row0 = {}
        while i < len(oa) and oa[i] == 0:
            row0[nb[i]] = w[i]
            i += 1
        first = orig[0].name
        for j, c in enumerate(contigs):
            if j in row0:
                self.add_edge(first, c.name, weight=row0[j])
            else:
                self.add_node(c.name)
        for o, j, wt in zip(oa[i:], nb[i:], w[i:]):
            self.add_edge(orig[o].name, contigs[j].name, weight=wt)

    # ---------------------------------------------------------- queries ----
    def _small_view(self):
        """(nodes, degrees, node weights, edge_list bytes or None) of a small view
        copy (<= 1024 nodes) from one device launch (karma_adj_view_summary), or
        None: not a view copy, too large, or mutated other than by removals.
        A view copy with nodes removed is the view of the remaining nodes in the
        same order (removal keeps both adjacency orders), so the summary is
        recomputed from the root mirror; removing only nodes without edges leaves
        every other result as it was, and the cached one is filtered instead."""
        root = self._view_root
        n = len(self)
        if root is None or n > consumers.SMALL_VIEW:
            return None
        c = self._summary
        if c is not None:
            if c[0] == n:  # removals only: an unchanged count is an unchanged node set
                return c[1:]
            alive = self._node
            mask = np.fromiter((x in alive for x in c[1]), bool, len(c[1]))
            if not c[2][~mask].any():
                c = (n, [x for x, k in zip(c[1], mask) if k], c[2][mask], c[3][mask], c[4])
                self._summary = c
                return c[1:]
        nodes = list(self)
        pos = root.pos()
        order = np.fromiter((pos[x] for x in nodes), np.int64, n)
        # the text comes in the same launch: karma.py asks for it next (:318)
        r = root.adj.view_summary(order, root.names, True)
        if r is None:
            return None
        self._summary = (n, nodes) + r
        return self._summary[1:]

    def get_unconnected_nodes(self) -> list:
        """Nodes without any neighbour, in node order (read_graph.py:150-160); degrees on the device."""
        s = self._small_view()
        if s is not None:
            return [s[0][i] for i in np.flatnonzero(s[1] == 0).tolist()]
        m = self._device_mirror()
        deg = m.adj.degrees()
        return [m.nodes[i] for i in np.flatnonzero(deg == 0).tolist()]

    def get_connected_nodes(self) -> list:
        """Nodes with at least one neighbour (read_graph.py:162-172); degrees on the device."""
        s = self._small_view()
        if s is not None:
            return [s[0][i] for i in np.flatnonzero(s[1] != 0).tolist()]
        m = self._device_mirror()
        deg = m.adj.degrees()
        return [m.nodes[i] for i in np.flatnonzero(deg != 0).tolist()]

    def __calculate_node_weights(self) -> dict:
        """Sum of incident edge weights in adjacency order (read_graph.py:174-190):
        0 + w_1 + w_2 + ... in f64 on the device; a node without edges keeps the int 0."""
        s = self._small_view()
        if s is not None:
            nodes, deg, w = s[0], s[1], s[2]
        else:
            m = self._device_mirror()
            nodes = m.nodes
            deg, w = m.adj.node_stats()
        w = w.tolist()
        for i in np.flatnonzero(deg == 0).tolist():
            w[i] = 0
        weights = dict(zip(nodes, w))
        if logger.isEnabledFor(logging.DEBUG):
            logger.debug(f"Node weights: {weights}")
        return weights

    def save_graph(self, filename: str) -> None:
        """abc file with explicit zero edges (read_graph.py:223-240)."""
        graph = nx.Graph(self)
        for a, b in itertools.combinations(self.nodes, 2):
            if not graph.has_edge(a, b):
                graph.add_edge(a, b, weight=0)
        if os.path.isfile(filename):
            os.remove(filename)
        nx.write_weighted_edgelist(graph, filename)

    def _split_mcl_lines(self, lines, original_contigs):
        if original_contigs is None:
            original_cluster = set(c.name for c in self.original_contigs)
        else:
            original_cluster = set(original_contigs)
        leftovers = []
        for line in lines:
            group = set(line.rstrip("\n").split("\t"))
            if original_cluster.intersection(group):
                self.mcl_cluster.append(list(group))
            else:
                leftovers += list(group)
        return leftovers, original_cluster

    def get_contigs_not_in_mcl_cluster(self, mcl_cluster_file, original_contigs=None):
        """read_graph.py:242-277."""
        with open(mcl_cluster_file, "r") as fh:
            leftovers, original_cluster = self._split_mcl_lines(fh, original_contigs)
        if len(self.mcl_cluster) == 0:
            logger.debug("MCL CLUSTER IS EMPTY")
            self.mcl_cluster = [[seq] for seq in original_cluster]
        return leftovers

    def get_contigs_not_in_mcl_cluster_stdout(self, stdout, original_contigs=None):
        """read_graph.py:279-313."""
        leftovers, _ = self._split_mcl_lines(stdout.split("\n")[:-1], original_contigs)
        return leftovers

    def calculate_representative_sequences(self, lowest: bool = False) -> list:
        """Highest (and optionally lowest) node-weight member per MCL cluster
        (read_graph.py:315-344; first maximum wins like max())."""
        node_weights = self.__calculate_node_weights()
        reps = []
        for cluster in self.mcl_cluster:
            sub = {k: node_weights[k] for k in cluster}
            reps.append(f">{max(sub, key=sub.get)}")
            if lowest:
                reps.append(f">{min(sub, key=sub.get)}")
        return reps

    def nodes_list(self) -> list:
        return list(self.nodes())

    def edge_list(self) -> str:
        """MCL stdin text "A B w" per edge, UTF-8 (read_graph.py:350-357): names and
        repr(weight) written on the device, edges in G.edges() order."""
        s = self._small_view()
        if s is not None:
            return s[3]
        m = self._device_mirror()
        return m.adj.edge_list(m.names)

    def calc_distance_between_subgraphs(self, nodes_a: list, nodes_b: list) -> int:
        """Sum of weights between two node sets (read_graph.py:359-373)."""
        total = 0
        for a, b in itertools.product(nodes_a, nodes_b):
            if self.has_edge(a, b):
                total += self[a][b]["weight"]
        return total
