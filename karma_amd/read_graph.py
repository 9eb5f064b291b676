"""Shared-read contig graph — drop-in for karma/read_graph.py:10-467.

Graph construction (the hot path) runs on the MI355X through libkarma_hip.so:
  from_contigs / update_graph  -> (read, contig) records -> per-read pair
                                  emission, bucket partition, LDS hash reduce
  from_equivalence_classes     -> eq-class pair emission + sort/reduce
The resulting networkx graph has the reference's nodes, edges, weights (bit
for bit) and insertion order (tests/test_gpu_parity.py compares
G.edges(data=True) lists with the reference's own output).  The query helpers
below are small pure-graph utilities kept for API completeness.
"""

import itertools
import os

import networkx as nx
import numpy as np

from . import engine, ingest
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


class ReadGraph(nx.Graph):
    """Read graph to find clusters (read_graph.py:10)."""

    def __init__(self, incoming_graph_data=None, **attr):
        super().__init__(incoming_graph_data, **attr)
        self.original_contigs = []
        self.mcl_cluster = []

    # ------------------------------------------------------------ build ----
    @classmethod
    def from_contigs(cls, contigs: list) -> "ReadGraph":
        """read_graph.py:19-50: every pair of contigs sharing reads becomes an
        edge with weight (s/|A| + s/|B|) / 2; computed on the GPU from the
        (read, contig) incidence instead of the O(N^2) pair loop."""
        logger.debug("Initial graph calculation.")
        graph = nx.Graph()
        n = len(contigs)
        if n >= 2:
            rec, _ = contig_records(contigs)
            e = _edges_or_zero_div(engine.graph_from_records, rec, n, grouped=False)
            names = [c.name for c in contigs]
            # combinations order: row 0 touches every contig, so nodes appear
            # in list order; edges are added in (i, j) order = sorted order
            graph.add_nodes_from(names)
            for a, b, w in zip(e.a.tolist(), e.b.tolist(), e.weight.tolist()):
                graph.add_edge(names[a], names[b], weight=w)
        return cls(incoming_graph_data=graph)

    @classmethod
    def from_sam(cls, sam, skip_headers: bool = True, threads: int = 0) -> "ReadGraph":
        """from_contigs over the contigs of SAM lines (contig.py:24,34 readsets,
        grouped by RNAME in order of first appearance) without building Python
        readsets: the C++ reader's (read, contig) records go straight to the GPU."""
        rec, _ = load_sam_records(sam, skip_headers, threads)
        graph = nx.Graph()
        names = rec.rnames
        if len(names) >= 2:
            e = _edges_or_zero_div(engine.graph_from_records, rec.records, len(names), grouped=False)
            graph.add_nodes_from(names)
            for a, b, w in zip(e.a.tolist(), e.b.tolist(), e.weight.tolist()):
                graph.add_edge(names[a], names[b], weight=w)
        return cls(incoming_graph_data=graph)

    def set_original_contigs(self, original_contigs: list) -> None:
        self.original_contigs = original_contigs

    @classmethod
    def from_equivalence_classes(cls, equivalence_class_file: str, sequences_from_fasta: dict) -> "ReadGraph":
        """read_graph.py:61-148 with the pair sums and weights on the GPU."""
        names, off, members, counts, skip = parse_eq_classes(equivalence_class_file)
        n = len(names)
        if n == 0:
            e = None
        else:
            e = _edges_or_zero_div(engine.graph_from_eq, off, members, counts, skip, n)
        weighted_graph = nx.Graph()
        weighted_graph.add_nodes_from(names)
        if e is not None and len(e.a):
            # the reference's intermediate graph yields edge (u, v) from its
            # lower-index endpoint u, in first-insertion order (read_graph.py:120)
            order = np.lexsort((e.first, e.a))
            a, b, w = e.a[order].tolist(), e.b[order].tolist(), e.weight[order].tolist()
            for x, y, wt in zip(a, b, w):
                weighted_graph.add_edge(names[x], names[y], weight=wt)
        assert len(weighted_graph.nodes()) == n
        original_sequence_names = set([name.lstrip(">") for name in sequences_from_fasta.keys()])
        for missing_node in original_sequence_names.difference(set(weighted_graph.nodes())):
            weighted_graph.add_node(missing_node)
        assert len(weighted_graph.nodes()) == len(sequences_from_fasta), (
            "The read graph has not enough nodes. Maybe Salmon could couldn't add all contigs to a equivalence class")
        return cls(incoming_graph_data=weighted_graph)

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
    def get_unconnected_nodes(self) -> list:
        """Nodes without any neighbour (read_graph.py:150-160)."""
        return [n for n in self.nodes() if len(self._adj[n]) == 0]

    def get_connected_nodes(self) -> list:
        """Nodes with at least one neighbour (read_graph.py:162-172)."""
        return [n for n in self.nodes() if len(self._adj[n]) != 0]

    def __calculate_node_weights(self) -> dict:
        """Sum of incident edge weights in adjacency order (read_graph.py:174-190)."""
        weights = {}
        for node in self.nodes():
            total = 0
            for _, _, d in self.edges(node, data=True):
                total += d["weight"]
            weights[node] = total
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
        """MCL stdin text "A B w" per edge (read_graph.py:350-357)."""
        return "\n".join(f"{a} {b} {d['weight']}" for a, b, d in self.edges(data=True)).encode("utf-8")

    def calc_distance_between_subgraphs(self, nodes_a: list, nodes_b: list) -> int:
        """Sum of weights between two node sets (read_graph.py:359-373)."""
        total = 0
        for a, b in itertools.product(nodes_a, nodes_b):
            if self.has_edge(a, b):
                total += self[a][b]["weight"]
        return total
