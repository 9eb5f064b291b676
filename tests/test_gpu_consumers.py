"""GPU parity of the read graph's consumers.

Two references:
  * tests/golden/consumers.json -- lmfaber/karma's own ReadGraph methods
    (edge_list, get_unconnected_nodes / get_connected_nodes, node weights,
    calculate_representative_sequences) on graphs and subgraph copies it built
    (tests/golden/make_golden_consumers.py);
  * the reference's expressions (read_graph.py:150-190, :315-357), restated
    below, on the same networkx objects in this process -- for seeded graphs,
    subgraphs small enough that networkx orders them by the filter set's hash
    order, node removals, mutations (export path) and hand-built graphs.
Everything is compared exactly: bytes of the edge list, node lists in order,
f64 node weights (bit-exact sums in adjacency order), representative names.
"""
import json
import os
import random
from collections import OrderedDict

import networkx as nx
import numpy as np
import pytest

from karma_amd import synth
from karma_amd.contig import Contig
from karma_amd.read_graph import ReadGraph

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
EXTRA = ("extra_a", "extra_b")


# ---- the reference's expressions (karma/read_graph.py) -----------------------
def ref_edge_list(g):  # :350-357
    return "\n".join(f"{A} {B} {data['weight']}" for A, B, data in g.edges(data=True)).encode("utf-8")


def ref_unconnected(g):  # :150-160
    return [n for n in g.nodes() if len(list(nx.all_neighbors(g, n))) == 0]


def ref_connected(g):  # :162-172
    return [n for n in g.nodes() if len(list(nx.all_neighbors(g, n))) != 0]


def ref_node_weights(g):  # :174-190
    out = {}
    for node in g.nodes():
        node_weight = 0
        for _, _, w in g.edges(node, data=True):
            node_weight += w["weight"]
        out[node] = node_weight
    return out


def ref_representatives(g, clusters, lowest=True):  # :315-344
    nw = ref_node_weights(g)
    reps = []
    for cluster in clusters:
        sub = dict((k, nw[k]) for k in cluster)
        reps.append(f">{max(sub, key=sub.get)}")
        if lowest:
            reps.append(f">{min(sub, key=sub.get)}")
    return reps


def check_against_reference(g, clusters=None):
    assert g.edge_list() == ref_edge_list(g)
    assert g.get_unconnected_nodes() == ref_unconnected(g)
    assert g.get_connected_nodes() == ref_connected(g)
    ours = g._ReadGraph__calculate_node_weights()
    want = ref_node_weights(g)
    assert list(ours) == list(want)
    assert [type(v) for v in ours.values()] == [type(v) for v in want.values()]
    assert np.array_equal(np.array(list(ours.values()), np.float64).view(np.uint64),
                          np.array(list(want.values()), np.float64).view(np.uint64))
    if clusters is not None:
        g.mcl_cluster = [list(c) for c in clusters]
        assert g.calculate_representative_sequences(lowest=True) == ref_representatives(g, clusters)


# ---- goldens ------------------------------------------------------------------
@pytest.fixture(scope="module")
def cgold():
    with open(os.path.join(HERE, "golden", "consumers.json")) as f:
        return json.load(f)


def canon(nodes):
    """FASTA-only nodes come in set-difference (hash) order: compare them as a set at the end."""
    return [n for n in nodes if n not in EXTRA] + sorted(n for n in nodes if n in EXTRA)


def chunks(nodes, k):
    s = sorted(nodes, key=str)
    return [s[i:i + k] for i in range(0, len(s), k)]


def check_golden(g, want, clusters):
    g.mcl_cluster = [list(c) for c in clusters]
    assert canon([str(n) for n in g.nodes()]) == canon(want["nodes"])
    text = g.edge_list()
    assert len(text) == want["edge_list"]["len"]
    import hashlib
    assert hashlib.sha256(text).hexdigest() == want["edge_list"]["sha256"]
    if want["edge_list"]["text"] is not None:
        assert text.decode() == want["edge_list"]["text"]
    assert canon(g.get_unconnected_nodes()) == canon(want["unconnected"])
    assert canon(g.get_connected_nodes()) == canon(want["connected"])
    got = g._ReadGraph__calculate_node_weights()
    wd = dict((k, v) for k, v in want["node_weights"])
    assert canon(list(got)) == canon(list(wd))
    for k, v in got.items():
        assert type(v) is type(wd[k]) and v == wd[k] and str(v) == str(wd[k]), k
    assert g.calculate_representative_sequences(lowest=True) == want["representatives"]


def run_case(g, out):
    nodes = sorted(g.nodes(), key=str)
    check_golden(g, out["full"], chunks(nodes, 7))
    for rec in out["subgraphs"]:
        sg = ReadGraph(g.subgraph(rec["pick"]))
        check_golden(sg, rec["before"], chunks(sg.nodes(), 5))
        sg.remove_nodes_from(rec["drop"])
        check_golden(sg, rec["after"], chunks(sg.nodes(), 4))


def test_consumers_golden_eq(cgold, tmp_path):
    for name, case in cgold["eq_synth"].items():
        classes = synth.eq_classes(case["seed"], case["n"], case["n_frags"], case["paired"])
        names = [f"ctg{i}" for i in range(case["n"])]
        p = tmp_path / f"{name}.txt"
        p.write_text(synth.eq_file_text(names, classes))
        fasta = OrderedDict((">" + x, "") for x in names + case["extra"])
        run_case(ReadGraph.from_equivalence_classes(str(p), fasta), case["out"])
    for name, case in cgold["eq_hand"].items():
        p = tmp_path / f"{name}.txt"
        p.write_text(case["text"])
        g = ReadGraph.from_equivalence_classes(str(p), OrderedDict((k, "") for k in case["fasta"]))
        run_case(g, case["out"])


def make_contigs(names, readsets):
    out = []
    for n, reads in zip(names, readsets):
        c = Contig(n)
        c.load_from_iterator([f"{r}\t0\t{n}\t1\t60\t*" for r in reads])
        out.append(c)
    return out


def test_consumers_golden_readset(cgold):
    case = cgold["readset_synth"]["small_pe"]
    recs = synth.read_records(case["seed"], case["n"], case["n_frags"], case["paired"])
    sets = [[] for _ in range(case["n"])]
    for r, c in recs:
        sets[c].append(f"r{r}")
    g = ReadGraph.from_contigs(make_contigs([f"ctg{i}" for i in range(case["n"])], sets))
    run_case(g, case["out"])


# ---- in-process against the reference's expressions ---------------------------
def eq_graph(tmp_path, seed, n, nf, paired, extra=()):
    classes = synth.eq_classes(seed, n, nf, paired)
    names = [f"ctg{i}" for i in range(n)]
    p = tmp_path / f"eq{seed}.txt"
    p.write_text(synth.eq_file_text(names, classes))
    return ReadGraph.from_equivalence_classes(str(p), OrderedDict((">" + x, "") for x in list(names) + list(extra)))


@pytest.mark.parametrize("seed,n,nf", [(31, 2000, 60_000), (32, 5000, 150_000)])
def test_consumers_subgraphs_vs_reference(tmp_path, seed, n, nf):
    g = eq_graph(tmp_path, seed, n, nf, True, extra=("iso1", "iso2", "iso3"))
    check_against_reference(g, chunks(g.nodes(), 9))
    rng = random.Random(seed)
    nodes = list(g.nodes())
    # small sets: networkx walks the filter set (hash order); large: the graph's order
    for frac in (0.01, 0.05, 0.2, 0.45, 0.5, 0.8, 1.0):
        pick = rng.sample(nodes, max(1, int(frac * len(nodes))))
        sg = ReadGraph(g.subgraph(pick))
        check_against_reference(sg, chunks(sg.nodes(), 6))
        # karma.py:285-286 / :331-337: drop unconnected and non-cluster nodes
        sg.remove_nodes_from(sg.get_unconnected_nodes())
        check_against_reference(sg)
        drop = rng.sample(list(sg.nodes()), min(len(sg), 11))
        sg.remove_nodes_from(drop)
        check_against_reference(sg, chunks(sg.nodes(), 3))
        # a copy of a copy, and a subgraph of a trimmed copy
        check_against_reference(ReadGraph(sg))
        if len(sg):
            sub2 = rng.sample(list(sg.nodes()), max(1, len(sg) // 3))
            check_against_reference(ReadGraph(sg.subgraph(sub2)))


def test_consumers_after_mutation_and_hand_built(tmp_path):
    g = eq_graph(tmp_path, 33, 800, 30_000, False)
    sg = ReadGraph(g.subgraph(list(g.nodes())[:300]))
    check_against_reference(sg)
    # any mutation other than node removal drops the mirror: the next call exports
    nodes = list(sg.nodes())
    sg.add_edge(nodes[0], nodes[-1], weight=0.125)
    sg.add_edge("new_node", nodes[3], weight=1e-7)
    sg.add_node("lonely")
    check_against_reference(sg, chunks(sg.nodes(), 4))
    sg.remove_edge(nodes[0], nodes[-1])
    check_against_reference(sg)
    # hand-built graph with unicode names, a self-loop and exponent-form weights
    h = ReadGraph()
    h.add_edge("α", "β", weight=1 / 3)
    h.add_edge("β", "β", weight=2.5e-5)
    h.add_edge("γ", "α", weight=1e16)
    h.add_node("δ")
    check_against_reference(h, [["α", "β"], ["γ", "δ"]])
    # update_graph (read_graph.py:192-221) mutates through add_edge / add_node
    c = make_contigs(["o1", "o2", "n1", "n2"], [["r1", "r2"], ["r3"], ["r2", "r9"], []])
    u = ReadGraph.from_contigs(c[:2])
    u.set_original_contigs(c[:2])
    u.update_graph(c[2:])
    check_against_reference(u, [["o1", "n1"], ["o2", "n2"]])


def test_consumers_empty_and_edgeless(tmp_path):
    check_against_reference(ReadGraph())
    g = eq_graph(tmp_path, 34, 50, 2_000, False)
    sg = ReadGraph(g.subgraph([]))
    check_against_reference(sg)
    iso = ReadGraph(g.subgraph(ref_unconnected(g)[:5]))
    check_against_reference(iso)


def test_consumers_non_float_weight_raises():
    h = ReadGraph()
    h.add_edge("a", "b", weight=1)
    with pytest.raises(TypeError):
        h.edge_list()
    h2 = ReadGraph()
    h2.add_edge("a", "b")
    with pytest.raises(KeyError):
        h2.edge_list()


def test_small_view_one_launch_path(tmp_path):
    """karma.py:255-282's cluster loop on gene-sized clusters goes through the
    one-launch view summary (karma_adj_view_summary); views over its limits
    (> 1024 nodes, > 4096 adjacency entries) take the general path.  Both are
    compared with the reference's expressions."""
    g = eq_graph(tmp_path, 35, 3000, 200_000, True)
    nodes = list(g.nodes())
    for i in range(0, 1200, 40):
        cl = nodes[i:i + 40]
        sg = ReadGraph(g.subgraph(cl))
        un = sg.get_unconnected_nodes()
        assert sg._summary is not None, "small view did not take the one-launch path"
        assert un == ref_unconnected(sg)
        sg.remove_nodes_from(un)
        check_against_reference(sg, chunks(sg.nodes(), 5))
        # removing nodes that have edges: recomputed as the view of what is left
        if len(sg) > 3:
            sg.remove_nodes_from(list(sg.nodes())[1:3])
            check_against_reference(sg, chunks(sg.nodes(), 4))
    big = ReadGraph(g.subgraph(nodes[:1500]))
    check_against_reference(big)
    assert big._summary is None
    # a clique of 100 contigs: 9,900 adjacency entries, over the LDS budget
    names = [f"q{i}" for i in range(100)]
    clique = ReadGraph.from_contigs(make_contigs(names, [["shared", f"own{i}"] for i in range(100)]))
    sq = ReadGraph(clique.subgraph(names[::-1]))
    check_against_reference(sq, chunks(sq.nodes(), 10))
    assert sq._summary is None
    sq.remove_nodes_from(names[:60])  # 40 nodes left: 1,560 entries, one launch again
    check_against_reference(sq, chunks(sq.nodes(), 10))
    assert sq._summary is not None
