"""GPU parity of --rearrange (karma/karma.py:409-437).

* tests/golden/rearrange.json: the reference's own helpers (taken from
  karma.py's syntax tree, tests/golden/make_golden_rearrange.py) on graphs the
  reference built, at four weight cutoffs -- the connection list (with its
  duplicates) and the rearranged nesting must match exactly;
* in process: the reference's O(N^2) has_edge walk (karma.py:103-118, restated
  below) on larger seeded graphs, including nodes outside the graph, FASTA-only
  nodes and a graph built by hand (export path).
"""
import itertools
import json
import os
import random
from collections import OrderedDict

import pytest

from karma_amd import rearrange, synth
from karma_amd.read_graph import ReadGraph

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def ref_calc_connections(mcl_subclusters, full_graph, weight_cutoff=0):
    """karma.py:103-118 with full_graph passed in (the reference reads a global)."""
    mcl_groups_to_combine = []
    for index_A, index_B in itertools.combinations(mcl_subclusters, 2):
        nodes_A = mcl_subclusters[index_A]["mcl_subcluster"]
        nodes_B = mcl_subclusters[index_B]["mcl_subcluster"]
        weight = 0
        for A, B in itertools.product(nodes_A, nodes_B):
            if full_graph.has_edge(A, B):
                weight += full_graph[A][B]["weight"]
                if weight > weight_cutoff:
                    mcl_groups_to_combine.append([index_A, index_B])
    return mcl_groups_to_combine


def lookup(nesting):
    """The index -> {previous_cluster, mcl_subcluster} dict karma.py:78-100 builds
    (the caller's own helper; only its shape matters here)."""
    flat = [(no, sub) for no, cl in enumerate(nesting, 1) for sub in cl]
    return {i: {"previous_cluster": no, "mcl_subcluster": sub} for i, (no, sub) in enumerate(flat)}


def eq_graph(tmp_path, seed, n, nf, paired, extra=()):
    classes = synth.eq_classes(seed, n, nf, paired)
    names = [f"ctg{i}" for i in range(n)]
    p = tmp_path / f"eq{seed}.txt"
    p.write_text(synth.eq_file_text(names, classes))
    return ReadGraph.from_equivalence_classes(str(p), OrderedDict((">" + x, "") for x in names + list(extra))), names


def test_rearrange_golden(tmp_path):
    with open(os.path.join(HERE, "golden", "rearrange.json")) as f:
        gold = json.load(f)
    for name, case in gold["cases"].items():
        g, names = eq_graph(tmp_path, case["seed"], case["n"], case["n_frags"], case["paired"])
        for run in case["runs"]:
            subs = lookup(case["nesting"])
            groups = rearrange.calc_connections_between_mcl_subclusters(subs, weight_cutoff=run["cutoff"],
                                                                        full_graph=g)
            assert groups == run["groups"], (name, run["cutoff"])


def nesting(nodes, rng, max_cluster=10):
    out, i = [], 0
    while i < len(nodes):
        k = rng.randint(1, max_cluster)
        cl = nodes[i:i + k]
        i += k
        cuts = sorted(rng.sample(range(1, len(cl)), min(len(cl) - 1, rng.randint(0, 3)))) if len(cl) > 1 else []
        parts, s = [], 0
        for c in cuts + [len(cl)]:
            parts.append(cl[s:c])
            s = c
        out.append(parts)
    return out


@pytest.mark.parametrize("seed", [41, 42])
def test_rearrange_vs_reference_walk(tmp_path, seed):
    g, names = eq_graph(tmp_path, seed, 1500, 60_000, True, extra=("iso_x",))
    rng = random.Random(seed)
    nodes = names + ["iso_x", "not_in_graph"]
    rng.shuffle(nodes)  # subclusters that mix genes: many cross pairs
    nest = nesting(nodes, rng)
    for cutoff in (0, 0.01, 0.3, 2.0):
        subs = lookup(nest)
        assert rearrange.calc_connections_between_mcl_subclusters(subs, cutoff, full_graph=g) == \
            ref_calc_connections(subs, g, cutoff)
    # the module global the reference reads, and the NameError without it
    subs = lookup(nest)
    with pytest.raises(NameError):
        rearrange.calc_connections_between_mcl_subclusters(subs, 0)
    rearrange.full_graph = g
    try:
        assert rearrange.calc_connections_between_mcl_subclusters(subs, 0.1) == ref_calc_connections(subs, g, 0.1)
    finally:
        rearrange.full_graph = None


def test_rearrange_hand_graph_and_partition_check():
    h = ReadGraph()
    h.add_edge("a", "b", weight=0.25)
    h.add_edge("b", "c", weight=0.5)
    h.add_edge("c", "d", weight=0.125)
    h.add_edge("a", "d", weight=0.0625)
    h.add_node("e")
    nest = [[["a"], ["b"]], [["c", "d"]], [["e"]]]
    seqs = ["a", "b", "c", "d", "e"]
    for cutoff in (0, 0.1, 0.3, 0.6):
        subs = lookup(nest)
        assert rearrange.calc_connections_between_mcl_subclusters(subs, cutoff, full_graph=h) == \
            ref_calc_connections(subs, h, cutoff)
    with pytest.raises(ValueError):
        subs = lookup([[["a", "b"], ["b"]]])
        rearrange.calc_connections_between_mcl_subclusters(subs, 0, full_graph=h)


def test_rearrange_config5_scale():
    """BASELINE configs[4] --rearrange leg (karma.py:409-437) at config-5 size: the
    graph of config 5's 1M contigs, from 25M of its fragments as salmon eq
    classes through the drop-in's eq constructor (the path karma.py:240 calls),
    ~250k MCL-like subclusters (2-8 contigs, some mixing genes); the connection
    list of karma.py:103-118 at three cutoffs equals the large-graph
    restatement oracle.calc_connections (pinned on the CPU against the
    reference's goldens and its own walk, tests/test_rearrange_oracle_cpu.py),
    computed from the oracle's own eq graph."""
    import numpy as np

    from karma_amd import engine
    from oracle import oracle

    n = 1_000_000
    genes = engine.synth_genes(5, n)
    off, mem, cnt = engine.synth_eq_classes(5, n, 0, 25_000_000, True, genes=genes)
    skip = (np.diff(off) == 1).astype(np.uint8)
    names = [f"ctg{i}" for i in range(n)]
    g = ReadGraph._from_eq_arrays(names, off, mem, cnt, skip, dict.fromkeys((">" + x for x in names), ""))
    og = oracle.graph_groups(off, mem, cnt, skip, n, dedup=False)
    assert g.number_of_edges() == len(og["a"]) > 500_000
    rng = random.Random(55)
    order = list(range(n))
    for i in range(0, n - 1, 2):  # a fifth of neighbouring pairs swapped: subclusters that mix genes
        if rng.random() < 0.2:
            order[i], order[i + 1] = order[i + 1], order[i]
    nest, i = [], 0
    while i < n:
        k = rng.randint(2, 8)
        cl = order[i:i + k]
        i += k
        cut = rng.randint(1, len(cl))
        nest.append([[names[x] for x in cl[:cut]]] + ([[names[x] for x in cl[cut:]]] if cl[cut:] else []))
    subs = lookup(nest)
    keys = list(subs)
    sub = np.full(n, -1, np.int64)
    rank = np.zeros(n, np.int64)
    for si, key in enumerate(keys):
        for r, node in enumerate(subs[key]["mcl_subcluster"]):
            x = int(node[3:])
            sub[x], rank[x] = si, r
    assert len(keys) > 200_000
    for cutoff in (0, 0.2, 1.0):
        got = rearrange.calc_connections_between_mcl_subclusters(subs, cutoff, full_graph=g)
        want = []
        for a, b, c in oracle.calc_connections(og["a"], og["b"], og["weight"], sub, rank, cutoff):
            want.extend([keys[a], keys[b]] for _ in range(c))
        assert got == want, cutoff
        assert len(want) > (1000 if cutoff < 1 else 0)
