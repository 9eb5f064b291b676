"""The large-graph restatement of --rearrange's connection walk
(oracle.calc_connections, karma.py:103-118) against the reference itself: the
goldens the reference's own helpers produced (tests/golden/rearrange.json) and
the reference's O(N^2) has_edge walk on seeded graphs.  CPU only: the graphs
come from the oracle's eq-class graph (read_graph.py:86-131), which has the
reference's edges and weights.  The GPU test at config-5 size
(tests/test_gpu_rearrange.py) is checked against this restatement."""
import itertools
import json
import os
import random

import networkx as nx
import numpy as np

from karma_amd import synth
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def oracle_graph(seed, n, n_frags, paired):
    classes = synth.eq_classes(seed, n, n_frags, paired)
    off = np.r_[0, np.cumsum([len(c[0]) for c in classes])].astype(np.int64)
    mem = np.array([x for c in classes for x in c[0]], np.uint32)
    cnt = np.array([c[1] for c in classes], np.int64)
    skip = np.array([len(c[0]) == 1 for c in classes], np.uint8)
    return oracle.graph_groups(off, mem, cnt, skip, n, dedup=False)


def lookup(nesting):
    flat = [(no, sub) for no, cl in enumerate(nesting, 1) for sub in cl]
    return {i: {"previous_cluster": no, "mcl_subcluster": sub} for i, (no, sub) in enumerate(flat)}


def groups_via_oracle(g, subs, names, cutoff):
    pos = {x: i for i, x in enumerate(names)}
    sub = np.full(len(names), -1, np.int64)
    rank = np.zeros(len(names), np.int64)
    keys = list(subs)
    for i, k in enumerate(keys):
        for r, node in enumerate(subs[k]["mcl_subcluster"]):
            if node in pos:
                sub[pos[node]], rank[pos[node]] = i, r
    out = []
    for i, j, c in oracle.calc_connections(g["a"], g["b"], g["weight"], sub, rank, cutoff):
        out.extend([keys[i], keys[j]] for _ in range(c))
    return out


def ref_walk(subs, graph, cutoff):
    """karma.py:103-118 with full_graph passed in."""
    out = []
    for ia, ib in itertools.combinations(subs, 2):
        weight = 0
        for A, B in itertools.product(subs[ia]["mcl_subcluster"], subs[ib]["mcl_subcluster"]):
            if graph.has_edge(A, B):
                weight += graph[A][B]["weight"]
                if weight > cutoff:
                    out.append([ia, ib])
    return out


def test_calc_connections_matches_reference_goldens():
    with open(os.path.join(HERE, "golden", "rearrange.json")) as f:
        gold = json.load(f)
    for name, case in gold["cases"].items():
        g = oracle_graph(case["seed"], case["n"], case["n_frags"], case["paired"])
        names = [f"ctg{i}" for i in range(case["n"])]
        for run in case["runs"]:
            assert groups_via_oracle(g, lookup(case["nesting"]), names, run["cutoff"]) == run["groups"], name


def test_calc_connections_matches_reference_walk():
    for seed in (3, 4):
        n = 400
        g = oracle_graph(seed, n, 20_000, True)
        names = [f"ctg{i}" for i in range(n)]
        graph = nx.Graph()
        graph.add_nodes_from(names)
        for a, b, w in zip(g["a"].tolist(), g["b"].tolist(), g["weight"].tolist()):
            graph.add_edge(names[a], names[b], weight=w)
        rng = random.Random(seed)
        nodes = names + ["absent"]
        rng.shuffle(nodes)
        nest, i = [], 0
        while i < len(nodes):
            k = rng.randint(1, 9)
            cl = nodes[i:i + k]
            i += k
            cut = rng.randint(1, len(cl)) if len(cl) > 1 else 1
            nest.append([cl[:cut], cl[cut:]] if cl[cut:] else [cl])
        for cutoff in (0, 0.05, 0.4, 3.0):
            assert groups_via_oracle(g, lookup(nest), names, cutoff) == ref_walk(lookup(nest), graph, cutoff)
