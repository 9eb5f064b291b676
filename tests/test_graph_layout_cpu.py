"""read_graph._copied_graph builds, without the intermediate graph, exactly
what the reference's constructors return: cls(incoming_graph_data=G) of a G
made by add_nodes_from + an add_edge loop (read_graph.py:19-50, :96-148).
Compared here with networkx itself on random edge lists: node order, every
node's adjacency-dict order, G.edges(data=True) order, weights, and the
sharing of one data dict by both directions.  CPU only (no device calls)."""
import networkx as nx
import numpy as np
import pytest

from karma_amd.read_graph import ReadGraph, _copied_graph


def reference_build(nodes, a, b, w):
    g = nx.Graph()
    g.add_nodes_from(nodes)
    for x, y, wt in zip(a, b, w):
        g.add_edge(nodes[x], nodes[y], weight=wt)
    return ReadGraph(incoming_graph_data=g)


def layout(g):
    return [(u, list(g.adj[u].items())) for u in g]


@pytest.mark.parametrize("seed", range(12))
def test_copied_graph_matches_networkx(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 300))
    nodes = [f"c{i}" if rng.random() < 0.9 else f"n{i}x" for i in range(n)]
    m = int(rng.integers(0, 4 * n))
    pairs = {}
    for _ in range(m):
        x, y = (int(v) for v in rng.integers(0, n, 2))
        if seed % 3 == 0 and x > y:
            x, y = y, x  # sorted orientation (the eq and readset constructors)
        key = (min(x, y), max(x, y))
        if key not in pairs:
            pairs[key] = (x, y)
    order = list(pairs.values())
    if seed % 2:
        rng.shuffle(order)  # any add order
    a = [p[0] for p in order]
    b = [p[1] for p in order]
    w = rng.random(len(order)).tolist()
    ref = reference_build(nodes, a, b, w)
    got = _copied_graph(ReadGraph, nodes, np.array(a, np.int64), np.array(b, np.int64), np.array(w))
    assert type(got) is ReadGraph
    assert list(got) == list(ref)
    assert layout(got) == layout(ref)
    assert list(got.edges(data=True)) == list(ref.edges(data=True))
    assert [got.nodes[x] for x in got] == [ref.nodes[x] for x in ref]
    for u, v in got.edges():
        assert got.adj[u][v] is got.adj[v][u]
    # the built graph is an ordinary, mutable ReadGraph
    got.add_edge("new_a", "new_b", weight=1.0)
    assert got.has_edge("new_b", "new_a") and got.number_of_nodes() == n + 2


def test_from_edge_list_duplicate_names_falls_back():
    names = ["a", "b", "a", "c"]
    g = ReadGraph._from_edge_list(names, np.array([0, 1]), np.array([1, 3]), np.array([0.5, 0.25]))
    ref = reference_build(names, [0, 1], [1, 3], [0.5, 0.25])
    assert layout(g) == layout(ref)
