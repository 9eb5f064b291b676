"""--rearrange: join MCL subclusters that share reads.

Drop-in for ONE function of karma/karma.py, the O(N^2) one main() calls when
--rearrange is set (karma.py:409-437):

  calc_connections_between_mcl_subclusters  karma.py:103-118   (on the device)

The caller keeps its own bookkeeping helpers (flatten, create_lookup_dict,
remove_already_added_clusters, combine_connected_subclusters,
add_remaining_kmer_based_clusters; karma.py:64-163): they are list/dict work
outside the hot path and are not shipped here.

For every pair of subclusters (itertools.combinations of the lookup dict) the
reference walks product(nodes_A, nodes_B) with full_graph.has_edge -- O(N^2)
lookups -- and appends [index_A, index_B] once for every edge after which the
running weight exceeds weight_cutoff.  Here the device reduces the graph's
edges by (subcluster A, subcluster B) in that product order
(csrc/consumers.hip, karma_adj_cross_sums: the same f64 partial sums, and how
many exceed the cutoff) and the list is rebuilt from those counts, duplicates
included.

The reference reads `full_graph` as a module global that main() never sets
(it is main's local, karma.py:240), so reaching it raises NameError.  The
intended graph is main's full_graph; pass it as `full_graph=` or assign
rearrange.full_graph.  Without either this raises the same NameError.
"""

import numpy as np

from . import consumers

full_graph = None  # the global karma.py:114 looks up


def _graph_mirror(graph):
    if hasattr(graph, "_device_mirror"):
        return graph._device_mirror()
    return consumers.export(graph)


def calc_connections_between_mcl_subclusters(mcl_subclusters, weight_cutoff=0, full_graph=None):
    """karma.py:103-118 with the edge walk on the device (module docstring)."""
    graph = full_graph if full_graph is not None else globals()["full_graph"]
    if graph is None:
        raise NameError("name 'full_graph' is not defined")
    keys = list(mcl_subclusters)
    m = _graph_mirror(graph)
    pos = m.pos()
    sub = np.full(len(m.nodes), -1, np.int32)
    rank = np.zeros(len(m.nodes), np.int32)
    for i, key in enumerate(keys):
        for r, node in enumerate(mcl_subclusters[key]["mcl_subcluster"]):
            p = pos.get(node)
            if p is None:  # not in the graph: has_edge is False for it
                continue
            if sub[p] != -1:
                raise ValueError(f"node {node!r} is in two subclusters (MCL clusters partition the contigs)")
            sub[p] = i
            rank[p] = r
    a, b, _, _, over = m.adj.cross_sums(sub, rank, weight_cutoff)
    mcl_groups_to_combine = []
    for x, y, k in zip(a.tolist(), b.tolist(), over.tolist()):
        mcl_groups_to_combine.extend([keys[x], keys[y]] for _ in range(k))
    return mcl_groups_to_combine
