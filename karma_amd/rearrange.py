"""--rearrange: join MCL subclusters that share reads.

Drop-in for the module-level helpers of karma/karma.py that main() calls when
--rearrange is set (karma.py:409-437):
  flatten                                   karma.py:64-65
  create_lookup_dict                        karma.py:78-100
  calc_connections_between_mcl_subclusters  karma.py:103-118   (on the device)
  remove_already_added_clusters             karma.py:121-127
  combine_connected_subclusters             karma.py:130-143
  add_remaining_kmer_based_clusters         karma.py:146-163

calc_connections_between_mcl_subclusters is the heavy one: for every pair of
subclusters (itertools.combinations of the lookup dict) it walks
product(nodes_A, nodes_B) with full_graph.has_edge -- O(N^2) lookups -- and
appends [index_A, index_B] once for every edge after which the running weight
exceeds weight_cutoff.  Here the device reduces the graph's edges by
(subcluster A, subcluster B) in that product order (csrc/consumers.hip,
karma_adj_cross_sums: the same f64 partial sums, and how many exceed the cutoff)
and the list is rebuilt from those counts, duplicates included.

The reference reads `full_graph` as a module global that main() never sets
(it is main's local, karma.py:240), so reaching it raises NameError.  The
intended graph is main's full_graph; pass it as `full_graph=` or assign
rearrange.full_graph.  Without either this raises the same NameError.
The other helpers are list/dict bookkeeping over the subclusters and
networkx's connected components of the (small) subcluster graph, restated as
the reference writes them.
"""

import networkx as nx
import numpy as np

from . import consumers
from .logs import logger

full_graph = None  # the global karma.py:114 looks up


def flatten(lst):
    """karma.py:64-65."""
    return sum(([x] if not isinstance(x, list) else flatten(x) for x in lst), [])


def create_lookup_dict(clusters_with_subcluster, sequences):
    """karma.py:78-100: index -> {previous_cluster, mcl_subcluster}."""
    mcl_subclusters = {}
    index = 0
    for cl_no, cluster in enumerate(clusters_with_subcluster, 1):
        for mcl_cluster in cluster:
            mcl_subclusters[index] = {"previous_cluster": cl_no, "mcl_subcluster": mcl_cluster}
            index += 1
    length_of_dict = sum([len(subcluster["mcl_subcluster"]) for subcluster in mcl_subclusters.values()])
    logger.debug(f"length of dict: {length_of_dict}, {len(sequences)}")
    assert length_of_dict == len(sequences), "The creation of the lookup dictionary went wrong."
    return mcl_subclusters


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


def remove_already_added_clusters(from_dict, remove):
    """karma.py:121-127."""
    for mcl in remove:
        from_dict.pop(mcl)
    return from_dict


def combine_connected_subclusters(mcl_subclusters, mcl_groups_to_combine):
    """karma.py:130-143: connected components of the subcluster graph."""
    mcl_cluster_connection_graph = nx.Graph()
    mcl_cluster_connection_graph.add_edges_from(mcl_groups_to_combine)
    connected_subclusters = []
    for new_cluster in nx.k_edge_subgraphs(mcl_cluster_connection_graph, k=1):
        connected_subclusters.append([mcl_subclusters[a]["mcl_subcluster"] for a in new_cluster])
    assert len(list(nx.k_edge_subgraphs(mcl_cluster_connection_graph, k=1))) == len(
        connected_subclusters), "Combining went wrong"
    return connected_subclusters


def add_remaining_kmer_based_clusters(mcl_subclusters):
    """karma.py:146-163: the untouched subclusters, grouped by their k-mer cluster."""
    remaining_cluster = []
    first_cl_no = -1
    first = True
    for key, value in mcl_subclusters.items():
        current_orig_cluster = value["previous_cluster"]
        if first_cl_no != current_orig_cluster:
            first_cl_no = value["previous_cluster"]
            if first:
                first = False
            else:
                remaining_cluster.append(new_subgroup)  # noqa: F821 (set on the first pass)
            new_subgroup = []
        if first_cl_no == current_orig_cluster:
            new_subgroup.append(value["mcl_subcluster"])
    remaining_cluster.append(new_subgroup)
    return remaining_cluster


def rearrange(clusters_with_subcluster, sequences, graph, weight_cutoff=0):
    """karma.py:411-437 in one call: the rearranged nested cluster list."""
    mcl_subclusters = create_lookup_dict(clusters_with_subcluster, sequences)
    groups = calc_connections_between_mcl_subclusters(mcl_subclusters, weight_cutoff=weight_cutoff, full_graph=graph)
    new_cluster_subcluster = []
    new_cluster_subcluster += combine_connected_subclusters(mcl_subclusters, groups)
    mcl_subclusters = remove_already_added_clusters(from_dict=mcl_subclusters, remove=set(flatten(groups)))
    new_cluster_subcluster += add_remaining_kmer_based_clusters(mcl_subclusters)
    assert len(flatten(new_cluster_subcluster)) == len(sequences), "rearraning groups went wrong."
    return new_cluster_subcluster
