#!/usr/bin/env python3
"""Timing of the read graph's consumers, GPU vs the
reference's expressions (karma/read_graph.py:150-190, :315-357) on the same
networkx objects.

Workload: the eq-class graph of config 2 (50k contigs, 10M paired fragments;
--n / --frags to change), then karma.py:255-395's use of it: k-mer clusters
(here: consecutive runs of --cluster contigs, i.e. whole genes), for each
  cluster_graph = ReadGraph(full_graph.subgraph(cluster))
  unconnected   = cluster_graph.get_unconnected_nodes(); remove them
  text          = cluster_graph.edge_list()                (MCL stdin)
  reps          = cluster_graph.calculate_representative_sequences()
The subgraph copy itself is networkx (same cost on both sides) and is timed
separately.  Results (GPU outputs identical to the reference's) go to stdout
as one JSON line.  Usage (GPU box): python tools/bench_consumers.py
"""
import argparse
import json
import os
import sys
import tempfile
import time
from collections import OrderedDict

import networkx as nx
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from karma_amd import _lib, engine, synth  # noqa: E402
from karma_amd import rearrange  # noqa: E402
from karma_amd.read_graph import ReadGraph  # noqa: E402



def _lookup(nesting):
    """index -> {previous_cluster, mcl_subcluster}, the shape karma.py:78-100 builds."""
    flat = [(no, sub) for no, cl in enumerate(nesting, 1) for sub in cl]
    return {i: {"previous_cluster": no, "mcl_subcluster": sub} for i, (no, sub) in enumerate(flat)}

def ref_edge_list(g):
    return "\n".join(f"{A} {B} {data['weight']}" for A, B, data in g.edges(data=True)).encode("utf-8")


def ref_unconnected(g):
    return [n for n in g.nodes() if len(list(nx.all_neighbors(g, n))) == 0]


def ref_node_weights(g):
    out = {}
    for node in g.nodes():
        node_weight = 0
        for _, _, w in g.edges(node, data=True):
            node_weight += w["weight"]
        out[node] = node_weight
    return out


def ref_reps(g):
    nw = ref_node_weights(g)
    reps = []
    for cluster in g.mcl_cluster:
        sub = dict((k, nw[k]) for k in cluster)
        reps.append(f">{max(sub, key=sub.get)}")
    return reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--frags", type=int, default=10_000_000)
    ap.add_argument("--cluster", type=int, default=40)
    ap.add_argument("--clusters", type=int, default=300, help="clusters timed (a prefix of the graph)")
    ap.add_argument("--unlabeled", type=float, default=0.1,
                    help="fraction of contigs left unlabeled (karma.py:308 adds them to every cluster graph)")
    ap.add_argument("--with-unlabeled", type=int, default=40, help="clusters timed with the unlabeled set")
    args = ap.parse_args()

    t = time.perf_counter()
    classes = synth.eq_classes(2, args.n, args.frags, True)
    names = [f"ctg{i}" for i in range(args.n)]
    path = os.path.join(tempfile.mkdtemp(), "eq.txt")
    with open(path, "w") as f:
        f.write(synth.eq_file_text(names, classes))
    g = ReadGraph.from_equivalence_classes(path, OrderedDict((">" + x, "") for x in names))
    t_build = time.perf_counter() - t
    E = g.number_of_edges()

    res = {"n": args.n, "fragments": args.frags, "edges": E, "graph_build_s": round(t_build, 2)}
    # ---- full graph -----------------------------------------------------------
    t = time.perf_counter()
    g._device_mirror()  # layout on the device (once per graph)
    _lib.default_context().sync()
    res["mirror_build_s"] = round(time.perf_counter() - t, 4)
    for label, gpu, ref in (("edge_list", lambda: g.edge_list(), lambda: ref_edge_list(g)),
                            ("unconnected", lambda: g.get_unconnected_nodes(), lambda: ref_unconnected(g)),
                            ("node_weights", lambda: g._ReadGraph__calculate_node_weights(),
                             lambda: ref_node_weights(g))):
        gpu()  # warm
        t = time.perf_counter()
        a = gpu()
        tg = time.perf_counter() - t
        t = time.perf_counter()
        b = ref()
        tr = time.perf_counter() - t
        assert a == b, label
        res[f"full_{label}"] = {"gpu_s": round(tg, 4), "ref_s": round(tr, 4), "speedup": round(tr / tg, 1)}
    text = g.edge_list()
    res["full_edge_list_bytes"] = len(text)

    # ---- karma.py cluster loop ---------------------------------------------------
    nodes = list(g.nodes())
    clusters = [nodes[i:i + args.cluster] for i in range(0, len(nodes), args.cluster)][:args.clusters]
    t_copy = t_gpu = t_ref = 0.0
    nbytes = 0
    for cl in clusters:
        t = time.perf_counter()
        cg = ReadGraph(g.subgraph(cl))
        rg = nx.Graph(g.subgraph(cl))  # the reference side's own copy
        t_copy += (time.perf_counter() - t) / 2
        rg.mcl_cluster = cg.mcl_cluster = [list(cl[: len(cl) // 2]), list(cl[len(cl) // 2:])]
        t = time.perf_counter()
        un = cg.get_unconnected_nodes()
        cg.remove_nodes_from(un)
        cg.mcl_cluster = [[x for x in c if x in cg] for c in cg.mcl_cluster]
        cg.mcl_cluster = [c for c in cg.mcl_cluster if c]
        txt = cg.edge_list()
        reps = cg.calculate_representative_sequences()
        t_gpu += time.perf_counter() - t
        t = time.perf_counter()
        un2 = ref_unconnected(rg)
        rg.remove_nodes_from(un2)
        rg.mcl_cluster = [[x for x in c if x in rg] for c in rg.mcl_cluster]
        rg.mcl_cluster = [c for c in rg.mcl_cluster if c]
        txt2 = ref_edge_list(rg)
        reps2 = ref_reps(rg)
        t_ref += time.perf_counter() - t
        assert un == un2 and txt == txt2 and reps == reps2
        nbytes += len(txt)
    # one karma_adj_view_summary call (one launch + the status poll), repeated
    root = g._device_mirror()
    pos = root.pos()
    order = np.array([pos[x] for x in clusters[0]], np.int64)
    root.adj.view_summary(order, root.names, True)
    t = time.perf_counter()
    for _ in range(200):
        root.adj.view_summary(order, root.names, True)
    t_call = (time.perf_counter() - t) / 200
    res["clusters"] = {"count": len(clusters), "size": args.cluster, "subgraph_copy_s": round(t_copy, 3),
                       "gpu_s": round(t_gpu, 3), "ref_s": round(t_ref, 3), "speedup": round(t_ref / t_gpu, 2),
                       "edge_list_bytes": nbytes, "summary_call_us": round(t_call * 1e6, 1)}

    # ---- karma.py:301-345: cluster + every unlabeled contig, MCL text, trims, reps ----
    rng = np.random.default_rng(5)
    cl_list = clusters[:args.with_unlabeled]
    taken = set(x for c in cl_list for x in c)
    rest = [x for x in nodes if x not in taken]
    unl = [rest[i] for i in np.sort(rng.choice(len(rest), int(args.unlabeled * len(nodes)), replace=False))]
    unl_set = set(unl)
    t_copy = t_gpu = t_ref = 0.0
    nbytes = 0
    for cl in cl_list:
        sel = cl + unl
        t = time.perf_counter()
        cg = ReadGraph(g.subgraph(sel))
        t_copy += time.perf_counter() - t
        rg = nx.Graph(g.subgraph(sel))
        # MCL's clusters stand in as the k-mer cluster's two halves
        groups = [list(cl[: len(cl) // 2]), list(cl[len(cl) // 2:])]
        t = time.perf_counter()
        txt = cg.edge_list()
        un = cg.get_unconnected_nodes()
        un_set = set(un)
        cg.remove_nodes_from([x for x in cg if x in unl_set and x not in un_set][:50])  # non-MCL contigs
        cg.remove_nodes_from(un)
        cg.mcl_cluster = [[x for x in c if x in cg] for c in groups]
        cg.mcl_cluster = [c for c in cg.mcl_cluster if c]
        reps = cg.calculate_representative_sequences()
        t_gpu += time.perf_counter() - t
        t = time.perf_counter()
        txt2 = ref_edge_list(rg)
        un2 = ref_unconnected(rg)
        un2_set = set(un2)
        rg.remove_nodes_from([x for x in rg if x in unl_set and x not in un2_set][:50])
        rg.remove_nodes_from(un2)
        rg.mcl_cluster = [[x for x in c if x in rg] for c in groups]
        rg.mcl_cluster = [c for c in rg.mcl_cluster if c]
        reps2 = ref_reps(rg)
        t_ref += time.perf_counter() - t
        assert txt == txt2 and un == un2 and reps == reps2
        nbytes += len(txt)
    res["clusters_with_unlabeled"] = {"count": len(cl_list), "graph_nodes": len(cl_list[0]) + len(unl) if cl_list else 0,
                                      "subgraph_copy_s": round(t_copy, 3), "gpu_s": round(t_gpu, 3),
                                      "ref_s": round(t_ref, 3), "speedup": round(t_ref / max(t_gpu, 1e-9), 2),
                                      "edge_list_bytes": nbytes}
    # ---- --rearrange (karma.py:409-437) -------------------------------------------
    import itertools
    import random

    def ref_calc(subs, graph, cutoff):  # karma.py:103-118
        out = []
        for ia, ib in itertools.combinations(subs, 2):
            weight = 0
            for A, B in itertools.product(subs[ia]["mcl_subcluster"], subs[ib]["mcl_subcluster"]):
                if graph.has_edge(A, B):
                    weight += graph[A][B]["weight"]
                    if weight > cutoff:
                        out.append([ia, ib])
        return out

    rng = random.Random(9)
    nest, i = [], 0
    while i < len(nodes):  # k-mer clusters of 1..12 consecutive contigs, 1..3 MCL subclusters each
        k = rng.randint(1, 12)
        cl = nodes[i:i + k]
        i += k
        cuts = sorted(rng.sample(range(1, len(cl)), min(len(cl) - 1, rng.randint(0, 2)))) if len(cl) > 1 else []
        parts, s0 = [], 0
        for c in cuts + [len(cl)]:
            parts.append(cl[s0:c])
            s0 = c
        nest.append(parts)
    subs = _lookup(nest)
    rearrange.calc_connections_between_mcl_subclusters(subs, 0.05, full_graph=g)  # warm
    t = time.perf_counter()
    groups = rearrange.calc_connections_between_mcl_subclusters(subs, 0.05, full_graph=g)
    t_gpu = time.perf_counter() - t
    # the reference's walk is O(S^2): time it on the first clusters and scale by (S / s)^2
    small = nest[: max(1, len(nest) // 25)]
    small_nodes = [x for c in small for sc in c for x in sc]
    ssubs = _lookup(small)
    t = time.perf_counter()
    ref_small = ref_calc(ssubs, g, 0.05)
    t_ref_small = time.perf_counter() - t
    assert ref_small == rearrange.calc_connections_between_mcl_subclusters(ssubs, 0.05, full_graph=g)
    S, s_small = len(subs), len(ssubs)
    res["rearrange"] = {"subclusters": S, "groups": len(groups), "gpu_s": round(t_gpu, 4),
                        "ref_sample_subclusters": s_small, "ref_sample_s": round(t_ref_small, 3),
                        "ref_extrapolated_s": round(t_ref_small * (S / s_small) ** 2, 1),
                        "speedup_extrapolated": round(t_ref_small * (S / s_small) ** 2 / t_gpu, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
