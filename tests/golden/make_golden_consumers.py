#!/usr/bin/env python3
"""Golden outputs of the read graph's consumers, captured by running the
REFERENCE (lmfaber/karma) in this container.

The reference's ReadGraph methods are run on graphs it builds itself
(from_equivalence_classes / from_contigs on the eq_synth / readset_synth /
eq_hand inputs of make_golden.py) and on copies as karma.py:274 and :308 make
them -- ReadGraph(full_graph.subgraph(nodes)) -- before and after
remove_nodes_from (karma.py:286, :331-337):
  edge_list()                      read_graph.py:350-357 (text, or its sha256)
  get_unconnected_nodes()          read_graph.py:150-160
  get_connected_nodes()            read_graph.py:162-172
  _ReadGraph__calculate_node_weights()  read_graph.py:174-190
  calculate_representative_sequences(lowest=True) with set mcl clusters, :315-344
Subgraph node sets hold at least half the graph's nodes, so the copy's node
order is the graph's own (networkx walks the filter SET -- hash order, which
varies between processes -- only for smaller sets); smaller sets are compared
in-process against the same expressions (tests/test_gpu_consumers.py).

Usage:  python tests/golden/make_golden_consumers.py  (writes tests/golden/consumers.json)
"""

import hashlib
import json
import os
import random
import sys
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import import_reference, make_contigs, records_to_readsets  # noqa: E402

from karma_amd import synth  # noqa: E402


def digest(text: bytes):
    return {"len": len(text), "sha256": hashlib.sha256(text).hexdigest(),
            "text": text.decode("utf-8") if len(text) <= 4096 else None}


def consumers(g, clusters):
    g.mcl_cluster = [list(c) for c in clusters]
    return {
        "nodes": [str(n) for n in g.nodes()],
        "edge_list": digest(g.edge_list()),
        "unconnected": [str(n) for n in g.get_unconnected_nodes()],
        "connected": [str(n) for n in g.get_connected_nodes()],
        "node_weights": [[str(k), v] for k, v in g._ReadGraph__calculate_node_weights().items()],
        "representatives": g.calculate_representative_sequences(lowest=True),
    }


def chunks(nodes, k):
    # clusters and samples from the SORTED node list: the FASTA-only nodes sit
    # in set-difference (hash) order in the graph, which varies by process
    s = sorted(nodes, key=str)
    return [s[i:i + k] for i in range(0, len(s), k)]


def case(RG, g, seed):
    rng = random.Random(seed)
    nodes = sorted(g.nodes(), key=str)
    out = {"full": consumers(g, chunks(nodes, 7))}
    subs = []
    for frac in (0.5, 0.75, 1.0):
        k = max(1, int(round(frac * len(nodes))))
        pick = rng.sample(nodes, k)
        sg = RG(g.subgraph(pick))
        rec = {"frac": frac, "pick": [str(x) for x in pick]}
        sub_nodes = sorted(sg.nodes(), key=str)
        rec["before"] = consumers(sg, chunks(sub_nodes, 5))
        drop = sg.get_unconnected_nodes() + rng.sample(sub_nodes, min(len(sub_nodes), 3))
        sg.remove_nodes_from(drop)
        rec["drop"] = [str(x) for x in drop]
        rec["after"] = consumers(sg, chunks(sg.nodes(), 4))
        subs.append(rec)
    out["subgraphs"] = subs
    return out


def main():
    _, RG, Contig, scratch = import_reference()
    gold = {"generator": "tests/golden/make_golden_consumers.py", "reference": "lmfaber/karma (v0)"}
    eq = {}
    for name, (seed, n, nf, paired) in {"config1_se": (1, 1000, 100_000, False),
                                         "small_pe": (21, 300, 20_000, True)}.items():
        classes = synth.eq_classes(seed, n, nf, paired)
        names = [f"ctg{i}" for i in range(n)]
        path = os.path.join(scratch, f"{name}.eq.txt")
        with open(path, "w") as f:
            f.write(synth.eq_file_text(names, classes))
        # two FASTA-only contigs: isolated nodes appended by the set difference
        fasta = OrderedDict((">" + x, "") for x in names + ["extra_a", "extra_b"])
        g = RG.from_equivalence_classes(path, fasta)
        eq[name] = {"seed": seed, "n": n, "n_frags": nf, "paired": paired, "extra": ["extra_a", "extra_b"],
                    "out": case(RG, g, seed)}
    hand = {"dup_ids_self_loop": ("3\n2\nu\nv\nw\n3\t0\t0\t1\t6\n2\t1\t2\t3\n", [">u", ">v", ">w"]),
            "basic": ("4\n3\nc0\nc1\nc2\nc3\n2\t0\t1\t10\n1\t2\t5\n3\t0\t1\t2\t3\n",
                      [">c0", ">c1", ">c2", ">c3"])}
    eqh = {}
    for name, (text, fasta) in hand.items():
        path = os.path.join(scratch, f"{name}.eq.txt")
        with open(path, "w") as f:
            f.write(text)
        g = RG.from_equivalence_classes(path, OrderedDict((k, "") for k in fasta))
        eqh[name] = {"text": text, "fasta": fasta, "out": case(RG, g, 5)}
    gold["eq_synth"] = eq
    gold["eq_hand"] = eqh
    rs = {}
    seed, n, nf, paired = 21, 300, 20_000, True
    recs = synth.read_records(seed, n, nf, paired)
    sets = records_to_readsets(recs, n)
    g = RG.from_contigs(make_contigs(Contig, [f"ctg{i}" for i in range(n)], sets))
    rs["small_pe"] = {"seed": seed, "n": n, "n_frags": nf, "paired": paired, "out": case(RG, g, 7)}
    gold["readset_synth"] = rs
    out = os.path.join(HERE, "consumers.json")
    with open(out, "w") as f:
        json.dump(gold, f, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
