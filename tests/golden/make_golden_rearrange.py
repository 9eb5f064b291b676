#!/usr/bin/env python3
"""Golden outputs of --rearrange (karma/karma.py:409-437),
captured by running the REFERENCE's own helpers in this container.

karma.py does not import (numba.errors, circular import: SURVEY.md §8(c)), so
flatten, create_lookup_dict, calc_connections_between_mcl_subclusters,
remove_already_added_clusters, combine_connected_subclusters and
add_remaining_kmer_based_clusters are taken from karma.py's syntax tree and
executed in one namespace.  calc_connections_between_mcl_subclusters reads
`full_graph` as a module global, which main() never sets (NameError in the
shipped CLI); the namespace gets the graph the reference's own
ReadGraph.from_equivalence_classes built, which is what main() passes as
full_graph (karma.py:240).  Inputs: the eq_synth graphs of make_golden.py and
seeded "k-mer cluster -> MCL subcluster" nestings of their nodes (consecutive
runs of contigs, as assemblers list isoforms), at several weight cutoffs.

Usage:  python tests/golden/make_golden_rearrange.py  (writes tests/golden/rearrange.json)
"""

import ast
import itertools
import json
import logging
import os
import random
import sys
from collections import OrderedDict

import networkx as nx

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import REF, import_reference  # noqa: E402

from karma_amd import synth  # noqa: E402

FUNCS = ("flatten", "create_lookup_dict", "calc_connections_between_mcl_subclusters",
         "remove_already_added_clusters", "combine_connected_subclusters", "add_remaining_kmer_based_clusters")


def reference_helpers():
    tree = ast.parse(open(os.path.join(REF, "karma", "karma.py")).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert len(fns) == len(FUNCS)
    ns = {"itertools": itertools, "nx": nx, "logger": logging.getLogger("karma_ref_silent")}
    ns["logger"].setLevel(logging.CRITICAL)
    exec(compile(ast.Module(body=fns, type_ignores=[]), "karma.py", "exec"), ns)
    return ns


def nesting(nodes, seed):
    """k-mer clusters of 1..12 consecutive contigs, each split into 1..3 MCL subclusters."""
    rng = random.Random(seed)
    out, i = [], 0
    while i < len(nodes):
        k = rng.randint(1, 12)
        cl = nodes[i:i + k]
        i += k
        cuts = sorted(rng.sample(range(1, len(cl)), min(len(cl) - 1, rng.randint(0, 2)))) if len(cl) > 1 else []
        parts, s = [], 0
        for c in cuts + [len(cl)]:
            parts.append(cl[s:c])
            s = c
        out.append(parts)
    return out


def main():
    _, RG, _, scratch = import_reference()
    ns = reference_helpers()
    gold = {"generator": "tests/golden/make_golden_rearrange.py", "reference": "lmfaber/karma (v0)"}
    cases = {}
    for name, (seed, n, nf, paired) in {"small_pe": (21, 300, 20_000, True),
                                         "config1_se": (1, 1000, 100_000, False)}.items():
        classes = synth.eq_classes(seed, n, nf, paired)
        names = [f"ctg{i}" for i in range(n)]
        path = os.path.join(scratch, f"{name}.eq.txt")
        with open(path, "w") as f:
            f.write(synth.eq_file_text(names, classes))
        g = RG.from_equivalence_classes(path, OrderedDict((">" + x, "") for x in names))
        ns["full_graph"] = g
        nest = nesting(names, seed)
        runs = []
        for cutoff in (0, 0.05, 0.5, 1.0):
            subs = ns["create_lookup_dict"](nest, names)
            groups = ns["calc_connections_between_mcl_subclusters"](subs, weight_cutoff=cutoff)
            new = []
            new += ns["combine_connected_subclusters"](subs, groups)
            subs = ns["remove_already_added_clusters"](from_dict=subs, remove=set(ns["flatten"](groups)))
            new += ns["add_remaining_kmer_based_clusters"](subs)
            assert len(ns["flatten"](new)) == len(names)
            runs.append({"cutoff": cutoff, "groups": groups, "new_cluster_subcluster": new})
        cases[name] = {"seed": seed, "n": n, "n_frags": nf, "paired": paired, "nesting": nest, "runs": runs}
    gold["cases"] = cases
    out = os.path.join(HERE, "rearrange.json")
    with open(out, "w") as f:
        json.dump(gold, f, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
