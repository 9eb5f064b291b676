"""CPU check of --rearrange's bookkeeping (karma.py:64-65, :78-100, :121-163):
from the reference's own connection lists (tests/golden/rearrange.json), the
lookup dict, the connected-component merge and the leftover regrouping must
rebuild the reference's rearranged nesting exactly.  No GPU calls."""
import json
import os

from karma_amd import rearrange

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rearrange_bookkeeping_from_reference_groups():
    with open(os.path.join(HERE, "golden", "rearrange.json")) as f:
        gold = json.load(f)
    for name, case in gold["cases"].items():
        names = [f"ctg{i}" for i in range(case["n"])]
        for run in case["runs"]:
            subs = rearrange.create_lookup_dict(case["nesting"], names)
            groups = [list(x) for x in run["groups"]]
            new = []
            new += rearrange.combine_connected_subclusters(subs, groups)
            subs = rearrange.remove_already_added_clusters(from_dict=subs, remove=set(rearrange.flatten(groups)))
            new += rearrange.add_remaining_kmer_based_clusters(subs)
            assert new == run["new_cluster_subcluster"], (name, run["cutoff"])
            assert len(rearrange.flatten(new)) == len(names)


def test_flatten_and_lookup_assert():
    assert rearrange.flatten([[["a"], ["b", "c"]], [["d"]], "e"]) == ["a", "b", "c", "d", "e"]
    try:
        rearrange.create_lookup_dict([[["a"]]], ["a", "b"])
    except AssertionError:
        pass
    else:
        raise AssertionError("create_lookup_dict must assert on a lost sequence")
