"""Pin the CPU oracle (oracle/) against the reference's own outputs.

tests/golden/golden.json was captured by running lmfaber/karma itself
(tests/golden/make_golden.py).  The reference's own unit test
(tests/test_kmer.py:7-8) is included as the `is_palindrome` entries.
"""
import hashlib
import os
import tempfile
from collections import OrderedDict

import numpy as np
import pytest

from karma_amd import synth
from oracle import oracle


def check_profile(out, seqs, kmer):
    if "exit" in out:
        with pytest.raises(SystemExit) as e:
            oracle.calc_kmer_profile(OrderedDict(seqs), kmer)
        assert e.value.code == out["exit"]
        return
    if "raises" in out:
        with pytest.raises(Exception) as e:
            oracle.calc_kmer_profile(OrderedDict(seqs), kmer)
        assert type(e.value).__name__ == out["raises"]
        return
    prof, cols, _ = oracle.calc_kmer_profile(OrderedDict(seqs), kmer)
    assert list(prof.shape) == out["shape"]
    assert cols == out["columns"]
    assert hashlib.sha256(prof.astype("<f8").tobytes()).hexdigest() == out["sha256"]
    if "nz" in out:
        r, c = prof.nonzero()
        got = [[int(a), int(b), float(prof[a, b])] for a, b in zip(r, c)]
        assert got == out["nz"]


def test_is_palindrome_reference_unit_test(golden):
    # reference tests/test_kmer.py:7-8
    assert oracle.is_palindrome("ACGT") is False
    assert oracle.is_palindrome("AAAA") is True
    for s, v in golden["is_palindrome"].items():
        assert oracle.is_palindrome(s) is v


def test_profile_hand_cases(golden):
    for name, case in golden["profile_hand"].items():
        check_profile(case["out"], [tuple(x) for x in case["seqs"]], case["kmer"])


def test_profile_random_cases(golden):
    for name, case in golden["profile_rand"].items():
        seqs = synth.contig_sequences(case["seed"], case["n"], case["len_min"], case["len_span"], case["n_rate"])
        check_profile(case["out"], list(seqs.items()), case["kmer"])


def test_profile_config1_digest(golden):
    case = golden["profile_config1"]
    seqs = synth.contig_sequences(case["seed"], case["n"])
    check_profile(case["out"], list(seqs.items()), case["kmer"])


def edges_canon(edges):
    return sorted((min(a, b), max(a, b), w) for a, b, w in edges)


def check_graph(out, fn):
    if "raises" in out:
        with pytest.raises(Exception) as e:
            fn()
        assert type(e.value).__name__ == out["raises"]
        return
    d = oracle.graph_dump(fn())
    assert d["edges"] == out["edges"]  # same weights AND same networkx edge order
    return d


def test_eq_graph_hand(golden, tmp_path):
    for name, case in golden["eq_hand"].items():
        p = tmp_path / f"{name}.txt"
        p.write_text(case["text"])
        d = check_graph(case["out"], lambda: oracle.graph_from_eq_file(str(p), case["fasta"]))
        if d:
            n_txp = int(case["text"].split("\n")[0])
            assert d["nodes"][:n_txp] == case["out"]["nodes"][:n_txp]
            assert set(d["nodes"][n_txp:]) == set(case["out"]["nodes"][n_txp:])


def test_eq_graph_synth(golden, tmp_path):
    for name, case in golden["eq_synth"].items():
        classes = synth.eq_classes(case["seed"], case["n"], case["n_frags"], case["paired"])
        names = [f"ctg{i}" for i in range(case["n"])]
        p = tmp_path / f"{name}.txt"
        p.write_text(synth.eq_file_text(names, classes))
        d = check_graph(case["out"], lambda: oracle.graph_from_eq_file(str(p), [">" + x for x in names]))
        assert d["nodes"][: case["n"]] == case["out"]["nodes"][: case["n"]]


def test_readset_graph_hand(golden):
    for name, case in golden["readset_hand"].items():
        d = check_graph(case["out"], lambda: oracle.graph_from_readsets(case["names"], case["readsets"]))
        assert d["nodes"] == case["out"]["nodes"]


def test_readset_graph_synth_direct_and_grouped(golden):
    for name, case in golden["readset_synth"].items():
        recs = synth.read_records(case["seed"], case["n"], case["n_frags"], case["paired"])
        assert len(recs) == case["n_records"]
        n = case["n"]
        sets = [[] for _ in range(n)]
        for r, c in recs:
            sets[c].append(f"r{r}")
        names = [f"ctg{i}" for i in range(n)]
        d = check_graph(case["out"], lambda: oracle.graph_from_readsets(names, sets))
        assert d["nodes"] == case["out"]["nodes"]
        # group-by-read restatement (used at scale) must agree exactly
        rec = np.array(recs, dtype=np.int64)
        starts = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
        off = np.r_[starts, len(rec)]
        r = oracle.graph_groups(off, rec[:, 1], None, None, n, dedup=True)
        got = [[names[a], names[b], float(w)] for a, b, w in zip(r["a"], r["b"], r["weight"])]
        assert got == case["out"]["edges"]


def test_update_graph_hand(golden):
    import networkx as nx
    for name, case in golden["update_hand"].items():
        g = nx.Graph()
        for a, b, w in case["base_edges"]:
            g.add_edge(a, b, weight=w)
        g = oracle.update_graph(g, case["orig_names"], case["orig_sets"], case["new_names"], case["new_sets"])
        d = oracle.graph_dump(g)
        assert d == case["out"], name


def test_omp_column_table_equals_scalar():
    # the CPU baseline's parallel column table (oracle_omp_kmer_columns) is the
    # scalar restatement's union, key for key, with non-ACGT bytes and every kmode
    from collections import OrderedDict

    from karma_amd import engine

    blob, offs, _ = engine.synth_contigs(9, 3000, 1, 400, 50)
    seqs = OrderedDict((f">c{i}", bytes(blob[offs[i]:offs[i + 1]]).decode("latin-1")) for i in range(3000))
    for k in ("5p6", 1, 3, 5, 7, 8):
        r1, m1 = oracle.kmer_columns(seqs, k)
        r2, m2 = oracle.omp_kmer_columns_packed(blob, offs, k)
        assert m1 == m2 and oracle.decode_keys(r1, m1) == oracle.decode_keys(r2, m2)
