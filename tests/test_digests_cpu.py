"""The oracle at config 2 size against the REFERENCE's own digests (CPU).

tests/golden/digests.json holds, for BASELINE configs[1] (50k contigs, 10M
paired fragments, 5p6 -- bench.py's config2 workload):
  * reference_config2: digests of lmfaber/karma's own outputs, recorded in the
    build container by tests/golden/make_digests.py --reference
    (KmerClustering.__calc_kmer_profile, kmer.py:199-264;
    ReadGraph.from_equivalence_classes, read_graph.py:61-148);
  * config2: the oracle's digests of the same workload, which the GPU tests
    (tests/test_gpu_configs.py) compare the HIP path against.
This test reruns the oracle (OpenMP twin, ~15 s) and checks it against both,
so the oracle digests the GPU is held to are pinned by the reference itself.
"""
import numpy as np

import digests as D
from oracle import oracle


def test_oracle_config2_matches_reference_digests():
    gold = D.load()
    ref, orc = gold["reference_config2"], gold["config2"]
    inp = D.bench_inputs("config2")
    from collections import OrderedDict

    seqs = OrderedDict()
    for i in range(inp["n_loc"]):
        seqs[f">ctg{i}"] = bytes(inp["blob"][inp["offs"][i]:inp["offs"][i + 1]]).decode("latin-1")
    raw, M = oracle.kmer_columns(seqs, inp["kmer"])
    cols = oracle.decode_keys(raw, M)
    prof = oracle.omp_kmer_profile_packed(inp["blob"], inp["offs"], inp["key_len"], inp["kmer"], raw, M)
    got = (int(M), D.columns_digest(cols), D.profile_digest(prof))
    assert got == (ref["M"], ref["columns"], ref["profile"])
    assert got == (orc["M"], orc["columns"], orc["profile"])
    assert D.profile_rows_digest(prof) == orc["profile_rows"]
    del prof
    rec = inp["rec"]
    starts = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    g = oracle.omp_graph_reads(np.r_[starts, len(rec)].astype(np.int64), rec[:, 1], inp["n_glob"])
    assert D.edge_digests(g["a"], g["b"], g["weight"]) == ref["edges"]
    assert D.edge_digests(g["a"], g["b"], g["weight"], g["shared"], g["totals"]) == orc["edges"]


def test_config3_digests_are_the_reference_outputs():
    """reference_config3: lmfaber/karma's own config-3 outputs (profile 424 s,
    eq graph 10 s in the build container, tests/golden/time_reference.py,
    tests/golden/reference_config3.json).  The oracle digests that the GPU tests
    and bench.py's in-run parity check use for config 3 are the same bytes."""
    gold = D.load()
    ref, orc = gold["reference_config3"], gold["config3"]
    assert (ref["M"], ref["columns"], ref["profile"], ref["profile_rows"]) == \
        (orc["M"], orc["columns"], orc["profile"], orc["profile_rows"])
    assert ref["edges"] == {k: orc["edges"][k] for k in ("E", "ab", "weight")}
    assert ref["nodes"] == orc["N"]


def test_profile_rows_digest_is_shard_independent():
    rng = np.random.default_rng(5)
    prof = rng.random((1000, 37))
    whole = D.profile_rows_digest(prof)
    parts = b"".join(D.row_digests(np.ascontiguousarray(prof[lo:hi])) for lo, hi in ((0, 333), (333, 334), (334, 1000)))
    assert D.profile_rows_digest(rows=parts) == whole
