"""GPU parity at BASELINE config sizes, on the exact workloads bench.py times.

The production path (ShardedBuild.run, the library's HIP kernels through the C
ABI) runs each workload once with keep=True; its outputs are hashed with the
canonical encodings of tests/digests.py and compared with tests/golden/digests.json:
  * the oracle's digests (oracle/oracle.c OpenMP twin, computed in the build
    container by tests/golden/make_digests.py) for config 2, config 3, rank
    0's share of config 5 (k = 7, 1M global contig ids) and config 5 whole
    on this one GPU (1M contigs, 500M fragments, a 131 GB profile);
  * for config 2 also the REFERENCE's own digests (kmer.py:199-264 profile,
    read_graph.py:61-148 eq graph), recorded by make_digests.py --reference;
  * config 4 (BASELINE configs[3]: config 3 split over 8 ranks, strong
    scaling): 8 ranks as threads on this one GPU, exchange host-staged
    (HostComm; RCCL refuses two ranks on one device), every other step the
    production code; the union of the ranks' outputs must hash to config 3's
    digests;
  * config 3 with its contig ids shuffled (bench.py --shuffle-contigs: most
    reads leave the compact-code path): relabelled back, the same digests.
Everything is bit-exact.
"""
import hashlib

import numpy as np
import pytest

import digests as D
from karma_amd import _lib, engine
from karma_amd.comm import HostComm, SoloComm
from karma_amd.distributed import ShardedBuild
from karma_amd.hostgroup import run_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold():
    return D.load()


def device_profile_digests(prof, plain=True, threads=8, in_flight=12):
    """(plain sha256 or None, block digest) of the device profile's C-order
    bytes, copied to the host one D.BLOCK_ROWS-row block at a time (config 5's
    131 GB profile never sits in host memory whole).  Block digests are hashed
    on a thread pool; the plain digest, when asked for, on one ordered thread."""
    from concurrent.futures import ThreadPoolExecutor

    n, M = prof.shape
    h = hashlib.sha256()
    digs, pend = [], []
    with ThreadPoolExecutor(threads) as pool, ThreadPoolExecutor(1) as seq:
        for lo in range(0, n, D.BLOCK_ROWS):
            blk = prof.view(lo * M, (min(n, lo + D.BLOCK_ROWS) - lo) * M).numpy()
            mv = memoryview(blk).cast("B")
            pend.append((pool.submit(lambda m: hashlib.sha256(m).digest(), mv),
                         seq.submit(h.update, mv) if plain else None))
            while len(pend) > in_flight:
                f, g = pend.pop(0)
                digs.append(f.result())
                g and g.result()
        for f, g in pend:
            digs.append(f.result())
            g and g.result()
    return (h.hexdigest() if plain else None), hashlib.sha256(b"".join(digs)).hexdigest()


def run_build(ctx, comm, inp, host_profile=False):
    build = ShardedBuild(ctx, comm, engine.kmode_of(inp["kmer"]), inp["n_glob"], inp["c_lo"], inp["n_loc"])
    store = engine.ContigStore(ctx, inp["blob"], inp["offs"], inp["key_len"])
    rec_dev = _lib.DevBuf.from_numpy(ctx, inp["rec"].view(np.int64).reshape(-1))
    try:
        res = build.run(store, rec_dev.ptr, len(inp["rec"]), keep=True)
        out = {"M": res["M"], "cols": engine.decode_keys(res["columns"], engine.kmode_of(inp["kmer"])),
               "edges": res["edges"]}
        if host_profile:
            out["profile"] = res["profile"].numpy()
        else:
            # the plain digest too where the profile is small enough to hash on one thread in seconds
            out["profile_sha"], out["profile_blocks"] = device_profile_digests(
                res["profile"], plain=res["profile"].nbytes < (32 << 30))
    finally:
        build.close()
        store.close()
        rec_dev.close()
    return out


def edge_digest_of(e):
    return D.edge_digests(e.a, e.b, e.weight, e.shared, e.totals)


@pytest.mark.parametrize("name", ["config2", "config3", "config5_rank0of8", "config5_1gpu"])
def test_config_digests(gold, name):
    g = gold[name]
    inp = D.bench_inputs(name)
    assert (inp["n_loc"], inp["n_glob"], inp["f_loc"], len(inp["rec"])) == (g["N"], g["n_glob"], g["fragments"],
                                                                           g["records"])
    ctx = _lib.Context(0)
    try:
        out = run_build(ctx, SoloComm(), inp)
    finally:
        ctx.close()
    assert out["M"] == g["M"]
    assert D.columns_digest(out["cols"]) == g["columns"]
    assert out["profile_blocks"] == g["profile_blocks"]
    assert out["profile_sha"] in (None, g["profile"])
    assert edge_digest_of(out["edges"]) == g["edges"]
    if name == "config2":  # the reference's own outputs (read_graph.py:61-148 has no shared/totals)
        r = gold["reference_config2"]
        assert (out["M"], D.columns_digest(out["cols"]), out["profile_sha"]) == \
            (r["M"], r["columns"], r["profile"])
        e = out["edges"]
        assert D.edge_digests(e.a, e.b, e.weight) == r["edges"]


@pytest.mark.parametrize("name", ["config2", "config3"])
def test_config_eq_path_digests(gold, name):
    """The path karma.py:240 calls (read_graph.py:61-148) on the same fragments
    as salmon eq classes: the same graph as the readset path."""
    inp = D.bench_inputs(name)
    cls_off, mem, cnt = engine.synth_eq_classes(inp["seed"], inp["n_glob"], inp["f_lo"], inp["f_lo"] + inp["f_loc"],
                                                inp["paired"], genes=inp["genes"])
    assert len(cnt) == gold[name]["eq_classes"] and len(mem) == gold[name]["eq_members"]
    skip = (np.diff(cls_off) == 1).astype(np.uint8)
    e = engine.graph_from_eq(cls_off, mem, cnt, skip, inp["n_glob"])
    assert edge_digest_of(e) == gold[name]["edges"]
    # the drop-in's form: compact inputs, (a, b, w) in insertion order (by a,
    # then first emission) -- the same edges, that order of the wide result
    sz, c32 = engine.eq_compact(cls_off, cnt, skip)
    a, b, w = engine.graph_from_eq_compact_ordered(sz, mem, c32, inp["n_glob"])
    order = np.lexsort((e.first, e.a))
    assert np.array_equal(a, e.a[order]) and np.array_equal(b, e.b[order])
    assert np.array_equal(w.view(np.uint64), e.weight[order].view(np.uint64))


def test_config3_shuffled_contig_ids(gold):
    inp = D.bench_inputs("config3", shuffle_contigs=True)
    perm = inp["perm"].astype(np.int64)
    e = engine.graph_from_records(inp["rec"], inp["n_glob"])
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(perm))
    x, y = inv[e.a], inv[e.b]
    a, b = np.minimum(x, y), np.maximum(x, y)
    o = np.lexsort((b, a))
    got = D.edge_digests(a[o], b[o], e.weight[o], e.shared[o], e.totals[perm])
    assert got == gold["config3"]["edges"]


def _strong_rank(group, rank, world):
    ctx = _lib.Context(0)
    try:
        inp = D.bench_inputs("config3", rank=rank, world=world, strong=True)
        out = run_build(ctx, HostComm(group), inp, host_profile=True)
        out["n_loc"], out["c_lo"] = inp["n_loc"], inp["c_lo"]
        return out
    finally:
        ctx.close()


def test_config4_strong_8_ranks(gold):
    """BASELINE configs[3]: config 3's contigs and fragments over 8 ranks."""
    world = 8
    parts = run_ranks(world, _strong_rank, world)
    g = gold["config3"]
    assert [p["c_lo"] for p in parts] == sorted(p["c_lo"] for p in parts)
    for p in parts:
        assert p["M"] == g["M"] and D.columns_digest(p["cols"]) == g["columns"]
    assert D.sha(*[p["profile"] for p in parts]) == g["profile"]
    cat = {k: np.concatenate([getattr(p["edges"], k) for p in parts]) for k in ("a", "b", "weight", "shared")}
    for p in parts:
        lo, hi = p["c_lo"], p["c_lo"] + p["n_loc"]
        assert np.all((p["edges"].a >= lo) & (p["edges"].a < hi)), "an edge left its owner (contig a's rank)"
    assert D.edge_digests(cat["a"], cat["b"], cat["weight"], cat["shared"], parts[0]["edges"].totals) == g["edges"]


@pytest.mark.parametrize("name,flagged", [("config2", False), ("config3", False), ("config2", True),
                                          ("config3", True)])
def test_config_deferred_step_digests(gold, name, flagged):
    """The code path bench.py TIMES at these sizes: a stream of deferred steps
    (count=False: karma_step's run_deferred, two main streams at config 2's
    size, one at config 3's), then sync.  The newest deferred step's own outputs
    -- its profile (karma_step_profile) and its edges straight from the tail
    buffers step_edge_count / step_edge_write filled (karma_step_newest_edges)
    -- must hash to the same digests as the kept synchronous step above."""
    g = gold[name]
    inp = D.bench_inputs(name)
    ctx = _lib.Context(0)
    build = ShardedBuild(ctx, SoloComm(), engine.kmode_of(inp["kmer"]), inp["n_glob"], inp["c_lo"], inp["n_loc"],
                         flagged=flagged)
    store = engine.ContigStore(ctx, inp["blob"], inp["offs"], inp["key_len"])
    rec_dev = _lib.DevBuf.from_numpy(ctx, engine.flag_records(inp["rec"]) if flagged
                                     else inp["rec"].view(np.int64).reshape(-1))
    try:
        assert build.native is not None
        for _ in range(4):
            build.run(store, rec_dev.ptr, len(inp["rec"]), count=False)
        build.sync()
        info = build.native.info()
        assert info[5] == 4 and info[6] == 0, info.tolist()  # 4 deferred steps, none run again
        assert int(info[0]) == g["M"]
        e, deferred = build.native.newest_edges()
        assert deferred
        assert int(info[1]) == len(e.a)
        assert edge_digest_of(e) == g["edges"]
        prof = build.native.profile()
        assert tuple(prof.shape) == (g["N"], g["M"])
        sha, blocks = device_profile_digests(prof)
        assert blocks == g["profile_blocks"] and sha == g["profile"]
    finally:
        build.close()
        store.close()
        rec_dev.close()
        ctx.close()
