"""The native step (karma_step, csrc/step.hip) against the oracle.

karma_amd/distributed.py ShardedBuild drives the library's karma_step for the
production path (one GPU, an emulated rank, RCCL ranks).  Its deferred steps
(outputs not read: count=False) wait for nothing: M, the records job's control
block and the tail's sizes stay on the device, a status kernel reports the
checks through mapped memory, and a step whose checks call for the general
path (relabelled contigs, bucket overflow, reads of > 8 records) runs again
synchronously.  Here: deferred steps, then sync, then the profile of the
newest deferred step and a kept step -- all bit-exact against the oracle --
and the slow paths and errors seen through the deferred checks."""
from collections import OrderedDict

import numpy as np
import pytest

from karma_amd import _lib, engine
from karma_amd.comm import SoloComm
from karma_amd.distributed import ShardedBuild
from oracle import oracle

pytestmark = pytest.mark.gpu

SEED = 41


def contigs(n, c_lo=0, n_rate=300):
    blob, offs, key_len = engine.synth_contigs(SEED, n, 30, 900, n_rate, first=c_lo)
    return blob, offs, key_len


def oracle_graph(rec, n):
    rs = np.asarray(rec, np.int64)
    st = np.flatnonzero(np.r_[True, rs[1:, 0] != rs[:-1, 0]]) if len(rs) else np.zeros(0, np.int64)
    return oracle.graph_groups(np.r_[st, len(rs)], rs[:, 1] if len(rs) else np.zeros(0), None, None, n, dedup=True)


def oracle_profile(blob, offs, c_lo, n):
    seqs = OrderedDict((f">ctg{c_lo + i}", bytes(blob[offs[i]:offs[i + 1]]).decode()) for i in range(n))
    prof, cols, _ = oracle.calc_kmer_profile(seqs, "5p6")
    return prof, cols


class Run:
    def __init__(self, n_glob, rec, emulate=1, n_rate=300, flagged=False):
        self.ctx = _lib.Context(0)
        self.n_glob = n_glob
        n_loc = n_glob // emulate if emulate > 1 else n_glob
        self.n_loc = n_loc
        self.blob, self.offs, kl = contigs(n_loc, n_rate=n_rate)
        self.build = ShardedBuild(self.ctx, SoloComm(), -1, n_glob, 0, n_loc, emulate_ranks=emulate,
                                  flagged=flagged)
        assert self.build.native is not None, "the native step drives the production path"
        self.store = engine.ContigStore(self.ctx, self.blob, self.offs, kl)
        self.rec = np.ascontiguousarray(rec)
        # the records as the step takes them: (read, contig) pairs or KARMA_REC_FLAGGED words
        self.dev = _lib.DevBuf.from_numpy(self.ctx, engine.flag_records(self.rec) if flagged
                                          else self.rec.view(np.int64).reshape(-1))

    def step(self, **kw):
        return self.build.run(self.store, self.dev.ptr, len(self.rec), **kw)

    def close(self):
        self.build.close()
        self.store.close()
        self.dev.close()
        self.ctx.close()


def check_edges(e, o):
    assert np.array_equal(e.a, o["a"]) and np.array_equal(e.b, o["b"])
    assert np.array_equal(e.shared, o["shared"])
    assert np.array_equal(e.weight.view(np.uint64), o["weight"].view(np.uint64))
    assert np.array_equal(e.totals, o["totals"])


@pytest.mark.parametrize("emulate,n_rate,flagged", [(1, 300, False), (3, 300, False), (1, 0, False), (8, 0, False),
                                                    (1, 300, True), (3, 0, True), (8, 300, True)])
def test_deferred_steps_then_kept_step_match_oracle(emulate, n_rate, flagged):
    n = 3000 if emulate == 1 else 3001  # 3001 / 3: owner bounds that do not divide evenly
    rec = engine.synth_records(SEED, n, 0, 300_000, True)
    r = Run(n, rec, emulate, n_rate, flagged)
    try:
        r.step(count=False)  # warm: allocations, events
        calls0 = _lib.api_calls()
        for _ in range(4):
            res = r.step(count=False)
            assert res["E_local"] is None
        calls = (_lib.api_calls() - calls0) / 4
        r.build.sync()
        info = r.build.native.info()
        assert info[5] == 5 and info[6] == 0, info  # 5 deferred steps, none run again
        # the newest deferred step's profile (M read by the kernels on the device)
        prof_o, cols_o = oracle_profile(r.blob, r.offs, 0, r.n_loc)
        assert info[1] is not None
        got = r.build.native.profile().numpy()
        assert got.shape == prof_o.shape
        assert np.array_equal(got.view(np.uint64), prof_o.view(np.uint64))
        # ... and its edges, from the arrays the deferred tail kernels wrote
        # (step_edge_count / step_edge_write; emulated: step_merge_kernel first)
        o = oracle_graph(rec, n)
        e_def, deferred = r.build.native.newest_edges()
        assert deferred
        check_edges(e_def, o)
        assert int(info[1]) == len(o["a"]), (info.tolist(), len(o["a"]))
        # an ACGT-only store: a deferred step enqueues ~30 HIP calls and waits
        # for nothing (with non-ACGT bases the exception keys' count is read back)
        if n_rate == 0:
            assert calls <= 40, calls
        res = r.step(keep=True)
        assert engine.decode_keys(res["columns"], -1) == cols_o
        assert np.array_equal(res["profile"].numpy().view(np.uint64), prof_o.view(np.uint64))
        check_edges(res["edges"], o)
        assert res["E_local"] == len(res["edges"].a)
        # after sync, the newest deferred step's M and edge count (its status words)
        assert int(info[0]) == len(cols_o)
        assert int(info[1]) == len(res["edges"].a), (info.tolist(), len(res["edges"].a))
        # after a kept (synchronous) step the accessor answers with its edges
        e_sync, deferred = r.build.native.newest_edges()
        assert not deferred
        check_edges(e_sync, o)
    finally:
        r.close()


@pytest.mark.parametrize("big,flagged", [(True, False), (False, False), (True, True), (False, True)])
def test_deferred_steps_slow_path_runs_again(big, flagged):
    """Shuffled contig ids (most reads leave the compact path: the relabel vote)
    plus (big) reads of > 8 records: the deferred step's status calls for the
    general path and the step runs again synchronously; the next deferred steps
    run synchronously for a while; results stay exact.  Without big reads the
    relabel verdict alone calls for the rerun: on the step's own control block
    (from the second deferred step of each main stream) it comes from
    classify's chunk votes, not from the probe kernel."""
    n = 4000
    rec = np.ascontiguousarray(engine.synth_records(SEED, n, 0, 200_000, True))
    perm = np.random.default_rng(3).permutation(n).astype(np.uint32)
    rec[:, 1] = perm[rec[:, 1]]
    if big:
        rng = np.random.default_rng(4)
        r0 = int(rec[-1, 0]) + 1
        extra = np.array([(r0 + i, int(c)) for i in range(200) for c in rng.integers(0, n, 12)], np.uint32)
        rec = np.concatenate([rec, extra])
    r = Run(n, rec, flagged=flagged)
    try:
        for _ in range(3 if big else 12):
            r.step(count=False)
        r.build.sync()
        info = r.build.native.info()
        assert info[6] >= 1, info  # run again on the general path
        if not big:
            assert info[14] >= 1, info  # some verdicts came from the votes on the step's own block
        res = r.step(keep=True)
        check_edges(res["edges"], oracle_graph(rec, n))
    finally:
        r.close()


def test_deferred_steps_on_own_control_block_launch_no_probe():
    """From the second deferred step of each main stream on, the records job
    takes the step's own zeroed control block: no relabel probe launch ahead of
    classify (the relabel verdict comes from classify's votes); results exact."""
    n = 3000
    rec = engine.synth_records(SEED, n, 0, 300_000, True)
    r = Run(n, rec)
    try:
        for _ in range(3):
            r.step(count=False)  # each main stream's first job sizes its control block
        r.build.sync()
        own0 = int(r.build.native.info()[14])
        r.ctx.timing(True, "relabel_probe")
        r.ctx.timing_reset()
        for _ in range(6):
            r.step(count=False)
        r.build.sync()
        probes = r.ctx.timing_read().get("relabel_probe", (0.0, 0))[1]
        r.ctx.timing(False)
        info = r.build.native.info()
        assert int(info[14]) - own0 == 6, info
        assert probes == 0, probes
        assert info[6] == 0, info
        res = r.step(keep=True)
        check_edges(res["edges"], oracle_graph(rec, n))
    finally:
        r.close()


def test_deferred_step_bucket_overflow_runs_again():
    rng = np.random.default_rng(1)
    R = 60_000
    reads = np.repeat(np.arange(R, dtype=np.uint32), 8)
    cs = rng.integers(0, 1000, R * 8).astype(np.uint32)
    rec = np.stack([reads, cs], 1)
    r = Run(1000, rec)
    try:
        r.step(count=False)
        r.build.sync()
        assert r.build.native.info()[6] == 1
        res = r.step(keep=True)
        check_edges(res["edges"], oracle_graph(rec, 1000))
    finally:
        r.close()


def test_deferred_step_unsorted_records_error_reported():
    rec = engine.synth_records(SEED, 2000, 0, 50_000, True)
    shuf = rec[np.random.default_rng(0).permutation(len(rec))]
    r = Run(2000, shuf)
    try:
        r.step(count=False)  # returns at once; the error arrives with the deferred check
        with pytest.raises(_lib.KarmaError) as ei:
            r.build.sync()
        assert ei.value.code == _lib.KARMA_ERR_UNSORTED
    finally:
        r.close()


def test_native_step_equals_python_driver():
    """The native step and the Python driver (HipOps, kept for the host-staged
    rehearsal transport) give the same bytes, one GPU and an emulated rank."""
    from karma_amd.distributed import HipOps

    n = 2500
    rec = engine.synth_records(SEED + 1, n, 0, 150_000, True)
    for emulate in (1, 4):
        outs = []
        for python in (False, True):
            ctx = _lib.Context(0)
            n_loc = n // emulate
            blob, offs, kl = contigs(n_loc)
            b = ShardedBuild(ctx, SoloComm(), -1, n, 0, n_loc, ops=HipOps(ctx) if python else None,
                             emulate_ranks=emulate)
            assert (b.native is None) == python
            st = engine.ContigStore(ctx, blob, offs, kl)
            d = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
            res = b.run(st, d.ptr, len(rec), keep=True)
            e = res["edges"]
            outs.append([res["profile"].numpy(), np.asarray(res["columns"]), e.a, e.b, e.shared, e.weight, e.totals,
                         np.array([res["M"], res["E_local"], res["entries"], res["pairs_local"]])])
            b.close()
            st.close()
            d.close()
            ctx.close()
        for x, y in zip(*outs):
            assert x.shape == y.shape and np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_two_steps_on_one_context_keep_their_own_status():
    """Two live native steps on one context (two ShardedBuilds of different
    shapes) interleave deferred steps: each has its own mapped status ring, so
    neither reads the other's verdicts, and each one's newest profile, M and
    edge count are its own (csrc/step.hip karma_step::ring_mem)."""
    ctx = _lib.Context(0)
    objs = []
    try:
        runs = []
        for n, nf, seed in ((2000, 120_000, SEED), (3500, 200_000, SEED + 7)):
            blob, offs, kl = engine.synth_contigs(seed, n, 30, 900, 0)
            rec = np.ascontiguousarray(engine.synth_records(seed, n, 0, nf, True))
            b = ShardedBuild(ctx, SoloComm(), -1, n, 0, n)
            st = engine.ContigStore(ctx, blob, offs, kl)
            d = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
            objs += [b, st, d]
            runs.append((b, st, d, rec, n, blob, offs))
        for _ in range(4):
            for b, st, d, rec, *_ in runs:
                b.run(st, d.ptr, len(rec), count=False)
        for b, st, d, rec, n, blob, offs in runs:
            b.sync()
            info = b.native.info()
            assert info[5] == 4 and info[6] == 0, info.tolist()  # 4 deferred, none run again
            prof_o, cols_o = oracle_profile(blob, offs, 0, n)
            assert int(info[0]) == len(cols_o)
            assert int(info[1]) == len(oracle_graph(rec, n)["a"])
            got = b.native.profile().numpy()
            assert np.array_equal(got.view(np.uint64), prof_o.view(np.uint64))
    finally:
        for o in objs:
            o.close()
        ctx.close()


def test_middle_deferred_step_rerun_keeps_newest_outputs():
    """Three deferred steps of which the middle one holds reads of > 8 records
    (its status calls for the general path, so karma_step_sync runs it again
    synchronously): the newest step's M and edge count stay the ones reported
    after sync, not the re-run's."""
    n = 3000
    rec = np.ascontiguousarray(engine.synth_records(SEED, n, 0, 150_000, True))
    rng = np.random.default_rng(9)
    r0 = int(rec[-1, 0]) + 1
    big = np.array([(r0 + i, int(c)) for i in range(50) for c in rng.integers(0, n, 12)], np.uint32)
    rec_big = np.concatenate([rec, big])
    r = Run(n, rec, n_rate=0)
    d_big = _lib.DevBuf.from_numpy(r.ctx, rec_big.view(np.int64).reshape(-1))
    try:
        r.step(count=False)
        r.build.run(r.store, d_big.ptr, len(rec_big), count=False)
        r.step(count=False)
        r.build.sync()
        info = r.build.native.info()
        assert info[6] == 1, info.tolist()  # the middle step ran again
        e_new = len(oracle_graph(rec, n)["a"])
        assert len(oracle_graph(rec_big, n)["a"]) != e_new  # the big reads add edges
        assert int(info[1]) == e_new, (info.tolist(), e_new)
        prof_o, cols_o = oracle_profile(r.blob, r.offs, 0, n)
        assert int(info[0]) == len(cols_o)
        assert np.array_equal(r.build.native.profile().numpy().view(np.uint64), prof_o.view(np.uint64))
    finally:
        d_big.close()
        r.close()


@pytest.mark.parametrize("fault_seq", [4, 5])
def test_failed_deferred_step_leaves_control_block_zeroed(monkeypatch, fault_seq):
    """A deferred step that fails after its records job and tail kernels ran
    (KARMA_STEP_FAULT_SEQ: the error path before the status kernel, which is
    what clears the tail's own control block) must leave that block zeroed:
    the next deferred jobs on the same tail take it as such.  Later deferred
    steps' profile and edges stay bit-exact (ADVICE r05, step.hip FailGuard)."""
    monkeypatch.setenv("KARMA_STEP_FAULT_SEQ", str(fault_seq))
    n = 3000
    rec = engine.synth_records(SEED, n, 0, 200_000, True)
    r = Run(n, rec, n_rate=0)
    try:
        failed = 0
        for _ in range(fault_seq + 4):  # both main streams' tails run again after the failure
            try:
                r.step(count=False)
            except _lib.KarmaError as e:
                assert "injected fault" in str(e)
                failed += 1
        assert failed == 1
        r.build.sync()
        info = r.build.native.info()
        assert info[6] == 0, info.tolist()  # no stale flag asked for a re-run
        o = oracle_graph(rec, n)
        e, deferred = r.build.native.newest_edges()
        assert deferred
        check_edges(e, o)
        prof_o, _ = oracle_profile(r.blob, r.offs, 0, n)
        assert np.array_equal(r.build.native.profile().numpy().view(np.uint64), prof_o.view(np.uint64))
    finally:
        r.close()
