"""GPU ranks sharing cuda:0 through the production ShardedBuild + HipOps path.

RCCL refuses two ranks on one device, so on the one-GPU box the ranks are
threads of one process, each with its own karma context and streams, and the
exchange goes through the host-staged transport (karma_amd/comm.py HostComm
over a ThreadGroup).  Everything else -- presence bitmaps, exception keys, the
device split, the wire format, the owner's merge, totals, weights -- is the
production code.  The union of the ranks' outputs must equal the
single-process oracle bit for bit."""
import subprocess
import sys
from collections import OrderedDict

import numpy as np
import pytest

from karma_amd import _lib, engine
from karma_amd.comm import HostComm, SoloComm
from karma_amd.distributed import ShardedBuild
from karma_amd.hostgroup import run_ranks
from oracle import oracle

pytestmark = pytest.mark.gpu

N_LOC, F_LOC, SEED, NRATE = 700, 60_000, 23, 300


def _inputs(rank, world):
    n_glob = N_LOC * world
    blob, offs, key_len = engine.synth_contigs(SEED, N_LOC, 30, 900, NRATE, first=rank * N_LOC)
    genes = engine.synth_genes(SEED, n_glob)
    rec = engine.synth_records(SEED, n_glob, rank * F_LOC, (rank + 1) * F_LOC, True, genes=genes)
    return blob, offs, key_len, rec


def _rank(group, rank, overlap):
    world = group.world
    ctx = _lib.Context(0)
    try:
        comm = HostComm(group)
        blob, offs, key_len, rec = _inputs(rank, world)
        # overlap: the local graph build runs concurrently on a second context;
        # otherwise the default order (profile on the side stream beside the
        # graph's tail and the exchange)
        build = ShardedBuild(ctx, comm, -1, N_LOC * world, rank * N_LOC, N_LOC, overlap=overlap)
        store = engine.ContigStore(ctx, blob, offs, key_len)
        rec_dev = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
        res = build.run(store, rec_dev.ptr, len(rec), keep=True)
        e = res["edges"]
        out = dict(profile=res["profile"].numpy(), cols=res["columns"], a=e.a, b=e.b, w=e.weight, tot=e.totals)
        build.close()
        store.close()
        rec_dev.close()
        return out
    finally:
        ctx.close()


@pytest.mark.parametrize("world,overlap", [(2, True), (2, False), (3, False)])
def test_gpu_ranks_match_oracle(world, overlap):
    parts = run_ranks(world, _rank, overlap)
    seqs, recs = OrderedDict(), []
    for r in range(world):
        blob, offs, _, rec = _inputs(r, world)
        for i in range(N_LOC):
            seqs[f">ctg{r * N_LOC + i}"] = bytes(blob[offs[i]:offs[i + 1]]).decode()
        recs.append(rec)
    prof, cols, _ = oracle.calc_kmer_profile(seqs, "5p6")
    for p in parts:
        assert engine.decode_keys(p["cols"], -1) == cols
    got = np.concatenate([p["profile"] for p in parts])
    assert np.array_equal(got.view(np.uint64), prof.view(np.uint64))
    rec = np.concatenate(recs).astype(np.int64)
    st = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    o = oracle.graph_groups(np.r_[st, len(rec)], rec[:, 1], None, None, N_LOC * world, dedup=True)
    a = np.concatenate([p["a"] for p in parts])
    b = np.concatenate([p["b"] for p in parts])
    w = np.concatenate([p["w"] for p in parts])
    assert np.array_equal(a, o["a"]) and np.array_equal(b, o["b"])
    assert np.array_equal(w.view(np.uint64), o["weight"].view(np.uint64))
    for p in parts:
        assert np.array_equal(p["tot"], o["totals"])


def test_overlap_equals_sequential_single_gpu():
    # the graph build on a second context/stream, concurrent with the profile,
    # gives the same bytes as the sequential and the side-stream builds
    ctx = _lib.Context(0)
    blob, offs, key_len, rec = _inputs(0, 1)
    store = engine.ContigStore(ctx, blob, offs, key_len)
    rec_dev = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
    outs = []
    for overlap, sequential in ((False, False), (True, False), (False, True)):
        build = ShardedBuild(ctx, SoloComm(), -1, N_LOC, 0, N_LOC, overlap=overlap)
        res = build.run(store, rec_dev.ptr, len(rec), keep=True, sequential=sequential)
        e = res["edges"]
        outs.append([res["profile"].numpy(), np.array(e.a), np.array(e.b), np.array(e.weight), np.array(e.totals)])
        build.close()
    for other in outs[1:]:
        for x, y in zip(outs[0], other):
            assert x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    assert len(outs[0][1]) > 0
    store.close()
    rec_dev.close()
    ctx.close()


def test_product_path_never_imports_torch():
    # north_star: no PyTorch on this path -- the drop-in classes, the sharded
    # driver and the bench run with torch absent from sys.modules
    code = (
        "import sys; sys.path.insert(0, '.')\n"
        "from collections import OrderedDict\n"
        "from karma_amd import engine, _lib\n"
        "from karma_amd.kmer import KmerClustering\n"
        "from karma_amd.read_graph import ReadGraph\n"
        "from karma_amd.distributed import ShardedBuild\n"
        "from karma_amd.comm import SoloComm\n"
        "import numpy as np\n"
        "blob, offs, kl = engine.synth_contigs(3, 200, 50, 500, 0)\n"
        "seqs = OrderedDict((f'>ctg{i}', bytes(blob[offs[i]:offs[i+1]]).decode()) for i in range(200))\n"
        "KmerClustering(seqs, '/tmp', '5p6', 2)._KmerClustering__calc_kmer_profile()\n"
        "ctx = _lib.Context(0)\n"
        "rec = engine.synth_records(3, 200, 0, 5000, True)\n"
        "b = ShardedBuild(ctx, SoloComm(), -1, 200, 0, 200)\n"
        "st = engine.ContigStore(ctx, blob, offs, kl)\n"
        "d = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))\n"
        "b.run(st, d.ptr, len(rec)); b.close()\n"
        "assert 'torch' not in sys.modules, 'torch was imported'\n"
        "print('no-torch ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "no-torch ok" in r.stdout


class _OneRankGroup:
    """The bootstrap group of a one-rank job (the unique id needs no exchange)."""

    world, rank = 1, 0

    def allgather(self, arr):
        return [np.asarray(arr)]

    def close(self):
        pass


def test_rccl_comm_world1_calls():
    """The library's RCCL communicator at world size 1: every call the sharded
    build makes (host-scalar reduces through mapped memory, the count exchange,
    the all-to-all-v own slice, all-gathers) returns its input unchanged."""
    from karma_amd.comm import RcclComm

    ctx = _lib.Context(0)
    comm = RcclComm(_OneRankGroup(), ctx)
    try:
        comm.barrier()
        assert comm.max_float(2.5) == 2.5
        assert comm.sum_int(7) == 7
        src = np.arange(2 * 1000, dtype=np.int64)
        buf = _lib.DevBuf.from_numpy(ctx, src)
        out, recv = comm.alltoallv(buf, [src.size])
        assert recv == [src.size]
        np.testing.assert_array_equal(out.numpy(), src)
        neg = _lib.DevBuf.from_numpy(ctx, -src)
        ka, kb, recv2 = comm.alltoallv_kv(buf, neg, [src.size])
        assert recv2 == [src.size]
        np.testing.assert_array_equal(ka.numpy(), src)
        np.testing.assert_array_equal(kb.numpy(), -src)
        for b in (neg, ka, kb):
            b.close()
        g = comm.allgather_fixed(buf)
        np.testing.assert_array_equal(g.numpy(), src)
        v = comm.allgather_var(_lib.DevBuf.from_numpy(ctx, src[:17]))
        np.testing.assert_array_equal(v.numpy(), src[:17])
        for b in (buf, out, g, v):
            b.close()
    finally:
        comm.close()
        ctx.close()


def _free_port_pair():
    import socket
    for _ in range(50):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
        if p >= 65535:
            continue
        try:
            with socket.socket() as s2:
                s2.bind(("127.0.0.1", p + 1))  # hostgroup's bootstrap port (MASTER_PORT + 1)
            return p
        except OSError:
            continue
    raise RuntimeError("no free port pair")


def _bench_two_ranks(*extra, timeout=240):
    """bench.py under the driver's launch (`python -m torch.distributed.run
    --nproc-per-node 2 ... bench.py --gpus 2`), both ranks on the one device:
    bootstrap through hostgroup, exchange through the host-staged transport
    (RCCL refuses two ranks on one device).  Returns the one JSON line."""
    import json
    import os

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KARMA_FORCE_DEVICE="0", KARMA_DIST_BACKEND="host")
    port = _free_port_pair()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(repo, "bench.py"), "--gpus", "2", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_under_torch_distributed_run_two_ranks():
    """Rank 0 prints exactly one JSON line: the strong headline (BASELINE
    configs[3] shape) with the whole-job value, and the weak leg as an extra key."""
    res = _bench_two_ranks("--steps", "2", "--warmup", "1", "--config", "tiny")
    assert res["n_gpus"] == 2 and res["steps"] == 2 and res["scaling"] == "strong"
    assert res["value"] > 0 and res["ms_per_step"] > 0
    assert res["weak"]["scaling"] == "weak" and res["weak"]["value"] > 0
    assert res["config"]["contigs_rank0"] == 2500  # tiny's 5,000 contigs split 2 ways
    assert res["build"]["defines"] == ""


def test_bench_strong_config3_two_ranks_in_run_parity():
    """The driver's N > 1 headline on BASELINE configs[3]'s workload split over
    2 ranks: bench.py's in-run digest check (every rank hashes its profile rows,
    rank 0 combines them with the ranks' edges and totals) must match
    tests/golden/digests.json config3 -- the oracle's digests, which the
    reference's own config-3 outputs also match."""
    res = _bench_two_ranks("--steps", "1", "--warmup", "1", "--no-weak-leg", "--no-timing", "--cpu-baseline", "off",
                           timeout=600)
    assert res["scaling"] == "strong" and res["config"]["contigs_rank0"] == 100_000
    d = res["parity_detail"]
    assert res["parity"] is True, d
    assert d["ranks"] == 2 and d["edges"] == 199_510 and d["mismatch"] == []


_RCCL_RANK = r"""
import os, sys
sys.path.insert(0, os.environ["KARMA_REPO"])
import numpy as np
from karma_amd import _lib, engine, comm as comm_mod
from karma_amd.distributed import ShardedBuild
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
sizes = [int(x) for x in os.environ["KARMA_SHARDS"].split(",")]
n_glob, c_lo, n_loc = sum(sizes), sum(sizes[:rank]), sizes[rank]
F = int(os.environ["KARMA_FRAGS"])
ctx = _lib.Context(rank)
comm = comm_mod.create(ctx, world, rank, backend="rccl")
blob, offs, key_len = engine.synth_contigs(29, n_loc, 30, 900, 300, first=c_lo)
genes = engine.synth_genes(29, n_glob)
f_lo, f_hi = F * rank // world, F * (rank + 1) // world
rec = engine.synth_records(29, n_glob, f_lo, f_hi, True, genes=genes)
build = ShardedBuild(ctx, comm, -1, n_glob, c_lo, n_loc)
store = engine.ContigStore(ctx, blob, offs, key_len)
rec_dev = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
res = build.run(store, rec_dev.ptr, len(rec), keep=True)
e = res["edges"]
np.savez(os.path.join(os.environ["KARMA_OUT"], f"rank{rank}.npz"), profile=res["profile"].numpy(),
         cols=res["columns"], a=e.a, b=e.b, w=e.weight, tot=e.totals)
build.close(); store.close(); rec_dev.close(); comm.close(); ctx.close()
"""


def test_rccl_ranks_on_separate_devices_match_oracle(tmp_path):
    """The library's RCCL communicator across real ranks (one process and one
    GPU each): unequal contig shards (the padded all-gather of the exception
    keys and the non-in-place totals all-gather), the grouped key/count
    all-to-all-v, the owners' merge; the union must equal the single-process
    oracle bit for bit.  Needs >= 2 GPUs: skipped on a one-GPU box (there the
    driver's multi-GPU bench runs the same exchange with its in-run parity
    check)."""
    import ctypes
    import os

    n = ctypes.c_int(0)
    _lib.load().karma_device_count(ctypes.byref(n))
    if n.value < 2:
        pytest.skip("needs >= 2 GPUs")
    world = min(n.value, 4)
    sizes = [700 + 131 * r for r in range(world)]
    frags = 50_000 * world
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port_pair()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), KARMA_REPO=repo, KARMA_OUT=str(tmp_path),
                   KARMA_SHARDS=",".join(map(str, sizes)), KARMA_FRAGS=str(frags))
        procs.append(subprocess.Popen([sys.executable, "-c", _RCCL_RANK], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    n_glob = sum(sizes)
    seqs, recs = OrderedDict(), []
    genes = engine.synth_genes(29, n_glob)
    lo = 0
    for r in range(world):
        blob, offs, _ = engine.synth_contigs(29, sizes[r], 30, 900, 300, first=lo)
        for i in range(sizes[r]):
            seqs[f">ctg{lo + i}"] = bytes(blob[offs[i]:offs[i + 1]]).decode()
        lo += sizes[r]
        recs.append(engine.synth_records(29, n_glob, frags * r // world, frags * (r + 1) // world, True, genes=genes))
    prof, cols, _ = oracle.calc_kmer_profile(seqs, "5p6")
    for p in parts:
        assert engine.decode_keys(p["cols"], -1) == cols
    got = np.concatenate([p["profile"] for p in parts])
    assert np.array_equal(got.view(np.uint64), prof.view(np.uint64))
    rec = np.concatenate(recs).astype(np.int64)
    st = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    o = oracle.graph_groups(np.r_[st, len(rec)], rec[:, 1], None, None, n_glob, dedup=True)
    a = np.concatenate([p["a"] for p in parts])
    b = np.concatenate([p["b"] for p in parts])
    w = np.concatenate([p["w"] for p in parts])
    assert np.array_equal(a, o["a"]) and np.array_equal(b, o["b"])
    assert np.array_equal(w.view(np.uint64), o["weight"].view(np.uint64))
    for p in parts:
        assert np.array_equal(p["tot"], o["totals"])
