"""Two GPU ranks (one process each, sharing cuda:0, gloo with host staging)
through the production ShardedBuild + HipOps path; the union of the ranks'
outputs must equal the single-process oracle bit for bit."""
import os
import socket
from collections import OrderedDict

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

N_LOC, F_LOC, SEED, NRATE = 700, 60_000, 23, 300


def _inputs(rank, world):
    from karma_amd import engine
    n_glob = N_LOC * world
    blob, offs, key_len = engine.synth_contigs(SEED, N_LOC, 30, 900, NRATE, first=rank * N_LOC)
    genes = engine.synth_genes(SEED, n_glob)
    rec = engine.synth_records(SEED, n_glob, rank * F_LOC, (rank + 1) * F_LOC, True, genes=genes)
    return blob, offs, key_len, rec


def _worker(rank, world, port, out_dir, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from karma_amd import _lib, engine
    from karma_amd.distributed import Comm, ShardedBuild
    comm = Comm.create(world, rank, backend="gloo")
    torch.cuda.set_device(0)
    ctx = _lib.Context(0)
    blob, offs, key_len, rec = _inputs(rank, world)
    # overlap: the local graph build runs concurrently on a second context;
    # otherwise the default order (profile on the side stream beside the
    # graph's tail and the exchange)
    build = ShardedBuild(ctx, comm, -1, N_LOC * world, rank * N_LOC, N_LOC, overlap=overlap)
    store = engine.ContigStore(ctx, blob, offs, key_len)
    rec_dev = torch.from_numpy(rec.view(np.int64).reshape(-1)).to(build.ops.dev)
    res = build.run(store, rec_dev.data_ptr(), len(rec), keep=True)
    e = res["edges"]
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), profile=res["profile"].cpu().numpy(),
             cols=res["columns"], a=e.a, b=e.b, w=e.weight, tot=e.totals)
    store.close()
    comm.close()


@pytest.mark.parametrize("overlap", [True, False])
def test_two_gpu_ranks_match_oracle(tmp_path, overlap):
    from karma_amd import engine
    from oracle import oracle
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    torch.multiprocessing.spawn(_worker, args=(world, port, str(tmp_path), overlap), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
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
    # gives the same bytes as the sequential build
    from karma_amd import _lib, engine
    from karma_amd.distributed import Comm, ShardedBuild
    comm = Comm.create(1, 0)
    ctx = _lib.Context(0)
    blob, offs, key_len, rec = _inputs(0, 1)
    store = engine.ContigStore(ctx, blob, offs, key_len)
    outs = []
    for overlap in (False, True):
        build = ShardedBuild(ctx, comm, -1, N_LOC, 0, N_LOC, overlap=overlap)
        rec_dev = torch.from_numpy(rec.view(np.int64).reshape(-1)).to(build.ops.dev)
        res = build.run(store, rec_dev.data_ptr(), len(rec), keep=True)
        e = res["edges"]
        outs.append([res["profile"].cpu().numpy().copy(), np.array(e.a), np.array(e.b), np.array(e.weight),
                     np.array(e.totals)])
        build.close()
    for x, y in zip(*outs):
        assert x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    assert len(outs[0][1]) > 0
    store.close()
    ctx.close()
