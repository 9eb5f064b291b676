"""Child process of tests/test_gpu_fake_rccl.py (not a test module).

W ranks as threads of this one process, each with its own karma context on
cuda:0 and the library's RCCL communicator (karma_amd/comm.py RcclComm over
csrc/comm.hip) -- the communicator code a real multi-GPU job runs.  RCCL itself
refuses several ranks on one device, so the parent starts this process with
LD_LIBRARY_PATH pointing at tools/fake_rccl/ (a host-staged test double of the
RCCL entry points the library binds, ahead of ROCm's librccl in the search
order).  Everything else is the product: the presence all-gather (one
communicator on the exchange stream by default, the side communicator with
KARMA_STEP_SIDE_COMM=1), the padded variable all-gather of the exception keys, the count
exchange, the grouped key/count all-to-all-v, the owners' merge, the totals
all-gather (in place for equal shards, padded otherwise).

Cases (--case):
  collectives  every RcclComm call with unequal sizes, checked against numpy
  oracle       the sharded build over unequal contig shards; outputs to npz
               (the parent compares them with the single-process oracle)
  defer        deferred steps over RCCL (several processes): a first synchronous
               step on 1 % of the records sizes the exchange's slots, so
               the deferred full steps overflow them and run again; then a
               second build whose deferred steps fit; a third where only
               rank 0's batches hold a read for the general path; infos,
               newest profiles and kept results to npz
  config4      BASELINE configs[3]: config 3 over W ranks (bench.py's exact
               strong workload); the union of outputs hashed with
               tests/digests.py (the parent compares with digests.json config3)
Prints one JSON line.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

import numpy as np  # noqa: E402

from karma_amd import _lib, engine  # noqa: E402
from karma_amd.comm import RcclComm  # noqa: E402
from karma_amd.distributed import ShardedBuild  # noqa: E402
from karma_amd.hostgroup import run_ranks  # noqa: E402


def fake_loaded():
    with open("/proc/self/maps") as f:
        maps = f.read()
    return any("fake_rccl/librccl.so.1" in ln for ln in maps.splitlines())


def collectives(group, rank):
    world = group.world
    ctx = _lib.Context(0)
    comm = RcclComm(group, ctx)
    try:
        out = {}
        comm.barrier()
        out["max"] = comm.max_float(1.5 * rank)
        out["sum"] = comm.sum_int(rank + 1)
        fixed = _lib.DevBuf.from_numpy(ctx, np.full(5, 10 + rank, np.uint32))
        out["fixed"] = comm.allgather_fixed(fixed).numpy().tolist()
        # variable sizes, rank 0 empty (the padded all-gather + per-rank copies)
        mine = np.arange(3 * rank * rank, dtype=np.uint64) + 1000 * rank
        v = comm.side.allgather_var(_lib.DevBuf.from_numpy(ctx, mine) if mine.size else
                                    _lib.DevBuf(ctx, (0,), np.uint64))
        out["var"] = v.numpy().tolist()
        # unequal slices (not in place): rank r owns [bounds[r], bounds[r+1])
        sizes = [2 + 3 * r for r in range(world)]
        bounds = np.r_[0, np.cumsum(sizes)].astype(np.int64)
        host = np.full(int(bounds[-1]), -1, np.int64)
        host[bounds[rank]:bounds[rank + 1]] = 100 * rank + np.arange(sizes[rank])
        buf = _lib.DevBuf.from_numpy(ctx, host)
        out["slices"] = comm.allgather_slices_(buf, bounds).numpy().tolist()
        # equal slices (in place)
        eb = np.arange(world + 1, dtype=np.int64) * 4
        host = np.full(4 * world, -1, np.int64)
        host[4 * rank:4 * rank + 4] = 7 * rank
        out["slices_eq"] = comm.allgather_slices_(_lib.DevBuf.from_numpy(ctx, host), eb).numpy().tolist()
        # all-to-all-v of a key/count list: rank s sends (s + 1) * (r + 1) % 4 items to r
        cnt = [(rank + 1) * (r + 1) % 4 for r in range(world)]
        keys = np.concatenate([np.full(c, 1000 * rank + r, np.uint64) for r, c in enumerate(cnt)])
        vals = -keys.astype(np.int64)
        kd = _lib.DevBuf.from_numpy(ctx, keys) if keys.size else _lib.DevBuf(ctx, (0,), np.uint64)
        vd = _lib.DevBuf.from_numpy(ctx, vals) if vals.size else _lib.DevBuf(ctx, (0,), np.int64)
        rk, rv, recv = comm.alltoallv_kv(kd, vd, cnt)
        out["recv"] = recv
        out["rk"] = rk.numpy().tolist() if rk.size else []
        out["rv"] = rv.numpy().tolist() if rv.size else []
        ra, recv1 = comm.alltoallv(kd, cnt)
        out["a2a_same"] = (ra.numpy().tolist() if ra.size else []) == out["rk"] and recv1 == recv
        return out
    finally:
        comm.close()
        ctx.close()


def check_collectives(outs):
    world = len(outs)
    errs = []
    for r, o in enumerate(outs):
        if o["max"] != 1.5 * (world - 1) or o["sum"] != world * (world + 1) // 2:
            errs.append(f"rank {r}: scalars {o['max']}, {o['sum']}")
        if o["fixed"] != [10 + s for s in range(world) for _ in range(5)]:
            errs.append(f"rank {r}: allgather_fixed")
        var = [1000 * s + i for s in range(world) for i in range(3 * s * s)]
        if o["var"] != var:
            errs.append(f"rank {r}: allgather_var")
        sl = [100 * s + i for s in range(world) for i in range(2 + 3 * s)]
        if o["slices"] != sl:
            errs.append(f"rank {r}: allgather_slices_ (unequal)")
        if o["slices_eq"] != [7 * s for s in range(world) for _ in range(4)]:
            errs.append(f"rank {r}: allgather_slices_ (equal, in place)")
        cnt_in = [(s + 1) * (r + 1) % 4 for s in range(world)]
        if o["recv"] != cnt_in:
            errs.append(f"rank {r}: received counts {o['recv']} != {cnt_in}")
        rk = [1000 * s + r for s in range(world) for _ in range(cnt_in[s])]
        if o["rk"] != rk or o["rv"] != [-x for x in rk]:
            errs.append(f"rank {r}: all-to-all-v payload")
        if not o["a2a_same"]:
            errs.append(f"rank {r}: alltoallv != alltoallv_kv")
    return errs


def oracle_rank(group, rank, sizes, frags, seed):
    world = group.world
    n_glob, c_lo, n_loc = sum(sizes), sum(sizes[:rank]), sizes[rank]
    ctx = _lib.Context(0)
    comm = RcclComm(group, ctx)
    try:
        blob, offs, key_len = engine.synth_contigs(seed, n_loc, 30, 900, 300, first=c_lo)
        genes = engine.synth_genes(seed, n_glob)
        rec = engine.synth_records(seed, n_glob, frags * rank // world, frags * (rank + 1) // world, True,
                                   genes=genes)
        build = ShardedBuild(ctx, comm, -1, n_glob, c_lo, n_loc)
        store = engine.ContigStore(ctx, blob, offs, key_len)
        rec_dev = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
        try:
            for _ in range(2):  # a stream of steps, then the kept one
                build.run(store, rec_dev.ptr, len(rec), count=False)
            res = build.run(store, rec_dev.ptr, len(rec), keep=True)
            e = res["edges"]
            return dict(profile=res["profile"].numpy(), cols=res["columns"], a=e.a, b=e.b, w=e.weight, tot=e.totals)
        finally:
            build.close()
            store.close()
            rec_dev.close()
    finally:
        comm.close()
        ctx.close()


FLAGGED = False  # --flagged: the deferred case's records as KARMA_REC_FLAGGED words


def dev_records(ctx, rec):
    return _lib.DevBuf.from_numpy(ctx, engine.flag_records(rec) if FLAGGED else
                                  np.ascontiguousarray(rec).view(np.int64).reshape(-1))


def defer_rank(group, rank, sizes, frags, seed):
    world = group.world
    n_glob, c_lo, n_loc = sum(sizes), sum(sizes[:rank]), sizes[rank]
    ctx = _lib.Context(0)
    comm = RcclComm(group, ctx)
    out = {}
    try:
        blob, offs, key_len = engine.synth_contigs(seed, n_loc, 30, 100, 0, first=c_lo)
        genes = engine.synth_genes(seed, n_glob)
        rec = engine.synth_records(seed, n_glob, frags * rank // world, frags * (rank + 1) // world, True,
                                   genes=genes)
        # 1 % of the reads (records stay grouped by read)
        k = int(np.searchsorted(rec[:, 0], rec[len(rec) // 100, 0]))
        store = engine.ContigStore(ctx, blob, offs, key_len)
        full = dev_records(ctx, rec)
        small = dev_records(ctx, rec[:k])
        try:
            # rank 0 alone gets a read of 12 records (the general path): every
            # rank must run the deferred steps again
            rp = rec
            if rank == 0:
                big = np.stack([np.full(12, rec[-1, 0] + 1, np.uint32),
                                (np.arange(12, dtype=np.uint32) * 37) % n_glob], axis=1)
                rp = np.concatenate([rec, big])
            out["peer_rec"] = rp
            peer = dev_records(ctx, rp)
            for tag, first, batch in (("over", (small, k), (full, len(rec))), ("fit", (full, len(rec)), (full, len(rec))),
                                      ("peer", (peer, len(rp)), (peer, len(rp)))):
                build = ShardedBuild(ctx, comm, -1, n_glob, c_lo, n_loc, flagged=FLAGGED)
                try:
                    assert build.native is not None
                    build.run(store, first[0].ptr, first[1], count=False)  # synchronous: sizes the slots
                    for _ in range(3):
                        build.run(store, batch[0].ptr, batch[1], count=False)
                    build.sync()
                    out[f"{tag}_info"] = build.native.info()
                    out[f"{tag}_profile"] = build.native.profile().numpy()
                    # the newest step's edges: a deferred step's from its tail
                    # (slots, step_merge_kernel, step_edge_*), a re-run's synchronous
                    ne, dfr = build.native.newest_edges()
                    out.update({f"{tag}_na": ne.a, f"{tag}_nb": ne.b, f"{tag}_nw": ne.weight,
                                f"{tag}_ns": ne.shared, f"{tag}_ntot": ne.totals,
                                f"{tag}_ndeferred": np.array(dfr)})
                    res = build.run(store, batch[0].ptr, batch[1], keep=True)
                    e = res["edges"]
                    out.update({f"{tag}_a": e.a, f"{tag}_b": e.b, f"{tag}_w": e.weight, f"{tag}_tot": e.totals})
                finally:
                    build.close()
            return out
        finally:
            store.close()
            full.close()
            small.close()
            peer.close()
    finally:
        comm.close()
        ctx.close()


def config4_rank(group, rank):
    import digests as D

    world = group.world
    ctx = _lib.Context(0)
    comm = RcclComm(group, ctx)
    try:
        inp = D.bench_inputs("config3", rank=rank, world=world, strong=True)
        build = ShardedBuild(ctx, comm, engine.kmode_of(inp["kmer"]), inp["n_glob"], inp["c_lo"], inp["n_loc"])
        store = engine.ContigStore(ctx, inp["blob"], inp["offs"], inp["key_len"])
        rec_dev = _lib.DevBuf.from_numpy(ctx, inp["rec"].view(np.int64).reshape(-1))
        try:
            res = build.run(store, rec_dev.ptr, len(inp["rec"]), keep=True)
            e = res["edges"]
            return dict(M=int(res["M"]), cols=D.columns_digest(engine.decode_keys(res["columns"], -1)),
                        rows=D.row_digests(res["profile"].numpy()), c_lo=inp["c_lo"], n_loc=inp["n_loc"],
                        a=np.asarray(e.a), b=np.asarray(e.b), w=np.asarray(e.weight), s=np.asarray(e.shared),
                        tot=np.asarray(e.totals))
        finally:
            build.close()
            store.close()
            rec_dev.close()
    finally:
        comm.close()
        ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", choices=("collectives", "oracle", "defer", "config4"), required=True)
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--out", default=".")
    ap.add_argument("--sizes", default="")
    ap.add_argument("--frags", type=int, default=0)
    ap.add_argument("--seed", type=int, default=29)
    ap.add_argument("--flagged", action="store_true", help="defer case: KARMA_REC_FLAGGED records")
    ap.add_argument("--env", action="append", default=[],
                    help="KEY=VALUE set before the communicators and steps are created (mode A/B)")
    a = ap.parse_args()
    global FLAGGED
    FLAGGED = a.flagged
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    _lib.load()
    summary = {"fake_rccl_loaded": fake_loaded(), "case": a.case, "world": a.world}
    if not summary["fake_rccl_loaded"]:
        print(json.dumps(summary))
        return 3
    if a.case == "collectives":
        outs = run_ranks(a.world, collectives)
        summary["errors"] = check_collectives(outs)
    elif a.case in ("oracle", "defer"):
        sizes = [int(x) for x in a.sizes.split(",")]
        parts = run_ranks(a.world, oracle_rank if a.case == "oracle" else defer_rank, sizes, a.frags, a.seed)
        for r, p in enumerate(parts):
            np.savez(os.path.join(a.out, f"rank{r}.npz"), **p)
    else:
        import digests as D

        parts = run_ranks(a.world, config4_rank)
        order = np.argsort([p["c_lo"] for p in parts], kind="stable")
        summary["M"] = sorted({p["M"] for p in parts})
        summary["columns"] = sorted({p["cols"] for p in parts})
        summary["profile_rows"] = D.profile_rows_digest(rows=b"".join(parts[r]["rows"] for r in order))
        cat = {k: np.concatenate([parts[r][k] for r in order]) for k in ("a", "b", "w", "s")}
        summary["edges"] = D.edge_digests(cat["a"], cat["b"], cat["w"], cat["s"], parts[0]["tot"])
        summary["totals_equal"] = all(np.array_equal(p["tot"], parts[0]["tot"]) for p in parts)
        summary["owners_ok"] = all(bool(np.all((p["a"] >= p["c_lo"]) & (p["a"] < p["c_lo"] + p["n_loc"])))
                                   for p in parts)
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
