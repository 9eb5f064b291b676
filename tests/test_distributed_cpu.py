"""World-size-2 gloo test of the sharded build's exchange logic (CPU only).

karma_amd.distributed.ShardedBuild is the production driver; here its compute
backend is an oracle-backed CPU implementation of the same ops interface
(presence bytes in the HIP ordinal layout, exception keys in the karma.h key
encoding, sorted (a << 32 | b, count) pair lists), so what is under test is the
sharding, the presence MAX-allreduce, the exception all-gather, the pair
all-to-all-v to contig owners, the owned-totals all-gather and the owner-side
weights.  The result must equal a single-process oracle run bit for bit.
"""
import os
import socket
from collections import OrderedDict

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from karma_amd import engine  # noqa: E402  (host-only synth functions)
from karma_amd.distributed import Comm, ShardedBuild  # noqa: E402
from oracle import oracle  # noqa: E402

KMODE_5P6 = -1


def ordinal_space(kmode):
    return 5120 if kmode == KMODE_5P6 else 4 ** kmode


def key_of(kmer: bytes, kmode):
    k = 0
    for j, b in enumerate(kmer):
        k |= b << (56 - 8 * j)
    return k if kmode == 8 else k | len(kmer)


def ordinal_of(kmer: bytes, kmode):
    code = 0
    for b in kmer:
        code = code * 4 + b"ACGT".index(bytes([b]))
    if kmode != KMODE_5P6:
        return code
    return code * 5 if len(kmer) == 5 else (code >> 2) * 5 + 1 + (code & 3)


def kmers_of(seq: bytes, kmode):
    if kmode == KMODE_5P6:
        out = [seq[i:i + 5] for i in range(len(seq) - 4)]
        out += [seq[i:i + 6] for i in range(len(seq) - 5) if seq[i:i + 6] == seq[i:i + 6][::-1]]
        return out
    return [seq[i:i + kmode] for i in range(len(seq) - kmode + 1)]


def decode_key(k, kmode):
    ln = 8 if kmode == 8 else k & 0xFF
    return k.to_bytes(8, "big")[:ln]


class OracleOps:
    """CPU implementation of the HipOps interface (test backend)."""

    def kmer_plan(self, store, kmode):
        return {"seqs": store, "kmode": kmode}

    def presence_bytes(self, plan):
        S = ordinal_space(plan["kmode"])
        pres = np.zeros(S, np.uint8)
        exc = set()
        for s in plan["seqs"].values():
            for km in kmers_of(s.encode("latin-1"), plan["kmode"]):
                if all(c in b"ACGT" for c in km):
                    pres[ordinal_of(km, plan["kmode"])] = 1
                else:
                    exc.add(key_of(km, plan["kmode"]))
        plan["exc"] = sorted(exc)
        return torch.from_numpy(pres)

    def set_presence_bytes(self, plan, pres):
        plan["pres"] = pres.numpy().copy()

    def exceptions(self, plan):
        return torch.tensor([np.int64(np.uint64(k).view(np.int64)) for k in plan["exc"]], dtype=torch.int64)

    def set_exceptions(self, plan, keys):
        plan["exc_all"] = sorted(set(int(np.int64(k).view(np.uint64)) for k in keys.tolist()))

    def finalize(self, plan):
        kmode = plan["kmode"]
        keys = set(plan["exc_all"])
        for o in np.flatnonzero(plan["pres"]):
            if kmode == KMODE_5P6:
                q, r = divmod(int(o), 5)
                code, ln = (q, 5) if r == 0 else ((q << 2) | (r - 1), 6)
            else:
                code, ln = int(o), kmode
            km = bytes(b"ACGT"[(code >> (2 * (ln - 1 - j))) & 3] for j in range(ln))
            keys.add(key_of(km, kmode))
        plan["cols"] = sorted(keys)
        return len(plan["cols"])

    def profile_buffer(self, n, M):
        return torch.zeros((n, M), dtype=torch.float64)

    def profile(self, plan, out):
        seqs = plan["seqs"]
        blob, offs, key_len = oracle.pack_sequences(seqs)
        M = len(plan["cols"])
        raw = np.zeros(max(M, 1) * oracle.KEY_BYTES, np.uint8)
        for i, k in enumerate(plan["cols"]):
            b = decode_key(k, plan["kmode"])
            raw[i * 16] = len(b)
            raw[i * 16 + 1: i * 16 + 1 + len(b)] = np.frombuffer(b, np.uint8)
        prof = np.zeros((len(seqs), M), np.float64)
        import ctypes
        rc = oracle.lib().oracle_kmer_profile(
            blob.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            key_len.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(seqs), plan["kmode"],
            raw.ctypes.data_as(ctypes.c_void_p), M, prof.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), None)
        assert rc == 0
        out.copy_(torch.from_numpy(prof))

    def columns(self, plan):
        return plan["cols"]

    def graph_local(self, records, n_records, n_contigs):
        r = np.asarray(records, np.int64)
        starts = np.flatnonzero(np.r_[True, r[1:, 0] != r[:-1, 0]]) if len(r) else np.zeros(0, np.int64)
        g = oracle.graph_groups(np.r_[starts, len(r)], r[:, 1] if len(r) else [], None, None, n_contigs, dedup=True)
        keys = [(int(a) << 32) | int(b) for a, b in zip(g["a"], g["b"])]
        counts = list(g["shared"])
        for c in np.flatnonzero(g["totals"]):
            keys.append((int(c) << 32) | int(c))
            counts.append(int(g["totals"][c]))
        order = np.argsort(np.array(keys, np.uint64), kind="stable")
        return {"keys": np.array(keys, np.uint64)[order], "counts": np.array(counts, np.int64)[order]}

    def pairs_split(self, pairs, bounds):
        starts = np.searchsorted(pairs["keys"], np.asarray(bounds, np.uint64) << np.uint64(32))
        return (torch.from_numpy(pairs["keys"].view(np.int64).copy()), torch.from_numpy(pairs["counts"].copy()),
                starts)

    def pairs_kc_split(self, pairs, bounds):
        keys, counts, starts = self.pairs_split(pairs, bounds)
        return torch.stack([keys, counts], 1), starts

    def merge_kc(self, kc, runs):
        kc = kc.reshape(-1, 2)
        return self.merge(kc[:, 0].contiguous(), kc[:, 1].contiguous(), runs)

    def merge(self, keys, counts, runs):
        k = keys.numpy().view(np.uint64)
        # the contract of karma_pairs_merge_runs: one sorted slice per sender
        off = np.r_[0, np.cumsum(runs)]
        assert off[-1] == len(k) and all(np.all(k[off[r] + 1:off[r + 1]] >= k[off[r]:off[r + 1] - 1])
                                         for r in range(len(runs)))
        u, inv = np.unique(k, return_inverse=True)
        c = np.zeros(len(u), np.int64)
        np.add.at(c, inv, counts.numpy())
        return {"keys": u, "counts": c}

    def totals(self, pairs, n):
        t = np.zeros(n, np.int64)
        a = (pairs["keys"] >> np.uint64(32)).astype(np.int64)
        b = (pairs["keys"] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        d = a == b
        t[a[d]] = pairs["counts"][d]
        return torch.from_numpy(t)

    def edges(self, pairs, n, totals=None):
        tot = self.totals(pairs, n).numpy() if totals is None else totals.numpy()
        a = (pairs["keys"] >> np.uint64(32)).astype(np.int64)
        b = (pairs["keys"] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        keep = (a != b) & (pairs["counts"] != 0)
        a, b, s = a[keep], b[keep], pairs["counts"][keep]
        w = (s / tot[a] + s / tot[b]) / 2  # numpy f64 division is IEEE
        return {"a": a, "b": b, "shared": s, "weight": w, "totals": tot}

    def edge_count(self, e):
        return len(e["a"])

    def edge_arrays(self, e):
        return e

    def entries(self, pairs):
        return int(pairs["counts"].sum())

    def pair_count(self, pairs):
        return len(pairs["keys"])

    def close(self, *objs):
        pass


N_LOC, F_LOC, SEED, NRATE = 150, 4000, 17, 40


def shard_inputs(rank, world):
    n_glob = N_LOC * world
    blob, offs, key_len = engine.synth_contigs(SEED, N_LOC, 20, 300, NRATE, first=rank * N_LOC)
    seqs = OrderedDict((f">ctg{rank * N_LOC + i}", bytes(blob[offs[i]:offs[i + 1]]).decode())
                       for i in range(N_LOC))
    genes = engine.synth_genes(SEED, n_glob)
    rec = engine.synth_records(SEED, n_glob, rank * F_LOC, (rank + 1) * F_LOC, True, genes=genes)
    return seqs, rec


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    comm = Comm.create(world, rank, backend="gloo")
    seqs, rec = shard_inputs(rank, world)
    build = ShardedBuild(None, comm, KMODE_5P6, N_LOC * world, rank * N_LOC, N_LOC, ops=OracleOps())
    res = build.run(seqs, rec, len(rec), keep=True)
    e = res["edges"]
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), profile=res["profile"].numpy(),
             cols=np.array(res["columns"], np.uint64), a=e["a"], b=e["b"], w=e["weight"], s=e["shared"],
             tot=e["totals"])
    comm.close()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_build_world2_matches_single_process(tmp_path):
    world = 2
    torch.multiprocessing.spawn(_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    # single-process reference on the union of the shards
    all_seqs, all_rec = OrderedDict(), []
    for r in range(world):
        s, rec = shard_inputs(r, world)
        all_seqs.update(s)
        all_rec.append(rec)
    rec = np.concatenate(all_rec).astype(np.int64)
    prof, cols, _ = oracle.calc_kmer_profile(all_seqs, "5p6")
    # every rank derived the same global column set ...
    for p in parts:
        assert [decode_key(int(k), KMODE_5P6).decode("latin-1") for k in p["cols"]] == cols
    # ... and wrote its own rows
    got = np.concatenate([p["profile"] for p in parts])
    assert np.array_equal(got.view(np.uint64), prof.view(np.uint64))
    # edges: rank r owns a in [r*N_LOC, (r+1)*N_LOC); union == global graph
    starts = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    o = oracle.graph_groups(np.r_[starts, len(rec)], rec[:, 1], None, None, N_LOC * world, dedup=True)
    a = np.concatenate([p["a"] for p in parts])
    b = np.concatenate([p["b"] for p in parts])
    w = np.concatenate([p["w"] for p in parts])
    assert np.array_equal(a, o["a"]) and np.array_equal(b, o["b"])
    assert np.array_equal(w.view(np.uint64), o["weight"].view(np.uint64))
    for r, p in enumerate(parts):
        assert np.all((p["a"] >= r * N_LOC) & (p["a"] < (r + 1) * N_LOC))
        assert np.array_equal(p["tot"], o["totals"])
    # the exchange is real: some fragments of each rank touch the other rank's contigs
    assert len(np.unique(a // N_LOC)) == world
