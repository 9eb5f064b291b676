"""Multi-rank CPU tests of the sharded build's exchange logic (no GPU, no torch).

karma_amd.distributed.ShardedBuild is the production driver; here its compute
backend is an oracle-backed CPU implementation of the same ops interface
(presence bytes in the HIP ordinal layout, exception keys in the karma.h key
encoding, sorted (a << 32 | b, count) pair lists), so what is under test is the
sharding, the presence all-gather + OR merge, the exception all-gather, the
pair all-to-all-v to contig owners, the owned-totals all-gather and the
owner-side weights, over the host-staged transport (karma_amd/comm.py HostComm)
with ranks as processes (TCP star, karma_amd/hostgroup.py SocketGroup) or as
threads (ThreadGroup).  The result must equal a single-process oracle run bit
for bit.
"""
import multiprocessing as mp
import os
import socket
from collections import OrderedDict

import numpy as np
import pytest

from karma_amd import engine  # host-only synth functions
from karma_amd.comm import HostComm
from karma_amd.distributed import ShardedBuild
from karma_amd.hostgroup import SocketGroup, ThreadGroup, run_ranks
from oracle import oracle

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

    def presence_words(self, plan):
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
        plan["pres"] = pres
        return np.packbits(pres, bitorder="little").view(np.uint32).copy()

    def presence_merge(self, plan, all_words, n_sets):
        w = np.bitwise_or.reduce(np.asarray(all_words, np.uint32).reshape(n_sets, -1), axis=0)
        plan["pres"] = np.unpackbits(w.view(np.uint8), bitorder="little")[: ordinal_space(plan["kmode"])]

    def exceptions(self, plan):
        return np.array(plan["exc"], np.uint64)

    def set_exceptions(self, plan, keys):
        plan["exc_all"] = sorted(set(int(k) for k in np.asarray(keys, np.uint64).tolist()))

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
        return np.zeros((n, M), dtype=np.float64)

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
        out[...] = prof

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

    def pairs_kc_split(self, pairs, bounds):
        starts = np.searchsorted(pairs["keys"], np.asarray(bounds, np.uint64) << np.uint64(32))
        kc = np.stack([pairs["keys"].view(np.int64), pairs["counts"]], 1).reshape(-1)
        return kc, starts

    def merge_kc(self, kc, runs):
        kc = np.asarray(kc, np.int64).reshape(-1, 2)
        return self.merge(kc[:, 0].copy(), kc[:, 1].copy(), runs)

    # the production exchange: keys and counts as two arrays (alltoallv_kv)
    def pairs_kv(self, pairs, bounds):
        starts = np.searchsorted(pairs["keys"], np.asarray(bounds, np.uint64) << np.uint64(32))
        return pairs["keys"].view(np.int64), pairs["counts"], starts

    def merge_kv(self, keys, counts, runs):
        return self.merge(np.asarray(keys, np.int64).copy(), np.asarray(counts, np.int64).copy(), list(runs))

    def merge(self, keys, counts, runs):
        k = keys.view(np.uint64)
        # the contract of karma_pairs_merge_runs: one sorted slice per sender
        off = np.r_[0, np.cumsum(runs)]
        assert off[-1] == len(k) and all(np.all(k[off[r] + 1:off[r + 1]] >= k[off[r]:off[r + 1] - 1])
                                         for r in range(len(runs)))
        u, inv = np.unique(k, return_inverse=True)
        c = np.zeros(len(u), np.int64)
        np.add.at(c, inv, counts)
        return {"keys": u, "counts": c}

    def totals(self, pairs, n):
        t = np.zeros(n, np.int64)
        a = (pairs["keys"] >> np.uint64(32)).astype(np.int64)
        b = (pairs["keys"] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        d = a == b
        t[a[d]] = pairs["counts"][d]
        return t

    def edges(self, pairs, n, totals=None):
        tot = self.totals(pairs, n) if totals is None else np.asarray(totals)
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


def run_rank(group, rank):
    comm = HostComm(group)
    world = group.world
    seqs, rec = shard_inputs(rank, world)
    build = ShardedBuild(None, comm, KMODE_5P6, N_LOC * world, rank * N_LOC, N_LOC, ops=OracleOps())
    res = build.run(seqs, rec, len(rec), keep=True)
    e = res["edges"]
    return dict(profile=res["profile"], cols=np.array(res["columns"], np.uint64), a=e["a"], b=e["b"],
                w=e["weight"], s=e["shared"], tot=e["totals"])


def _proc_worker(rank, world, port, out_dir):
    g = SocketGroup(world, rank, "127.0.0.1", port)
    out = run_rank(g, rank)
    g.close()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_union(parts, world):
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
    # the exchange is real: some fragments of each rank touch the other ranks' contigs
    assert len(np.unique(a // N_LOC)) == world


def test_sharded_build_world2_processes_match_single_process(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_proc_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    check_union([dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)], world)


@pytest.mark.parametrize("world", [3, 4, 8])
def test_sharded_build_thread_ranks_match_single_process(world):
    check_union(run_ranks(world, run_rank), world)


@pytest.mark.parametrize("kind", ["threads", "sockets"])
def test_host_comm_collectives(kind, tmp_path):
    world = 3

    def body(group, rank):
        c = HostComm(group)
        out = {}
        out["max"] = c.max_float(rank * 1.5)
        out["sum"] = c.sum_int(rank + 1)
        out["fixed"] = c.allgather_fixed(np.full(4, rank, np.uint32))
        out["var"] = c.allgather_var(np.arange(rank, dtype=np.int64))
        bounds = np.array([0, 2, 2, 7])
        buf = np.full(7, -1, np.int64)
        buf[bounds[rank]:bounds[rank + 1]] = 10 * rank + np.arange(bounds[rank + 1] - bounds[rank])
        out["slices"] = c.allgather_slices_(buf, bounds).copy()
        send = np.concatenate([np.full(r + 1, 100 * rank + r, np.int64) for r in range(world)])
        out["a2a"], out["recv"] = c.alltoallv(send, [r + 1 for r in range(world)])
        ka, kb, out["recv_kv"] = c.alltoallv_kv(send, -send, [r + 1 for r in range(world)])
        out["kv_ok"] = bool(np.array_equal(ka, out["a2a"]) and np.array_equal(kb, -out["a2a"]))
        c.barrier()
        return out

    if kind == "threads":
        outs = run_ranks(world, body)
    else:
        port = free_port()
        import threading
        outs = [None] * world

        def t(r):
            g = SocketGroup(world, r, "127.0.0.1", port)
            outs[r] = body(g, r)
            g.close()

        ts = [threading.Thread(target=t, args=(r,)) for r in range(world)]
        for x in ts:
            x.start()
        for x in ts:
            x.join(60)
    for r, o in enumerate(outs):
        assert o["max"] == 3.0 and o["sum"] == 6
        assert np.array_equal(o["fixed"], np.repeat(np.arange(world, dtype=np.uint32), 4))
        assert np.array_equal(o["var"], np.array([0, 0, 1], np.int64))
        assert np.array_equal(o["slices"], np.array([0, 1, 20, 21, 22, 23, 24], np.int64))
        assert o["recv"] == [r + 1] * world
        assert o["recv_kv"] == o["recv"] and o["kv_ok"]
        assert np.array_equal(o["a2a"], np.concatenate([np.full(r + 1, 100 * s + r) for s in range(world)]))


def test_socket_group_moves_off_a_taken_port(tmp_path):
    """MASTER_PORT + 1 held by a foreign listener: rank 0 listens on a free port
    and publishes it through the handshake file; the others find it there.  The
    foreign listener (no hello) is never taken for rank 0."""
    import threading

    base = free_port()
    squat = socket.socket()
    squat.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    squat.bind(("127.0.0.1", base))
    squat.listen(8)
    hs = str(tmp_path / "group.port")
    world, outs = 3, [None] * 3

    def t(r):
        g = SocketGroup(world, r, "127.0.0.1", base, timeout=30, handshake=hs)
        outs[r] = [int(x[0]) for x in g.allgather(np.array([10 + r]))]
        g.close()

    ts = [threading.Thread(target=t, args=(r,)) for r in range(world)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(60)
    squat.close()
    assert outs == [[10, 11, 12]] * world
    assert not os.path.exists(hs)  # rank 0 removes it at close


def test_socket_group_taken_port_fails_fast_without_handshake():
    base = free_port()
    squat = socket.socket()
    squat.bind(("127.0.0.1", base))
    squat.listen(1)
    import time as _t

    t0 = _t.time()
    with pytest.raises(OSError, match="KARMA_GROUP_PORT"):
        SocketGroup(2, 0, "127.0.0.1", base, timeout=30)
    assert _t.time() - t0 < 5
    squat.close()


def test_socket_group_duplicate_rank_fails_fast():
    """Two processes launched with the same RANK: rank 0 names the duplicate at
    once instead of waiting out the connect timeout (a valid hello with a rank
    the job already holds, or one outside the world size)."""
    import struct
    import threading
    import time as _t

    from karma_amd.hostgroup import _HELLO

    port = free_port()
    err = []

    def serve():
        try:
            SocketGroup(3, 0, "127.0.0.1", port, timeout=30)
        except ConnectionError as e:
            err.append(str(e))

    t = threading.Thread(target=serve)
    t0 = _t.time()
    t.start()
    socks = []
    for r in (1, 1):  # the second hello repeats rank 1
        while True:
            try:
                s = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                _t.sleep(0.05)
        s.sendall(_HELLO + struct.pack("<i", r))
        socks.append(s)
    t.join(20)
    for s in socks:
        s.close()
    assert err and "duplicate" in err[0] and "rank 1" in err[0]
    assert _t.time() - t0 < 10


def test_socket_group_port_fallback_only_for_single_node(monkeypatch):
    """The handshake file (rank 0's fallback port) is local: a job whose ranks
    are not all on this node keeps the fixed port (LOCAL_WORLD_SIZE < WORLD_SIZE)."""
    seen = {}

    def fake_init(self, world, rank, addr="127.0.0.1", port=29600, timeout=120.0, handshake=None):
        seen["handshake"] = handshake

    monkeypatch.setattr(SocketGroup, "__init__", fake_init)
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.delenv("KARMA_GROUP_PORT", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    SocketGroup.from_env(8, 1)
    assert seen["handshake"] is None
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    SocketGroup.from_env(8, 1)
    assert seen["handshake"] is not None
