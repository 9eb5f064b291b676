"""The library's RCCL communicator at world size > 1 on a one-GPU box.

RCCL refuses several ranks on one device, so these tests start a child process
(tests/fake_rccl_ranks.py) whose ranks are threads sharing cuda:0 and whose
librccl.so.1 is tools/fake_rccl/ (a host-staged test double of the RCCL entry
points, ahead of ROCm's in LD_LIBRARY_PATH; libkarma_hip.so itself is the
shipped build, unchanged).  What runs is the product's multi-GPU code --
karma_amd/comm.py RcclComm and csrc/comm.hip, the one-communicator exchange
stream (and the optional side-stream communicator), the sharded driver -- so the only piece left unverified before a real
multi-GPU run is RCCL's own transport.  The child refuses to run (exit 3) if
the fake is not the librccl it loaded."""
import json
import os
import subprocess
import sys
from collections import OrderedDict

import numpy as np
import pytest

import digests as D
from karma_amd import engine
from oracle import oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE_DIR = os.path.join(REPO, "tools", "fake_rccl")


def run_child(*args, timeout=240):
    assert os.path.exists(os.path.join(FAKE_DIR, "librccl.so.1")), \
        "tools/fake_rccl/librccl.so.1 not built (make -C karma_amd/csrc fake_rccl)"
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = FAKE_DIR + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tests", "fake_rccl_ranks.py"), *args],
                       capture_output=True, text=True, timeout=timeout, cwd=REPO, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    out = json.loads(lines[-1])
    assert out["fake_rccl_loaded"], "the child did not load tools/fake_rccl/librccl.so.1"
    return out


@pytest.mark.parametrize("world", [2, 3, 8])
def test_rccl_comm_collectives_unequal_sizes(world):
    """Every RcclComm call with unequal per-rank sizes: host scalars, the fixed
    all-gather, the padded variable all-gather on the side communicator (rank 0
    empty), unequal and equal (in place) totals slices, the count exchange and
    the grouped key/count all-to-all-v (some slices empty)."""
    out = run_child("--case", "collectives", "--world", str(world))
    assert out["errors"] == []


def oracle_of(sizes, frags, seed, n_rate=300, len_span=900):
    """The single-process oracle's profile, columns and graph for the union of
    the ranks' shards (tests/fake_rccl_ranks.py builds the same inputs)."""
    n_glob = sum(sizes)
    seqs, recs = OrderedDict(), []
    genes = engine.synth_genes(seed, n_glob)
    lo = 0
    W = len(sizes)
    for r in range(W):
        blob, offs, _ = engine.synth_contigs(seed, sizes[r], 30, len_span, n_rate, first=lo)
        for i in range(sizes[r]):
            seqs[f">ctg{lo + i}"] = bytes(blob[offs[i]:offs[i + 1]]).decode()
        lo += sizes[r]
        recs.append(engine.synth_records(seed, n_glob, frags * r // W, frags * (r + 1) // W, True, genes=genes))
    prof, cols, _ = oracle.calc_kmer_profile(seqs, "5p6")
    rec = np.concatenate(recs).astype(np.int64)
    st = np.flatnonzero(np.r_[True, rec[1:, 0] != rec[:-1, 0]])
    o = oracle.graph_groups(np.r_[st, len(rec)], rec[:, 1], None, None, n_glob, dedup=True)
    return prof, cols, o


def check_graph(parts, o, pre=""):
    a = np.concatenate([p[pre + "a"] for p in parts])
    b = np.concatenate([p[pre + "b"] for p in parts])
    w = np.concatenate([p[pre + "w"] for p in parts])
    assert np.array_equal(a, o["a"]) and np.array_equal(b, o["b"])
    assert np.array_equal(w.view(np.uint64), o["weight"].view(np.uint64))
    for p in parts:
        assert np.array_equal(p[pre + "tot"], o["totals"])


def test_rccl_sharded_build_three_unequal_ranks_match_oracle(tmp_path):
    """The sharded build through RcclComm at world 3 with unequal contig shards
    and N-injected contigs (exception keys on every rank), two stream steps then
    a kept one: the union must equal the single-process oracle bit for bit."""
    sizes, frags, seed = [700, 831, 962], 150_000, 29
    run_child("--case", "oracle", "--world", "3", "--sizes", ",".join(map(str, sizes)), "--frags", str(frags),
              "--seed", str(seed), "--out", str(tmp_path))
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(3)]
    prof, cols, o = oracle_of(sizes, frags, seed)
    for p in parts:
        assert engine.decode_keys(p["cols"], -1) == cols
    got = np.concatenate([p["profile"] for p in parts])
    assert np.array_equal(got.view(np.uint64), prof.view(np.uint64))
    check_graph(parts, o)


DEFER_MODES = {
    # default: one communicator, every collective on the exchange stream
    "one_comm": ([], 1, 3),
    # one main stream (the config-3 batch size's mode): the tail still on the exchange stream
    "one_comm_one_stream": (["KARMA_STEP_STREAMS=1"], 1, 3),
    # round 4's mode: the presence all-gather on a side communicator, on the side stream
    "side_comm": (["KARMA_STEP_SIDE_COMM=1"], 0, 3),
    # the default mode on KARMA_REC_FLAGGED records (u32 contig | read-start flag)
    "one_comm_flagged": ([], 1, 3),
}


@pytest.mark.parametrize("world,mode", [(2, "one_comm"), (3, "one_comm"), (2, "one_comm_one_stream"),
                                        (3, "side_comm"), (3, "one_comm_flagged")])
def test_rccl_deferred_steps_rerun_on_slot_overflow(tmp_path, world, mode):
    """Deferred steps with several processes (csrc/step.hip run_deferred: the
    padded fixed-slot all-to-all, the merge from slots, the totals all-gather
    and the summed slow flag).  A first synchronous step on 1 % of the
    reads sizes the slots, so the three deferred full steps overflow them: every
    rank runs them again synchronously.  A second build sized on the full step
    defers three steps that fit (no re-run).  In a third, only rank 0's batches
    hold a read for the general path (12 records): its verdict reaches the
    other ranks in the slot headers, and every rank re-runs the three steps.  The newest profile after sync and
    the kept step after each must equal the oracle bit for bit (ACGT-only
    contigs: the deferred path needs no exception keys)."""
    sizes = [5000, 6000, 5500][:world]  # ~5000 distinct pairs per owner's slice
    frags, seed = 200_000, 31
    env, one_comm, xs = DEFER_MODES[mode]
    run_child("--case", "defer", "--world", str(world), "--sizes", ",".join(map(str, sizes)), "--frags",
              str(frags), "--seed", str(seed), "--out", str(tmp_path), *[x for e in env for x in ("--env", e)],
              *(["--flagged"] if mode.endswith("_flagged") else []))
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    prof, _, o = oracle_of(sizes, frags, seed, n_rate=0, len_span=100)
    # rank 0's batches in the third build carry one more read, of 12 records
    recs = [p["peer_rec"].astype(np.int64) for p in parts]
    st = np.concatenate([np.flatnonzero(np.r_[True, r[1:, 0] != r[:-1, 0]]) + sum(map(len, recs[:i]))
                         for i, r in enumerate(recs)])
    rec = np.concatenate(recs)
    o_peer = oracle.graph_groups(np.r_[st, len(rec)], rec[:, 1], None, None, sum(sizes), dedup=True)
    for tag in ("over", "fit", "peer"):
        infos = [p[f"{tag}_info"] for p in parts]
        # [M, E, pairs, entries, synchronous, deferred, re-run, pending, ...]
        for i in infos:
            assert i[5] == 3 and i[7] == 0, (tag, i.tolist())
            assert i[6] == (0 if tag == "fit" else 3), (tag, i.tolist())
            # the mode that ran: one communicator or not, tails on the exchange stream, the ranks
            assert (int(i[12]) & 1) == one_comm and i[11] == xs and i[13] == world, (mode, tag, i.tolist())
        got = np.concatenate([p[f"{tag}_profile"] for p in parts])
        assert np.array_equal(got.view(np.uint64), prof.view(np.uint64)), tag
        check_graph(parts, o_peer if tag == "peer" else o, tag + "_")
        # the newest step's own edges (karma_step_newest_edges): in "fit" the
        # deferred step's tail outputs (fixed-slot all-to-all, merge from
        # slots, device-sized edge stage), else the synchronous re-run's
        og = o_peer if tag == "peer" else o
        check_graph(parts, og, tag + "_n")
        s_cat = np.concatenate([p[f"{tag}_ns"] for p in parts])
        assert np.array_equal(s_cat, og["shared"]), tag
        for p in parts:
            assert bool(p[f"{tag}_ndeferred"]) == (tag == "fit"), tag


def test_rccl_config4_strong_8_ranks_digests():
    """BASELINE configs[3] through the library's RCCL communicator: config 3
    split over 8 ranks (bench.py's strong workload), the union of the ranks'
    outputs against digests.json config3 (the oracle's digests, which the
    reference's own config-3 outputs also match)."""
    g = D.load()["config3"]
    out = run_child("--case", "config4", "--world", "8", timeout=600)
    assert out["M"] == [g["M"]] and out["columns"] == [g["columns"]]
    assert out["profile_rows"] == g["profile_rows"]
    assert out["edges"] == g["edges"]
    assert out["totals_equal"] and out["owners_ok"]
