"""Host parsers (csrc/ingest.cpp) against the reference's goldens
(tests/golden/ingest.json, made by make_golden_ingest.py) and the oracle's
restatements on seeded random texts.  CPU only: the parsers are host code in
libkarma_hip.so (loading it needs no GPU)."""
import json
import os
import random

import numpy as np
import pytest

from karma_amd import contig, engine, fasta, ingest, read_graph
from oracle import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ingest.json")))

EXC = {"UnicodeDecodeError": UnicodeDecodeError, "ValueError": ValueError, "KeyError": KeyError,
       "AssertionError": AssertionError}


def _write(tmp_path, name, data):
    p = tmp_path / name
    p.write_bytes(data)
    return str(p)


# ---------------------------------------------------------------- FASTA ----
@pytest.mark.parametrize("case", list(GOLD["fasta"]))
def test_fasta_golden(tmp_path, case):
    g = GOLD["fasta"][case]
    data = bytes.fromhex(g["hex"])
    path = _write(tmp_path, "x.fa", data)
    if "raises" in g["out"]:
        with pytest.raises(EXC[g["out"]["raises"]]):
            fasta.read_fasta_file(path)
        with pytest.raises(ingest.ParseDeferred):
            ingest.parse_fasta(data)
        return
    got = fasta.read_fasta_file(path)
    assert [[k, v] for k, v in got.items()] == g["out"]["items"]
    rec = ingest.parse_fasta(data)  # the C++ reader itself decided (no deferral)
    assert rec.names() == [k for k, _ in g["out"]["items"]]
    assert rec.sequences() == [v for _, v in g["out"]["items"]]
    assert rec.key_len.tolist() == [len(k) for k, _ in g["out"]["items"]]


def _rand_fasta(rng, n):
    alpha = ["A", "C", "G", "T", "N", "a", " ", "\t", ">", "é", "\x00"]
    nl = ["\n", "\r\n", "\r"]
    out = []
    if rng.random() < 0.1:
        out.append("".join(rng.choice(alpha) for _ in range(rng.randrange(6))) + rng.choice(nl))
    for _ in range(n):
        name = "".join(rng.choice("abcé x") for _ in range(rng.randrange(1, 5)))
        out.append(">" + name + rng.choice(nl))
        for _ in range(rng.randrange(4)):
            line = "".join(rng.choice(alpha[:6] if rng.random() < 0.8 else alpha) for _ in range(rng.randrange(12)))
            if line.startswith(">") and rng.random() < 0.5:
                line = "A" + line
            out.append(line + rng.choice(nl))
    s = "".join(out)
    if s and rng.random() < 0.3:
        s = s.rstrip("\r\n")
    return s.encode("utf-8")


@pytest.mark.parametrize("seed", range(40))
def test_fasta_random_vs_oracle(tmp_path, seed):
    rng = random.Random(seed)
    data = _rand_fasta(rng, rng.randrange(0, 30))
    path = _write(tmp_path, "r.fa", data)
    want = oracle.read_fasta_file(path)
    rec = ingest.parse_fasta(data, threads=1 + seed % 4)
    assert rec.names() == list(want.keys())
    assert rec.sequences() == list(want.values())
    assert rec.key_len.tolist() == [len(k) for k in want]
    got = fasta.read_fasta_file(path)
    assert list(got.items()) == list(want.items())


def test_fasta_threads_and_packed(tmp_path):
    rng = random.Random(7)
    parts = []
    for i in range(20000):
        parts.append(f">ctg{i} len\n")
        seq = "".join(rng.choice("ACGTN") for _ in range(rng.randrange(1, 300)))
        parts += [seq[j:j + 60] + "\n" for j in range(0, len(seq), 60)]
    data = "".join(parts).encode()
    one, many = ingest.parse_fasta(data, threads=1), ingest.parse_fasta(data, threads=8)
    assert np.array_equal(one.seq, many.seq) and np.array_equal(one.seq_off, many.seq_off)
    assert one.keys == many.keys and np.array_equal(one.key_len, many.key_len)
    path = _write(tmp_path, "big.fa", data)
    d = fasta.read_fasta_file(path)
    assert len(d) == 20000 and d.karma_packed is not None
    blob, offs, key_len = d.karma_packed
    vals = list(d.values())
    for i in (0, 1, 9999, 19999):
        assert bytes(blob[offs[i]:offs[i + 1]]).decode() == vals[i]
    assert key_len.tolist() == [len(k) for k in d]
    d[">new"] = "ACGT"  # any mutation drops the packed arrays
    assert d.karma_packed is None


# ------------------------------------------------------------- eq classes ----
def _eq_compact_matches(data, wide):
    """ingest.parse_eq(compact=True): the karma_graph_eq_compact form of the
    same classes when every class fits it, else the wide form."""
    names, off, mem, cnt, skip = wide
    q = ingest.parse_eq(data, compact=True)
    want = engine.eq_compact(off, cnt, skip)
    if want is None:
        assert q.sizes is None
        _eq_arrays_equal((q.names, q.cls_off, q.members, q.counts, q.pair_skip), wide)
        return False
    assert q.cls_off is None and list(q.names) == list(names)
    assert np.array_equal(q.sizes, want[0]) and np.array_equal(q.counts32, want[1])
    assert np.array_equal(q.members, mem[:off[-1]])
    return True


def _eq_arrays_equal(a, b):
    names_a, off_a, mem_a, cnt_a, skip_a = a
    names_b, off_b, mem_b, cnt_b, skip_b = b
    assert list(names_a) == list(names_b)
    assert np.array_equal(off_a, off_b)
    assert np.array_equal(mem_a[:off_a[-1]], mem_b[:off_b[-1]])
    assert np.array_equal(cnt_a, cnt_b) and np.array_equal(skip_a, skip_b)


@pytest.mark.parametrize("case", list(GOLD["eq"]))
def test_eq_parse_golden(tmp_path, case):
    g = GOLD["eq"][case]
    data = bytes.fromhex(g["hex"])
    path = _write(tmp_path, "eq.txt", data)
    raises = g["out"].get("raises")
    if raises is not None:
        try:
            oracle.parse_eq_file(path)
        except Exception as e:  # the failure is the parse's (not the graph build's)
            with pytest.raises(type(e)):
                read_graph.parse_eq_classes(path)
            return
    want = oracle.parse_eq_file(path)
    _eq_arrays_equal(read_graph.parse_eq_classes(path), want)
    q = ingest.parse_eq(data)  # accepted by the C++ parser itself
    _eq_arrays_equal((q.names, q.cls_off, q.members, q.counts, q.pair_skip), want)
    _eq_compact_matches(data, want)
    if raises is None:
        assert q.names == [n for n in g["out"]["nodes"][:len(q.names)]]


def _rand_eq(rng, n, c):
    nl = rng.choice(["\n", "\r\n", "\r"])
    lines = [str(n), str(c)] + [f"t{i}é" if i % 5 == 0 else f"t{i}" for i in range(n)]
    for _ in range(c):
        k = rng.randrange(1, 6)
        ids = [str(rng.randrange(n)) for _ in range(k)]
        size = str(k) if rng.random() < 0.9 else rng.choice(["1", "01", "x"])
        cnt = rng.choice([str(rng.randrange(0, 10**6)), f"+{rng.randrange(9)}", f" {rng.randrange(50)}",
                          "1_000", f"-{rng.randrange(3)}"])
        lines.append("\t".join([size] + ids + [cnt]))
    return (nl.join(lines) + (nl if rng.random() < 0.8 else "")).encode()


@pytest.mark.parametrize("seed", range(25))
def test_eq_random_vs_oracle(tmp_path, seed):
    rng = random.Random(100 + seed)
    data = _rand_eq(rng, rng.randrange(1, 40), rng.randrange(0, 300))
    path = _write(tmp_path, "eq.txt", data)
    want = oracle.parse_eq_file(path)
    q = ingest.parse_eq(data, threads=1 + seed % 8)
    _eq_arrays_equal((q.names, q.cls_off, q.members, q.counts, q.pair_skip), want)


@pytest.mark.parametrize("big", [0, 127, 128])
def test_eq_compact_form(tmp_path, big):
    """The parser's compact form (karma_eq_get_compact): sizes with the size
    token "1" in bit 7 and u32 counts, equal to the wide form's; a class of
    128 members or a count past 2^32 - 1 falls back to the wide form."""
    rng = random.Random(7 + big)
    n = 300
    lines = [str(n), "0"] + [f"t{i}" for i in range(n)]
    for c in range(2000):
        k = rng.randrange(1, 6)
        ids = [str(rng.randrange(n)) for _ in range(k)]
        size = "1" if rng.random() < 0.05 else str(k)
        lines.append("\t".join([size] + ids + [str(rng.randrange(0, 4_000_000_000))]))
    if big:
        lines.append("\t".join([str(big)] + [str(rng.randrange(n)) for _ in range(big)] + ["3"]))
    data = ("\n".join(lines) + "\n").encode()
    path = _write(tmp_path, "eq.txt", data)
    want = oracle.parse_eq_file(path)
    assert _eq_compact_matches(data, want) == (big <= 127)
    big_count = data.replace(b"\t3\n", b"\t4294967296\n") if big else data + b"1\t0\t4294967296\n"
    assert not _eq_compact_matches(big_count, oracle.parse_eq_file(_write(tmp_path, "eq2.txt", big_count)))


def test_eq_threads_large():
    rng = random.Random(5)
    data = _rand_eq(rng, 5000, 200000)
    a, b = ingest.parse_eq(data, threads=1), ingest.parse_eq(data, threads=8)
    _eq_arrays_equal((a.names, a.cls_off, a.members, a.counts, a.pair_skip),
                     (b.names, b.cls_off, b.members, b.counts, b.pair_skip))


# -------------------------------------------------------------------- SAM ----
@pytest.mark.parametrize("case", list(GOLD["sam"]))
def test_sam_golden_readsets(case):
    g = GOLD["sam"][case]
    data = bytes.fromhex(g["hex"])
    if "raises" in g["out"]:
        with pytest.raises(EXC[g["out"]["raises"]]):
            contig.contigs_from_sam(data)
        return
    cs = contig.contigs_from_sam(data)
    assert [[c.name, sorted(c.readset)] for c in cs] == g["out"]["readsets"]


def _check_sam_records(data, rec):
    want = oracle.sam_groups(data.decode("utf-8"))
    assert rec.rnames == [n for n, _ in want]
    # the same QNAME <-> the same read id, per line in file order
    lines = [ln for ln in data.decode().replace("\r\n", "\n").replace("\r", "\n").split("\n")
             if ln and not ln.startswith("@")]
    assert len(lines) == len(rec.records)
    q2id = {}
    for ln, (rid, cid) in zip(lines, rec.records.tolist()):
        f = ln.split("\t")
        assert q2id.setdefault(f[0], rid) == rid
        assert rec.rnames[cid] == f[2]
    assert len(set(q2id.values())) == len(q2id) == rec.n_reads
    assert rec.records[:, 0].max(initial=0) < max(rec.read_id_bound, 1)
    # the readsets the records imply are the oracle's
    sets = [set() for _ in rec.rnames]
    inv = {v: k for k, v in q2id.items()}
    for rid, cid in rec.records.tolist():
        sets[cid].add(inv[rid])
    assert sets == [s for _, s in want]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_sam_random_vs_oracle(threads):
    rng = random.Random(threads)
    lines = ["@HD\tVN:1.6"]
    for i in range(30000):
        q = f"read{rng.randrange(8000)}"
        lines.append(f"{q}\t{rng.choice([0, 16])}\tctg{rng.randrange(300)}\t{rng.randrange(1, 900)}\t60\t*")
    data = ("\n".join(lines) + "\n").encode()
    rec = ingest.parse_sam(data, threads=threads)
    _check_sam_records(data, rec)
