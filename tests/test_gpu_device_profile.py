"""Device-resident profile hand-off (kmer.py:283-290).

KmerClustering.calc_kmer_profile_device() leaves the profile in HBM as a
DeviceProfile.  Checked here:
  * same side effects and errors as __calc_kmer_profile, and its host copy is
    bit-identical to the drop-in's host profile and to the oracle;
  * the zero-copy exports: __cuda_array_interface__ fields, and DLPack into a
    GPU consumer (torch, in a child process so that torch's HIP runtime is the
    only one there: torch is a consumer here, not part of the product) sees
    the same device pointer, bit-identical values, and keeps the memory alive
    after the producer handle is closed; a GPU kNN over it (the first step of
    UMAP) agrees with the host kNN over the reference-format profile.
"""
import os
import subprocess
import sys
from collections import OrderedDict

import numpy as np
import pytest

from karma_amd import engine
from karma_amd.kmer import KmerClustering
from oracle import oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seqs(seed=41, n=700):
    blob, offs, _ = engine.synth_contigs(seed, n, 30, 900, 200)
    return OrderedDict((f">ctg{i}", bytes(blob[offs[i]:offs[i + 1]]).decode()) for i in range(n))


def test_device_profile_matches_host_and_oracle():
    seqs = _seqs()
    kh = KmerClustering(seqs, "/tmp", "5p6", 4)
    host = kh._KmerClustering__calc_kmer_profile()
    kd = KmerClustering(seqs, "/tmp", "5p6", 4)
    dev = kd.calc_kmer_profile_device()
    assert kd.kmers == kh.kmers and kd.sorted_kmer_set == [] == kh.sorted_kmer_set
    assert dev.shape == host.shape and dev.columns == list(kh.kmers)
    got = dev.numpy()
    assert np.array_equal(got.view(np.uint64), host.view(np.uint64))
    oprof, ocols, _ = oracle.calc_kmer_profile(seqs, "5p6")
    assert np.array_equal(got.view(np.uint64), oprof.view(np.uint64))
    cai = dev.__cuda_array_interface__
    assert cai["shape"] == host.shape and cai["typestr"] == "<f8" and cai["data"][0] == dev.ptr != 0
    assert cai["strides"] is None and cai["version"] == 3
    assert dev.__dlpack_device__() == (10, 0)
    dev.close()
    with pytest.raises(ValueError):
        dev.numpy()


def test_device_profile_errors_match_reference():
    with pytest.raises(SystemExit):  # kmer.py:250-258: a contig shorter than k
        KmerClustering(OrderedDict([(">a", "ACGTACGT"), (">b", "AC")]), "/tmp", 5, 1).calc_kmer_profile_device()
    with pytest.raises(ZeroDivisionError):  # a zero-length FASTA key
        KmerClustering(OrderedDict([("", "ACGTACGT")]), "/tmp", 5, 1).calc_kmer_profile_device()


CHILD = r"""
import sys
import numpy as np
import torch                      # first: its HIP runtime serves libkarma_hip.so too
sys.path.insert(0, sys.argv[1])
from collections import OrderedDict
from karma_amd import engine
from karma_amd.kmer import KmerClustering
blob, offs, _ = engine.synth_contigs(43, 3000, 300, 900, 0)
seqs = OrderedDict((f">ctg{i}", bytes(blob[offs[i]:offs[i + 1]]).decode()) for i in range(3000))
host = KmerClustering(seqs, "/tmp", "5p6", 4)._KmerClustering__calc_kmer_profile()
dev = KmerClustering(seqs, "/tmp", "5p6", 4).calc_kmer_profile_device()
t = torch.from_dlpack(dev)
assert t.is_cuda and t.dtype == torch.float64 and tuple(t.shape) == host.shape, (t.device, t.dtype, t.shape)
assert t.data_ptr() == dev.ptr, "DLPack export copied the profile"
dev.close()                       # the consumer tensor keeps the memory alive
torch.cuda.synchronize()
assert np.array_equal(t.cpu().numpy().view(np.uint64), host.view(np.uint64))
# first step of UMAP on the device: exact 15-NN by squared Euclidean distance
k = 15
x = t
d = (x * x).sum(1)[:, None] + (x * x).sum(1)[None, :] - 2.0 * (x @ x.T)
d.fill_diagonal_(float("inf"))
gd, gi = torch.topk(d, k, dim=1, largest=False)
h = host
hd = (h * h).sum(1)[:, None] + (h * h).sum(1)[None, :] - 2.0 * (h @ h.T)
np.fill_diagonal(hd, np.inf)
hi = np.argsort(hd, axis=1, kind="stable")[:, :k]
hd_k = np.take_along_axis(hd, hi, 1)
assert np.allclose(gd.cpu().numpy(), hd_k, rtol=1e-9, atol=1e-12)
agree = (np.sort(gi.cpu().numpy(), 1) == np.sort(hi, 1)).all(1).mean()
assert agree > 0.99, agree        # rows with distance ties at the k-th place may differ
print("ok", t.shape, agree)
"""


def test_dlpack_zero_copy_into_torch_consumer():
    p = subprocess.run([sys.executable, "-c", CHILD, REPO], capture_output=True, text=True, timeout=300)
    if "No module named 'torch'" in p.stderr:
        pytest.skip("torch not importable")
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.startswith("ok")


def test_streamed_profile_into_memmap(tmp_path):
    """SURVEY.md §8(e) C5 streaming: the host profile filled one row block at a
    time into a caller's numpy.memmap (KmerClustering.__calc_kmer_profile(out=)),
    bit-identical to the one-piece profile and the oracle."""
    from collections import OrderedDict

    from karma_amd import engine
    from karma_amd.kmer import KmerClustering
    from oracle import oracle

    blob, offs, key_len = engine.synth_contigs(31, 3000, 20, 900, 40)
    seqs = OrderedDict((f">c{i}", bytes(blob[offs[i]:offs[i + 1]]).decode("latin-1")) for i in range(3000))
    for k in ("5p6", 7):
        whole, cols, tot = engine.kmer_profile(seqs, k)
        mm = np.lib.format.open_memmap(str(tmp_path / f"p{k}.npy"), mode="w+", dtype=np.float64, shape=whole.shape)
        got, cols2, tot2 = engine.kmer_profile(seqs, k, out=mm, block_bytes=whole.shape[1] * 8 * 701)
        assert got is mm and cols2 == cols and np.array_equal(tot2, tot)
        assert np.array_equal(np.asarray(mm).view(np.uint64), whole.view(np.uint64))
        oprof, ocols, _ = oracle.calc_kmer_profile(seqs, k)
        assert ocols == cols and np.array_equal(whole.view(np.uint64), oprof.view(np.uint64))
    kc = KmerClustering(seqs, str(tmp_path), "5p6", 4)
    out = np.lib.format.open_memmap(str(tmp_path / "kc.npy"), mode="w+", dtype=np.float64,
                                    shape=(3000, kc.columns_count()))
    res = kc._KmerClustering__calc_kmer_profile(out=out)
    assert res is out and len(kc.kmers) == out.shape[1]
    ref = KmerClustering(seqs, str(tmp_path), "5p6", 4)._KmerClustering__calc_kmer_profile()
    assert np.array_equal(np.asarray(out).view(np.uint64), ref.view(np.uint64))


def test_config5_profile_streamed_in_row_blocks():
    """BASELINE configs[4] (1M contigs, k = 7, a 131 GB profile) streamed to the
    host in 8192-row blocks (1 GB each, a ring of 12 host buffers, blocks hashed
    on a thread pool): the block digests equal the oracle's (tests/golden/
    digests.json config5_1gpu).  Device memory holds one block, not the profile."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor

    import digests as D
    from karma_amd import engine

    g = D.load()["config5_1gpu"]
    assert g["N"] == 1_000_000 and g["kmer"] == 7
    packed = engine.synth_contigs(5, g["N"], 400, 800, 0)  # bench.make_inputs' contigs of config5_1gpu

    class Packed(dict):  # the store's input as is (FastaDict-style), no Python strings
        karma_packed = packed

    ring = 12
    cols, blocks = engine.kmer_profile_blocks(Packed(), 7, D.BLOCK_ROWS, ring=ring)
    assert len(cols) == g["M"] and D.columns_digest(cols) == g["columns"]
    digs, pend = [], []
    with ThreadPoolExecutor(ring - 2) as pool:
        for lo, hi, blk in blocks:
            pend.append(pool.submit(lambda m: hashlib.sha256(m).digest(), memoryview(blk).cast("B")))
            while len(pend) > ring - 2:  # a block is hashed before its buffer comes round again
                digs.append(pend.pop(0).result())
        digs += [f.result() for f in pend]
    assert len(digs) == -(-g["N"] // D.BLOCK_ROWS)
    assert hashlib.sha256(b"".join(digs)).hexdigest() == g["profile_blocks"]
