"""The RCCL group error paths of csrc/comm.hip, on the CPU.

karma_comm_alltoallv and karma_comm_exchange_counts queue their sends and
receives inside ncclGroupStart/ncclGroupEnd.  An error return from inside the
group would leave it open, and the next NCCL call on the thread would join it:
a hang on the other ranks, not an error.  comm_group.h validates every argument
before the group starts and closes the group on every path; this test drives
it against a scripted NCCL (comm_group_test.cpp: failing send/recv at several
positions, a failing ncclGroupEnd, an early return, bad all-to-all-v offsets)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "karma_amd", "csrc")


def test_nccl_group_always_closed():
    subprocess.run(["make", "-C", CSRC, "comm_group_test"], check=True, capture_output=True)
    r = subprocess.run([os.path.join(CSRC, "build", "comm_group_test")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().startswith("ok")


def test_comm_sources_use_the_guarded_group():
    # no bare ncclGroupStart/End (and so no early return inside a group) in comm.hip
    src = open(os.path.join(CSRC, "comm.hip")).read()
    assert "ncclGroupStart" not in src and "ncclGroupEnd" not in src
    assert src.count("NcclGroup g;") == 3  # count exchange, alltoallv, alltoallv_kv


def test_fake_rccl_double_builds_and_exports_the_bound_entry_points():
    """tools/fake_rccl/librccl.so.1 (the multi-rank test double, GPU tests only)
    provides every RCCL symbol libkarma_hip.so imports, under RCCL's soname."""
    import ctypes
    import subprocess

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(repo, "karma_amd", "csrc"), "fake_rccl"], check=True)
    fake = os.path.join(repo, "tools", "fake_rccl", "librccl.so.1")
    lib = ctypes.CDLL(fake)
    assert lib.fake_rccl_marker() == 0x7ACE
    need = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(repo, "karma_amd", "libkarma_hip.so")],
                          capture_output=True, text=True, check=True).stdout
    imported = sorted({ln.split()[-1] for ln in need.splitlines() if " nccl" in ln or ln.split()[-1].startswith("nccl")})
    assert len(imported) >= 10
    for name in imported:
        assert hasattr(lib, name), name
    soname = subprocess.run(["readelf", "-d", fake], capture_output=True, text=True, check=True).stdout
    assert "librccl.so.1" in soname
