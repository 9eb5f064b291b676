"""bench.py's own rank launcher (CPU): `--gpus N > 1` with no WORLD_SIZE in
the environment starts N rank processes itself, as torchrun would, and never
reports an N-GPU line from fewer visible devices (VERDICT r04 "next" #1)."""
import importlib.util
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_rank_envs_are_what_torchrun_sets():
    b = load_bench()
    envs = b.rank_envs(3, 23456, base={"KEEP": "1", "RANK": "stale"})
    assert len(envs) == 3
    for r, e in enumerate(envs):
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "23456"
        assert e["KARMA_BENCH_LAUNCHER"] == "self" and e["KEEP"] == "1"


def test_launch_ranks_children_see_their_environment(tmp_path):
    b = load_bench()
    code = ("import json, os, sys; keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'); "
            "json.dump({k: os.environ[k] for k in keys}, open(os.path.join(sys.argv[1], os.environ['RANK']), 'w'))")
    port = b.free_port()
    rc = b.launch_ranks(4, [sys.executable, "-c", code, str(tmp_path)], b.rank_envs(4, port))
    assert rc == 0
    for r in range(4):
        e = json.load(open(tmp_path / str(r)))
        assert e == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "4", "MASTER_ADDR": "127.0.0.1",
                     "MASTER_PORT": str(port)}


def test_launch_ranks_failing_rank_stops_the_others():
    """Rank 1 fails at once; rank 0 would wait 60 s (a peer stuck in a
    collective): the launcher returns rank 1's code and ends rank 0 now."""
    b = load_bench()
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(60) if r == 0 else sys.exit(7)"
    t0 = time.time()
    rc = b.launch_ranks(2, [sys.executable, "-c", code], b.rank_envs(2, b.free_port()))
    assert rc == 7
    assert time.time() - t0 < 30


def test_bench_refuses_more_gpus_than_visible():
    """No HIP device in this container: `bench.py --gpus 8` must exit non-zero
    with a message, not run one rank and print an n_gpus line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "KARMA_FORCE_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode != 0
    assert "HIP device(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_self_launch_under_a_profiler():
    """Under rocprofv3 (ROCPROF_* in the environment) the process may already
    have initialised the GPU: `bench.py --gpus 2` must not fork + exec rank
    processes from it, but exit with a message."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "KARMA_FORCE_DEVICE")}
    env["ROCPROF_KERNEL_TRACE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 2
    assert "under a profiler" in r.stderr
    assert "launching" not in r.stderr
