"""The host parsers under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

`make -C karma_amd/csrc asan` builds karma_amd/csrc/fuzz_ingest.cpp with
ingest.cpp (karma_fasta_parse, karma_eq_parse, karma_sam_parse: karma.py:40-61,
read_graph.py:75-92, contig.py:24,34) under -fsanitize=address,undefined with
-fno-sanitize-recover=all, and with thread chunks small enough that random
texts of a few hundred bytes split over 2-8 threads.  The driver parses random
texts (CR/LF/CRLF mixes, NUL, valid and invalid UTF-8, signs, underscores, huge
counts, short and extra fields) at 1 thread and at 2-8 threads, reads every
output back, and aborts on any sanitizer report or any difference between the
two runs.  No GPU code is built or run.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "karma_amd", "csrc")


@pytest.fixture(scope="module")
def fuzzer():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.run(["make", "-C", CSRC, "asan"], check=True, capture_output=True)
    return os.path.join(CSRC, "build", "fuzz_ingest_asan")


@pytest.mark.parametrize("seed", [1, 2])
def test_parsers_clean_under_sanitizers(fuzzer, seed):
    env = dict(os.environ, ASAN_OPTIONS="allocator_may_return_null=1:detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([fuzzer, "1500", str(seed)], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "rounds clean" in p.stdout
    assert "runtime error" not in p.stderr
