#!/bin/bash
# Round-6 GPU check: the deferred-path parity tests, then bench lines
# (config 3 at the driver's K = 20, the 8-rank strong preview at K = 20).
# Usage: tools/r06_check.sh TAG [PYTEST_K]   -> gpurun_out/TAG/
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
K=${2:-"deferred or step or rccl_deferred"}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 480 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py tests/test_gpu_configs.py \
    -k "$K" -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json 2>/dev/null || head -c 1500 $OUT/bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --emulate-ranks 8 > $OUT/emu8.json 2> $OUT/emu8.err || { echo "emu8 failed"; tail -30 $OUT/emu8.err; exit 1; }
python tools/summarize_bench.py $OUT/emu8.json 2>/dev/null || head -c 1500 $OUT/emu8.json
