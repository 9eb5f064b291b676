#!/bin/bash
# One GPU call: GPU tests, smoke, default bench, rocprofv3 trace + PMC passes, summaries.
# Usage (GPU box): tools/round_gpu.sh TAG   -> gpurun_out/{pytest_gpu,smoke,bench}_TAG.*, gpurun_out/prof_*
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
OUT=$REPO/gpurun_out
mkdir -p $OUT
cd $REPO
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke_$TAG.log; exit 1; }
cat $OUT/smoke_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
[ -n "$SKIP_PROF" ] || bash tools/prof_gpu.sh config3
