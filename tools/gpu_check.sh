#!/bin/bash
# GPU box: GPU tests, consumer bench, default bench and a kernel trace of the bench.
# Usage: tools/gpu_check.sh TAG  -> gpurun_out/{pytest,consumers,bench}_TAG.*, gpurun_out/prof_TAG/
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
OUT=$REPO/gpurun_out
mkdir -p $OUT
cd $REPO
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
if [ -z "$SKIP_CONSUMERS" ]; then
timeout -k 10 300 python tools/bench_consumers.py > $OUT/consumers_$TAG.json 2> $OUT/consumers_$TAG.err || { echo "consumers failed"; tail $OUT/consumers_$TAG.err; exit 1; }
cat $OUT/consumers_$TAG.json
fi
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-timing > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
head -25 $OUT/prof_$TAG/trace_kernel_stats.csv | cut -d, -f1-5
