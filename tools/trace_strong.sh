#!/bin/bash
# Kernel + HIP runtime + copy trace of the strong-scaling preview (one rank of
# config 3 over N emulated ranks), to locate host gaps.  GPU box.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/trace_strong${1:-8}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $OUT -o tr --output-format csv -- \
    python3 $REPO/bench.py --strong --emulate-ranks ${1:-8} --steps 5 --warmup 3 --cpu-baseline off --no-e2e --no-timing > $OUT.log 2>&1
