#!/bin/bash
# rocprofv3 collection for bench.py (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats.  Passes 2-3: PMC counters in their own runs
# (never combined with other trace domains).  Output under gpurun_out/prof_*.
set -e
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-config3}
OUT=${PROF_OUT:-$REPO/gpurun_out}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o trace --output-format csv -- \
    python3 $REPO/bench.py --config $CFG --steps 5 --warmup 2 --cpu-baseline off --no-e2e --no-timing > $OUT/prof_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_pmc1 -o pmc --output-format csv -- \
    python3 $REPO/bench.py --config $CFG --steps 2 --warmup 1 --cpu-baseline off --no-e2e --no-timing > $OUT/prof_pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_pmc2 -o pmc --output-format csv -- \
    python3 $REPO/bench.py --config $CFG --steps 2 --warmup 1 --cpu-baseline off --no-e2e --no-timing > $OUT/prof_pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d $OUT/prof_pmc3 -o pmc --output-format csv -- \
    python3 $REPO/bench.py --config $CFG --steps 2 --warmup 1 --cpu-baseline off --no-e2e --no-timing > $OUT/prof_pmc3.log 2>&1
echo done
