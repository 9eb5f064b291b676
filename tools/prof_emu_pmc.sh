#!/bin/bash
# GPU box: kernel trace + FETCH_SIZE / WRITE_SIZE passes of the W-rank strong
# preview (bench.py --emulate-ranks W), summarised into gpurun_out/emu<W>/ and
# the PMC traffic table row config3_strong_n<W> (gpurun_out/emu<W>/pmc_traffic.json).
# Usage: tools/prof_emu_pmc.sh [W]
set -e
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
W=${1:-8}
OUT=$REPO/gpurun_out/emu$W
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --cpu-baseline off --no-e2e --no-timing --no-parity --emulate-ranks $W"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o trace --output-format csv -- \
    python3 $REPO/bench.py $ARGS > $OUT/prof_trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_pmc1 -o pmc --output-format csv -- \
    python3 $REPO/bench.py $ARGS > $OUT/prof_pmc1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_pmc2 -o pmc --output-format csv -- \
    python3 $REPO/bench.py $ARGS > $OUT/prof_pmc2.log 2>&1
cd $REPO
python profiles/pmc_summary.py $OUT --json $OUT/pmc_summary.json > $OUT/prof_summary.txt
python tools/pmc_traffic.py $OUT/pmc_summary.json $OUT/pmc_traffic.json config3_strong_n$W \
    "rocprofv3 FETCH_SIZE/WRITE_SIZE passes of bench.py --emulate-ranks $W (rank 0 of config 3 over $W ranks)"
head -12 $OUT/prof_summary.txt
