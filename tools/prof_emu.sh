#!/bin/bash
# GPU box: kernel trace (every launch, library ones included) of the 8-rank
# weak and strong emulations; gpurun_out/prof_emu_{weak,strong}/
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in weak strong; do
  extra=""; [ $m = weak ] && extra="--weak"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_emu_$m -o trace --output-format csv -- \
      python3 $REPO/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity $extra \
      > $OUT/prof_emu_$m.log 2>&1 || { echo "rocprof $m failed"; tail $OUT/prof_emu_$m.log; exit 1; }
  echo "== $m"; head -40 $OUT/prof_emu_$m/trace_kernel_stats.csv | cut -d, -f1-5
done
