#!/bin/bash
# GPU box: code-reduce A/B on the 8-rank strong preview: kernel trace per library
# variant (karma_amd/variants/libkarma_<name>.so, tools/build_variant.sh); "base" = the in-tree build.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/abr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib=""; [ $v != base ] && lib=$REPO/karma_amd/variants/libkarma_$v.so
  KARMA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$v -o trace --output-format csv -- \
      python3 $REPO/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --strong \
      > $OUT/$v.log 2>&1 || { echo "rocprof $v failed"; tail $OUT/$v.log; exit 1; }
  echo "== $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/$v.log)"
  grep -E "code_reduce|partition_kernel|final_kernel" $OUT/$v/trace_kernel_stats.csv | cut -d, -f1-5
done
