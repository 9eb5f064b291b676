#!/bin/bash
# GPU box: code-reduce A/B: kernel trace per library variant
# (karma_amd/variants/libkarma_<name>.so, tools/build_variant.sh; "base" = the in-tree build)
# and per workload in MODES (strong = 8-rank strong preview, weak = 8-rank weak preview, one = config 3).
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/abr
MODES=${MODES:-strong}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in $MODES; do
  case $m in
    strong) extra="--emulate-ranks 8 --strong" ;;
    weak) extra="--emulate-ranks 8" ;;
    one) extra="" ;;
  esac
  for v in "$@"; do
    lib=""; [ $v != base ] && lib=$REPO/karma_amd/variants/libkarma_$v.so
    KARMA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/${m}_$v -o trace --output-format csv -- \
        python3 $REPO/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-timing --no-e2e $extra \
        > $OUT/${m}_$v.log 2>&1 || { echo "rocprof $m $v failed"; tail $OUT/${m}_$v.log; exit 1; }
    echo "== $m $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/${m}_$v.log) reduce_us $(grep code_reduce $OUT/${m}_$v/trace_kernel_stats.csv | python3 -c 'import sys,csv; r=next(csv.reader(sys.stdin)); print(round(float(r[3])/1000,1))')"
  done
done
