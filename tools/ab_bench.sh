#!/bin/bash
# A/B timing of library variants (karma_amd/variants/libkarma_<name>.so) on the bench
# workload, interleaved: base, v1, v2, ..., base.  Usage: tools/ab_bench.sh name1 name2 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/ab
mkdir -p $OUT
export KARMA_OVERLAP=0
run() {
  local tag=$1 lib=$2
  KARMA_LIB=$lib timeout -k 10 150 python $REPO/bench.py --cpu-baseline off --no-e2e --steps ${AB_STEPS:-10} > $OUT/$tag.json 2> $OUT/$tag.err
  local rc=$?
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); k=d['kernels_ms_per_step']
print('$tag', d['ms_per_step'], ' '.join(f'{n}={v:.4f}' for n,v in k.items() if v>0.02))" 2>/dev/null || echo "$tag rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
}
for r in $(seq 1 ${AB_ROUNDS:-1}); do
  run base$r ""
  for v in "$@"; do run $v.$r $REPO/karma_amd/variants/libkarma_$v.so; done
done
run base_end ""
