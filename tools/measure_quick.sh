#!/bin/bash
# GPU box: the one-GPU bench plus the 8-rank strong and weak previews (no
# tests); gpurun_out/quick/*.json
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/quick
mkdir -p $OUT
cd $REPO
run() {
  local n=$1; shift
  timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  [ $rc -ne 0 ] && { echo "$n failed rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels_ms_per_step']; print('$n', d['ms_per_step'], 'ms/step', {x: k[x] for x in k if k[x] > 0.015})"
}
run config3
run strong_emu8 --strong --emulate-ranks 8
run weak_emu8 --emulate-ranks 8
