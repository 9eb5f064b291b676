#!/bin/bash
# Secondary bench lines (GPU box): strong-scaling preview of BASELINE configs[3]
# (one rank's share of config 3 at N = 2/4/8 emulated ranks), the shuffled-contig
# locality bench, and config 5 whole on one GPU.  Output: gpurun_out/meas/*.json
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/meas
mkdir -p $OUT
cd $REPO
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  [ $rc -ne 0 ] && { echo "$n failed rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'], 'ms/step', d['value'])"
}
for w in 1 2 4 8; do run strong_emu$w --strong --emulate-ranks $w; done
run shuffled --shuffle-contigs
run weak_emu8 --emulate-ranks 8
run config2 --config config2
run config5_1gpu --config config5_1gpu --steps 5 --warmup 2
