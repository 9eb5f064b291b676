#!/bin/bash
# GPU box: the one-GPU bench plus the strong-scaling previews (W = 2, 4, 8
# emulated ranks, each rank's share of config 3) and the 8-rank weak preview
# (no tests); gpurun_out/quick/*.json.  STEPS / LEGS override the defaults.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${QUICK_OUT:-$REPO/gpurun_out/quick}
mkdir -p $OUT
cd $REPO
run() {
  local n=$1; shift
  timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e --steps ${STEPS:-20} "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  [ $rc -ne 0 ] && { echo "$n failed rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels_ms_per_step']; print('$n', d['ms_per_step'], 'ms/step', 'parity', d.get('parity'), 'host_us', d.get('host_us_per_step'), 'calls', d.get('api_calls_per_step'), 'wait_us', (d.get('step_driver') or {}).get('host_wait_us_per_step'), {x: k[x] for x in k if k[x] > 0.012})"
}
for leg in ${LEGS:-config3 strong_emu2 strong_emu4 strong_emu8 weak_emu8}; do
  case $leg in
    config3) run config3 ;;
    strong_emu*) run $leg --emulate-ranks ${leg#strong_emu} --no-parity ;;
    weak_emu*) run $leg --weak --emulate-ranks ${leg#weak_emu} --no-parity ;;
  esac
done
