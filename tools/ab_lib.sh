#!/bin/bash
# GPU box: A/B of library builds, alternating, same box and call.
# LIBS="base:karma_amd/variants/libkarma_base.so new: m3::KARMA_MARK_AT=3" (empty
# path = the tree's library; a third field: environment, comma-separated), LEGS (config3 strong_emu8 weak_emu8), REPS, STEPS;
# gpurun_out/ab/<leg>_<name>_r<rep>.json
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/ab
mkdir -p $OUT
cd $REPO
for rep in ${REPS:-1 2}; do
  for spec in ${LIBS:-new:}; do
    name=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}
    envs=""; [ "$rest" != "$lib" ] && envs=$(echo ${rest#*:} | tr ',' ' ')
    for leg in ${LEGS:-config3 strong_emu8}; do
      case $leg in
        config3) extra="" ;;
        strong_emu*) extra="--emulate-ranks ${leg#strong_emu}" ;;
        weak_emu*) extra="--weak --emulate-ranks ${leg#weak_emu}" ;;
      esac
      f=$OUT/${leg}_${name}_r${rep}
      env $envs KARMA_LIB=$lib KARMA_ALLOW_VARIANT=1 timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e --no-other-format ${AB_PARITY:---no-parity} \
        --steps ${STEPS:-30} $extra ${AB_EXTRA} > $f.json 2> $f.err || { echo "$leg $name failed"; tail -5 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); k=d['kernels_ms_per_step']; print('$leg', '$name', 'rep', $rep, d['ms_per_step'], 'live', (d.get('roofline') or {}).get('avg_launch_ms'), 'ceil', (d.get('profile_write_ceiling') or {}).get('profile_vs_ceiling'), {x: round(k[x], 4) for x in k if k[x] > 0.015})"
    done
  done
done
