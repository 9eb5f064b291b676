#!/bin/bash
# A/B of an environment toggle: ENVS="old:KARMA_AB_OLD=1 new:"
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/abe
mkdir -p $OUT
cd $REPO
for rep in ${REPS:-1 2}; do
  for spec in ${ENVS}; do
    name=${spec%%:*}; ev=${spec#*:}
    for leg in ${LEGS:-config3 strong_emu8}; do
      case $leg in
        config3) extra="" ;;
        strong_emu*) extra="--emulate-ranks ${leg#strong_emu}" ;;
        weak_emu*) extra="--weak --emulate-ranks ${leg#weak_emu}" ;;
      esac
      f=$OUT/${leg}_${name}_r${rep}
      env $ev timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e --no-parity --no-other-format \
        --steps ${STEPS:-30} $extra > $f.json 2> $f.err || { echo "$leg $name failed"; tail -5 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); print('$leg', '$name', 'rep', $rep, d['ms_per_step'])"
    done
  done
done
