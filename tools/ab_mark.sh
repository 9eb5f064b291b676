#!/bin/bash
# GPU box: A/B of where the side-stream profile may start (KARMA_MARK_AT, see
# graph_sets.hip SetsJob::launch), config 3 on one GPU and the 8-rank strong
# preview, alternating; gpurun_out/abm/*.json
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/abm
mkdir -p $OUT
cd $REPO
for rep in ${REPS:-1 2}; do
  for m in ${MARKS:-0 4 2}; do
    for w in config3 strong_emu8; do
      extra=""; [ $w = strong_emu8 ] && extra="--emulate-ranks 8"
      KARMA_MARK_AT=$m timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e --no-parity --steps ${STEPS:-30} $extra \
        > $OUT/${w}_m${m}_r${rep}.json 2> $OUT/${w}_m${m}_r${rep}.err || { echo "$w m$m failed"; tail -5 $OUT/${w}_m${m}_r${rep}.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${w}_m${m}_r${rep}.json')); print('$w', 'mark', $m, 'rep', $rep, d['ms_per_step'], 'classify', d['roofline']['avg_launch_ms'])"
    done
  done
done
