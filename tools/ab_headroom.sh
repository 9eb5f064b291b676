#!/bin/bash
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${ABDIR:-abhr}
mkdir -p $OUT
cd $REPO
for rep in ${REPS:-1 2}; do
  for spec in ${SPECS:-base_h0:0: base_h1:1: pw6_h0:0:karma_amd/variants/libkarma_pw6.so pw6_h1:1:karma_amd/variants/libkarma_pw6.so}; do
    name=${spec%%:*}; rest=${spec#*:}; hr=${rest%%:*}; lib=${rest#*:}
    for leg in ${LEGS:-config3 strong_emu8 weak_emu8}; do
      extra=""; case $leg in strong_emu*) extra="--emulate-ranks 8" ;; weak_emu*) extra="--weak --emulate-ranks 8" ;; esac
      # config3 uses h as given; emulated legs too (the default there is 1)
      f=$OUT/${leg}_${name}_r${rep}
      KARMA_SIDE_HEADROOM=$hr KARMA_LIB=$lib KARMA_ALLOW_VARIANT=1 timeout -k 10 240 python bench.py --cpu-baseline off --no-e2e --no-parity --steps 30 $extra > $f.json 2> $f.err || { echo "$leg $name failed"; tail -5 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); print('$leg', '$name', 'rep', $rep, d['ms_per_step'], 'prof', d['kernels_ms_per_step']['kmer_profile'])"
    done
  done
done
