#!/bin/bash
# Per-rank compute of the weak-scaled config at N emulated ranks (bench.py --emulate-ranks),
# base library vs variants.  Usage (GPU box): tools/ab_emul.sh N name1 name2 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/ab
mkdir -p $OUT
export KARMA_OVERLAP=0
W=$1; shift
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$REPO/karma_amd/variants/libkarma_$v.so
  KARMA_LIB=$lib timeout -k 10 150 python $REPO/bench.py --cpu-baseline off --no-e2e --steps ${AB_STEPS:-10} --emulate-ranks $W > $OUT/emu${W}_$v.json 2> $OUT/emu${W}_$v.err
  rc=$?
  python -c "
import json; d=json.load(open('$OUT/emu${W}_$v.json')); k=d['kernels_ms_per_step']
print('emu$W $v', d['ms_per_step'], ' '.join(f'{n}={v:.4f}' for n,v in k.items() if v>0.02))" 2>/dev/null || echo "emu$W $v rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
