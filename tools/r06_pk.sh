#!/bin/bash
# Round 6: packed staging of own reads (KARMA_CLS_PACKED), with and without the
# branch-free emit (KARMA_CLS_EMIT_DUMMY): parity subset on each variant, A/B, SQ counters.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06pk}
mkdir -p $O
for v in pk pkd; do
  KARMA_LIB=$REPO/$H/libkarma_$v.so KARMA_ALLOW_VARIANT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py \
      -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; grep -E "Error|assert|FAIL" $O/pytest_$v.log | head; tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
LIBS="new: pk:$H/libkarma_pk.so pkd:$H/libkarma_pkd.so" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh || exit 1
cd /tmp && export TMPDIR=/tmp
PASSES="trace;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
  $REPO/tools/pmc_ab.sh ${R06_TAG:-r06pk}/pmc "pk:KARMA_LIB=$REPO/$H/libkarma_pk.so KARMA_ALLOW_VARIANT=1" || exit 1
