#!/bin/bash
# Round 6: full-width range check of flagged contigs >= 2^28 (per-step guard) -- parity tests, then A/B against the previous build.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06r}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LIBS="head:karma_amd/variants/libkarma_head.so hlen1:karma_amd/variants/libkarma_hlen1.so new: dummy:karma_amd/variants/libkarma_dummy.so" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh
# instruction mix of classify (is the scalar unit a co-bound?): SQ counters, one pass each
cd /tmp && export TMPDIR=/tmp
PASSES="trace;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES;SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_WAVES" \
  $REPO/tools/pmc_ab.sh ${R06_TAG:-r06r}/pmc "new:" || exit 1
