#!/bin/bash
# Round 6: classify as a persistent grid of 2 blocks per CU (room for the profile
# beside it on every CU), with and without the profile started beside classify
# (KARMA_MARK_AT=3).  Parity subset on the variant, then the A/B.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06p2}
mkdir -p $O
KARMA_LIB=$REPO/$H/libkarma_p2.so KARMA_ALLOW_VARIANT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py -k "records or deferred or flagged" \
    -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LIBS=${AB_LIBS:-"head:$H/libkarma_head.so hm3:$H/libkarma_head.so:KARMA_MARK_AT=3 p2:$H/libkarma_p2.so p2m3:$H/libkarma_p2.so:KARMA_MARK_AT=3 p4m3:$H/libkarma_p4.so:KARMA_MARK_AT=3"} \
  LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh
