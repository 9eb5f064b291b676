#!/bin/bash
# Round 6: staged codes m0 << 4 | rel, range checked per code (RC) -- parity subset, then A/B.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06o}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_configs.py -k "records or deferred or flagged or digests or range" \
    -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
LIBS=${AB_LIBS:-"head:karma_amd/variants/libkarma_head.so norc:karma_amd/variants/libkarma_norc.so rc:"} LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh
