#!/bin/bash
# Round 6: slotted binned fronts -- parity tests, then A/B against packed granules.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
mkdir -p gpurun_out/r06j
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_configs.py -k "records or deferred or flagged or digests" \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/r06j/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" gpurun_out/r06j/pytest.log | head; tail -30 gpurun_out/r06j/pytest.log; exit 1; }
tail -2 gpurun_out/r06j/pytest.log
LIBS="packed:karma_amd/variants/libkarma_packed.so slot:" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
