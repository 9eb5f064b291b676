#!/bin/bash
# Round 6: pinned walk state (KARMA_CLS_PIN) -- parity subset, then A/B:
# 8 per lane (r06 final), 8 pinned, 16 pinned (tree); pairs records: 8 vs 8 pinned.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_configs.py -k "records or deferred or flagged or digests" \
    -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
LIBS="rpl8:karma_amd/variants/libkarma_rpl8.so pin8:karma_amd/variants/libkarma_pin8.so pin16:" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh || exit 1
echo "== pairs records"
mkdir -p gpurun_out/ab_pairs
LIBS="rpl8:karma_amd/variants/libkarma_rpl8.so pin8:karma_amd/variants/libkarma_pin8.so" LEGS="config3" STEPS=40 REPS="1 2" AB_EXTRA="--records pairs" tools/ab_lib.sh
