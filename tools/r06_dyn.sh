#!/bin/bash
# Round 6: the profile's contigs from a device counter (KARMA_PROF_DYN) -- parity
# tests on the tree build, then A/B against the fixed-stride profile, with the
# schedules it may allow (profile after the final kernel + join, profile beside
# classify) and the packed classify staging on top.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_device_profile.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
KARMA_LIB=$REPO/$H/libkarma_pk.so KARMA_ALLOW_VARIANT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest_pk.log 2>&1 || { echo "pytest pk failed"; tail -30 $O/pytest_pk.log; exit 1; }
tail -1 $O/pytest_pk.log
LIBS="nodyn:$H/libkarma_nodyn.so dyn: dm5j::KARMA_MARK_AT=5,KARMA_STEP_JOIN=1 dm3::KARMA_MARK_AT=3 pkdyn:$H/libkarma_pk.so" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
