#!/bin/bash
# Round 6: the step's tail beside the profile.  The final kernel (1,024 threads,
# 70 KB LDS) and the edge stage (1,024 threads) cannot start on a CU holding the
# profile's 3 resident blocks (24 of 32 wave slots): they wait for the whole
# profile.  With 512-thread blocks they fit beside it; the next classify then
# waits for the profile (join).  Parity subset on the variant, a kernel trace,
# then the A/B.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06t}
mkdir -p $O
KARMA_LIB=$REPO/$H/libkarma_t512.so KARMA_ALLOW_VARIANT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_fake_rccl.py \
    -x -q --timeout 300 --timeout-method thread > $O/pytest_t512.log 2>&1 || { echo "pytest t512 failed"; grep -E "Error|assert|FAIL" $O/pytest_t512.log | head; tail -30 $O/pytest_t512.log; exit 1; }
tail -1 $O/pytest_t512.log
(cd /tmp && export TMPDIR=/tmp && KARMA_LIB=$REPO/$H/libkarma_t512.so KARMA_ALLOW_VARIANT=1 KARMA_STEP_JOIN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/t512j -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format --no-timing > $REPO/$O/t512j.log 2>&1) || { echo "trace failed"; tail -5 $O/t512j.log; exit 1; }
python3 tools/trace_step.py $O/t512j classify2 1 | tail -16
LIBS="base: bj::KARMA_STEP_JOIN=1 t512:$H/libkarma_t512.so t512j:$H/libkarma_t512.so:KARMA_STEP_JOIN=1" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
