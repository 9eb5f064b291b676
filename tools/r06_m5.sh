#!/bin/bash
# Round 6: with 512-thread final / edge blocks, the profile after the final
# kernel (mark 5) + join again: the edge stage now fits beside the profile's
# blocks, so it should no longer delay the profile's grid.  Trace + A/B.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06m5}
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && KARMA_MARK_AT=5 KARMA_STEP_JOIN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/m5j -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format --no-timing > $REPO/$O/m5j.log 2>&1) || { echo "trace failed"; tail -5 $O/m5j.log; exit 1; }
python3 tools/trace_step.py $O/m5j classify2 1 | tail -16
LIBS="base: m5j::KARMA_MARK_AT=5,KARMA_STEP_JOIN=1 m5::KARMA_MARK_AT=5" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
