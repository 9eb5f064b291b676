#!/bin/bash
# Round 6: the step's schedule.  In the timed loop the final kernel is launched
# beside the profile and waits for its blocks; whether classify of the next
# step then overlaps the profile depends on which of the two is dispatched
# first (0.80 vs 0.88-0.99 ms per step).  A/B of deterministic orders: the
# profile after the final kernel (mark 5) with the next classify waiting for
# the profile (join), three reps each; kernel trace of the first.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06s}
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && KARMA_MARK_AT=5 KARMA_STEP_JOIN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/m5j -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format --no-timing > $REPO/$O/m5j.log 2>&1) || { echo "trace failed"; tail -5 $O/m5j.log; exit 1; }
python3 tools/trace_step.py $O/m5j classify2 1 | tail -16
LIBS="new: m5j::KARMA_MARK_AT=5,KARMA_STEP_JOIN=1 m4j::KARMA_MARK_AT=4,KARMA_STEP_JOIN=1 m2j::KARMA_STEP_JOIN=1" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
