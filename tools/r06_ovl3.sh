#!/bin/bash
# Round 6: where classify of step i+1 runs relative to the profile of step i
# (kernel traces of the timed loop, tree build vs packed staging), then the
# join A/B (classify waits for the previous profile).
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06o3}
mkdir -p $O
for spec in new: pk:$REPO/$H/libkarma_pk.so; do
  name=${spec%%:*}; lib=${spec#*:}
  (cd /tmp && export TMPDIR=/tmp && KARMA_LIB=$lib KARMA_ALLOW_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/$name -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format --no-timing > $REPO/$O/$name.log 2>&1) || { echo "trace $name failed"; tail -5 $O/$name.log; exit 1; }
  python3 tools/trace_overlap.py $O/$name/trace_kernel_trace.csv 8
done
LIBS="new: newj::KARMA_STEP_JOIN=1 pk:$H/libkarma_pk.so pkj:$H/libkarma_pk.so:KARMA_STEP_JOIN=1" LEGS="config3" STEPS=40 REPS="1 2" tools/ab_lib.sh
