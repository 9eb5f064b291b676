#!/bin/bash
# Round 6: does classify of step i+1 overlap the profile of step i (config 3,
# one main stream)?  Kernel traces of the timed loop for two builds, then the
# join A/B (classify waits for the previous profile).
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
mkdir -p gpurun_out/r06q
for spec in head:$REPO/$H/libkarma_head.so rc:; do
  name=${spec%%:*}; lib=${spec#*:}
  (cd /tmp && export TMPDIR=/tmp && KARMA_LIB=$lib KARMA_ALLOW_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/gpurun_out/r06q/$name -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format --no-timing > $REPO/gpurun_out/r06q/$name.log 2>&1) || { echo "trace $name failed"; tail -5 gpurun_out/r06q/$name.log; exit 1; }
  tail -c 300 gpurun_out/r06q/$name.log | head -c 0
  python3 -c "import json,sys; t=open('gpurun_out/r06q/$name.log').read(); i=t.rfind('{\"metric'); d=json.loads(t[i:t.index('\n',i)]); print('$name', d['ms_per_step'])"
done
LIBS="head:$H/libkarma_head.so headj:$H/libkarma_head.so:KARMA_STEP_JOIN=1 rc: rcj::KARMA_STEP_JOIN=1" LEGS="config3" STEPS=40 REPS="1 2" tools/ab_lib.sh
