#!/bin/bash
# Round 6: kernel traces of the instrumented timed loop (bench.py's default
# per-kernel timing) for two builds.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
mkdir -p gpurun_out/r06r
for spec in head:$REPO/$H/libkarma_head.so rc:; do
  name=${spec%%:*}; lib=${spec#*:}
  (cd /tmp && export TMPDIR=/tmp && KARMA_LIB=$lib KARMA_ALLOW_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/gpurun_out/r06r/$name -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format > $REPO/gpurun_out/r06r/$name.log 2>&1) || { echo "trace $name failed"; tail -5 gpurun_out/r06r/$name.log; exit 1; }
  python3 -c "import json,sys; t=open('gpurun_out/r06r/$name.log').read(); i=t.rfind('{\"metric'); d=json.loads(t[i:t.index('\n',i)]); print('$name', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
