#!/bin/bash
# Round 6: which part of RC costs (raw walk / per-code range check), the profile
# beside classify again (mark 3), and a kernel trace of the 8-rank preview.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
LIBS="head:$H/libkarma_head.so raw1:$H/libkarma_raw1.so chk2:$H/libkarma_chk2.so rc: m3:$H/libkarma_head.so:KARMA_MARK_AT=3" \
  LEGS="config3" STEPS=40 REPS="1 2" tools/ab_lib.sh || exit 1
mkdir -p gpurun_out/r06p && cd /tmp && export TMPDIR=/tmp
KARMA_LIB=$REPO/$H/libkarma_head.so KARMA_ALLOW_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/r06p/emu8 -o trace --output-format csv -- \
  python3 $REPO/bench.py --steps 20 --warmup 5 --emulate-ranks 8 --cpu-baseline off --no-e2e --no-parity --no-other-format > $REPO/gpurun_out/r06p/emu8.log 2>&1 || { echo "trace failed"; tail -5 $REPO/gpurun_out/r06p/emu8.log; exit 1; }
echo trace done
