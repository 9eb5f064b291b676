#!/bin/bash
# Round 6: FETCH/read-rate micro (128-byte segments), library A/B (HEAD vs tree),
# fork A/B and the weak 8-rank preview, flagged records.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
mkdir -p gpurun_out/r06i
timeout -k 10 120 tools/micro/seg_read 7 > gpurun_out/r06i/seg_read.txt 2>&1 && cat gpurun_out/r06i/seg_read.txt | tail -3 || exit 1
LIBS="head:karma_amd/variants/libkarma_head.so new:" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_lib.sh || exit 1
ENVS="nofork:KARMA_FORK=0" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2" tools/ab_env.sh || exit 1
LIBS="new:" LEGS="weak_emu8" STEPS=40 REPS="1" tools/ab_lib.sh
