#!/bin/bash
# Round 6: the profile's LDS per block padded to 41 KB (KARMA_PROF_LDS_MIN), so
# that at most 3 of its blocks fit a CU (an even resident grid) and classify's
# 39 KB blocks cannot start beside them; with the tree build and the packed
# classify staging.  A/B, three reps.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
LIBS="base: pad::KARMA_PROF_LDS_MIN=41984 pk:$H/libkarma_pk.so pkpad:$H/libkarma_pk.so:KARMA_PROF_LDS_MIN=41984" LEGS="config3 strong_emu8" STEPS=40 REPS="1 2 3" tools/ab_lib.sh
