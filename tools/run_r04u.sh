# A/B: pair-bucket geometry (KARMA_GEO_B=512: 391 buckets of 512 contigs at
# config 3's 200k contigs, against 196 of 1024), with config-3 parity on
source tools/gpu_step.sh
AB_PARITY=" " LIBS="base: geo512:karma_amd/variants/libkarma_geo512.so" LEGS="config3 strong_emu8 strong_emu4" REPS="1 2" STEPS=60 bash tools/ab_lib.sh
