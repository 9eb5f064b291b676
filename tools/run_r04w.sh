# A/B: profile waves per SIMD (KARMA_PROF_WAVES 6 default, 5, 8) in the deferred stream of steps
source tools/gpu_step.sh
LIBS="base: pw5:karma_amd/variants/libkarma_pw5.so pw8:karma_amd/variants/libkarma_pw8.so" LEGS="config3 strong_emu8" REPS="1 2" STEPS=60 bash tools/ab_lib.sh
