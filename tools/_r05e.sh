bash tools/gpu_run.sh r05h tests=tests/test_gpu_step.py quick=config3,strong_emu8 || exit 1
for v in plainskip nokarg both; do
  KARMA_LIB=$PWD/karma_amd/variants/libkarma_$v.so KARMA_ALLOW_VARIANT=1 bash tools/gpu_run.sh r05h_$v quick=config3,strong_emu8 || exit 1
done
KARMA_STEP_OWN_CTRL=0 bash tools/gpu_run.sh r05h_noown quick=config3,strong_emu8
