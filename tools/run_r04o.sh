source tools/gpu_step.sh
TAIL=6 step pytest_step 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -q --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_step.log && { echo "step tests failed: stop"; exit 1; }
for r in 1 2; do
  LEGS="strong_emu8 strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
  KARMA_STEP_SIDES=1 LEGS="strong_emu8 strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
  GPU_MAX_HW_QUEUES=8 LEGS="strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
LEGS="config3 weak_emu8" STEPS=30 bash tools/measure_quick.sh || exit 1
KARMA_STEP_JOIN=1 LEGS="weak_emu8" STEPS=30 bash tools/measure_quick.sh || exit 1
