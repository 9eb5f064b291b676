source tools/gpu_step.sh
TAIL=6 step pytest_step 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -q --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_step.log && { echo "step tests failed: stop"; exit 1; }
AB_PARITY=" " LIBS="base: stage1024:karma_amd/variants/libkarma_stage1024.so stage2048:karma_amd/variants/libkarma_stage2048.so" LEGS="config3" REPS="1 2 3" STEPS=30 bash tools/ab_lib.sh
for r in 1 2; do LEGS="strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1; done
