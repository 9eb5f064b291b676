source tools/gpu_step.sh
TAIL=8 step pytest_eq 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_consumers.py tests/test_gpu_rearrange.py -q -k "eq" --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/pytest_eq.log && ! grep -q "failed" gpurun_out/pytest_eq.log || { echo "eq tests failed: stop"; exit 1; }
cd $REPO && timeout -k 10 300 python3 tools/eq_phases.py > gpurun_out/eq_phases3.json 2> gpurun_out/eq_phases3.err; echo "eq rc=$?"; cat gpurun_out/eq_phases3.json
LIBS="base: w1:karma_amd/variants/libkarma_w1.so w2:karma_amd/variants/libkarma_w2.so w1c:karma_amd/variants/libkarma_w1c.so w3:karma_amd/variants/libkarma_w3.so" LEGS="config3 strong_emu8" REPS="1 2" STEPS=30 bash tools/ab_lib.sh
