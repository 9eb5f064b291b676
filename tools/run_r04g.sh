source tools/gpu_step.sh
TAIL=6 step pytest_g 600 python -u -m pytest tests/test_gpu_step.py -q --timeout 300 --timeout-method thread
LIBS="base: w1:karma_amd/variants/libkarma_w1.so w2:karma_amd/variants/libkarma_w2.so w1c:karma_amd/variants/libkarma_w1c.so w3:karma_amd/variants/libkarma_w3.so" LEGS="config3 strong_emu8" REPS="1 2" STEPS=30 bash tools/ab_lib.sh
TAIL=8 step pytest_eq 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_consumers.py tests/test_gpu_rearrange.py -q -k "eq" --timeout 300 --timeout-method thread
cd $REPO && timeout -k 10 300 python3 tools/eq_phases.py > gpurun_out/eq_phases2.json 2> gpurun_out/eq_phases2.err; echo "eq rc=$?"; cat gpurun_out/eq_phases2.json; tail -3 gpurun_out/eq_phases2.err
TAIL=4 step pytest_chunk 600 python -u -m pytest tests/test_gpu_parity.py -q -k "both_chunk_sizes" --timeout 300 --timeout-method thread
for r in 1 2; do
KARMA_CHUNK=2048 LEGS="strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
LEGS="strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
