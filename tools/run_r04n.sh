source tools/gpu_step.sh
TAIL=6 step pytest_step 600 python -u -m pytest tests/test_gpu_step.py -q --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_step.log && { echo "step tests failed: stop"; exit 1; }
for r in 1 2 3; do
  LEGS="config3" STEPS=30 bash tools/measure_quick.sh || exit 1
  mv gpurun_out/quick/config3.json gpurun_out/quick/config3_join_r$r.json
  KARMA_STEP_JOIN=0 LEGS="config3" STEPS=30 bash tools/measure_quick.sh || exit 1
  mv gpurun_out/quick/config3.json gpurun_out/quick/config3_nojoin_r$r.json
done
AB_PARITY=" " LIBS="base: split2:karma_amd/variants/libkarma_split2.so split3:karma_amd/variants/libkarma_split3.so split4:karma_amd/variants/libkarma_split4.so" LEGS="config3" REPS="1 2" STEPS=30 bash tools/ab_lib.sh
