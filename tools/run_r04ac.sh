# A/B: classify loading each lane's 8 records directly (KARMA_CLS_DIRECT=1) against the LDS transpose
source tools/gpu_step.sh
TAIL=4 step pytest_direct 600 env KARMA_LIB=karma_amd/variants/libkarma_direct.so KARMA_ALLOW_VARIANT=1 python -u -m pytest tests/test_gpu_parity.py -q -k "records or graph or chunk" --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_direct.log && { echo "variant tests failed: stop"; exit 1; }
AB_PARITY=" " LIBS="base: direct:karma_amd/variants/libkarma_direct.so" LEGS="config3 strong_emu8" REPS="1 2" STEPS=60 bash tools/ab_lib.sh
