source tools/gpu_step.sh
TAIL=12 step pytest_defer 600 python -u -m pytest tests/test_gpu_fake_rccl.py -x -v --timeout 300 --timeout-method thread
grep -q "failed\|Error" gpurun_out/pytest_defer.log && { echo "fake rccl tests failed: stop"; exit 1; }
TAIL=6 step pytest_step 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_distributed.py -q --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_step.log && { echo "step tests failed: stop"; exit 1; }
LEGS="config3 strong_emu8 weak_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
