source tools/gpu_step.sh
step launch1 60 ./tools/micro/launch_cost 16 400 256
step launch2 60 ./tools/micro/launch_cost 16 400 1
TAIL=25 step pytest_step 400 python -u -m pytest tests/test_gpu_step.py -x -v --timeout 200 --timeout-method thread
TAIL=30 step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
LEGS="config3 strong_emu8" STEPS=40 bash tools/measure_quick.sh
