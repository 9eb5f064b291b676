source tools/gpu_step.sh
TAIL=25 step pytest_b 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py "tests/test_gpu_parity.py::test_merge_runs_and_split" "tests/test_gpu_configs.py::test_config_digests" -v --timeout 300 --timeout-method thread
LEGS="config3 strong_emu8" STEPS=40 bash tools/measure_quick.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_emu8 -o trace --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity > $REPO/gpurun_out/prof_emu8.log 2>&1
echo "rocprof rc=$?"
cd $REPO && python3 tools/trace_step.py gpurun_out/prof_emu8 classify2 > gpurun_out/emu8_step.txt; cat gpurun_out/emu8_step.txt
