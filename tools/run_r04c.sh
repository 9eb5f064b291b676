source tools/gpu_step.sh
TAIL=25 step pytest_c 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -v --timeout 300 --timeout-method thread
LEGS="config3 strong_emu8" STEPS=40 bash tools/measure_quick.sh
mkdir -p gpurun_out/quick_nofork && cp -r gpurun_out/quick/* gpurun_out/quick_nofork/ 2>/dev/null
KARMA_FORK=0 LEGS="config3 strong_emu8" STEPS=40 bash tools/measure_quick.sh > gpurun_out/nofork.txt; cat gpurun_out/nofork.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_emu8c -o trace --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity > $REPO/gpurun_out/prof_emu8c.log 2>&1
echo "rocprof rc=$?"
cd $REPO && python3 tools/trace_step.py gpurun_out/prof_emu8c classify2 > gpurun_out/emu8c_step.txt; cat gpurun_out/emu8c_step.txt
cd $REPO && timeout -k 10 300 python3 tools/eq_phases.py > gpurun_out/eq_phases.json 2> gpurun_out/eq_phases.err; echo "eq rc=$?"; cat gpurun_out/eq_phases.json
