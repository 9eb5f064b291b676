source tools/gpu_step.sh
TAIL=6 step pytest_e 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -q --timeout 300 --timeout-method thread
for r in 1 2; do
LEGS="strong_emu8 strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_emu8e -o trace --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity > $REPO/gpurun_out/prof_emu8e.log 2>&1
echo "rocprof rc=$?"
cd $REPO && python3 tools/trace_step.py gpurun_out/prof_emu8e classify2 > gpurun_out/emu8e_step.txt; cat gpurun_out/emu8e_step.txt
cd $REPO && timeout -k 10 200 tools/micro/write_bw7 > gpurun_out/write_bw7.txt 2>&1; echo "write_bw7 rc=$?"; cat gpurun_out/write_bw7.txt
