source tools/gpu_step.sh
TAIL=16 step pytest_d 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -q --timeout 300 --timeout-method thread
LEGS="config3 strong_emu2 strong_emu4 strong_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
mkdir -p gpurun_out/quick_auto && cp gpurun_out/quick/* gpurun_out/quick_auto/
KARMA_STEP_STREAMS=2 LEGS="strong_emu2 strong_emu4" STEPS=40 bash tools/measure_quick.sh || exit 1
mkdir -p gpurun_out/quick_s2 && cp gpurun_out/quick/* gpurun_out/quick_s2/
KARMA_STEP_STREAMS=1 LEGS="strong_emu4 strong_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
mkdir -p gpurun_out/quick_s1 && cp gpurun_out/quick/* gpurun_out/quick_s1/
LEGS="strong_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_emu8d -o trace --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity > $REPO/gpurun_out/prof_emu8d.log 2>&1
echo "rocprof rc=$?"
cd $REPO && python3 tools/trace_step.py gpurun_out/prof_emu8d classify2 > gpurun_out/emu8d_step.txt; cat gpurun_out/emu8d_step.txt
cd $REPO && timeout -k 10 120 tools/micro/write_bw6 > gpurun_out/write_bw6.txt 2>&1; echo "write_bw6 rc=$?"; cat gpurun_out/write_bw6.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_nolib -o trace --output-format csv -- python3 -m pytest -q -x $REPO/tests/test_gpu_parity.py -k "readset_graph_golden or records_unsorted_and_detection or profile_lowercase_iupac_and_bytes" -p no:cacheprovider > $REPO/gpurun_out/prof_nolib.log 2>&1
echo "nolib rc=$?"; tail -3 $REPO/gpurun_out/prof_nolib.log
