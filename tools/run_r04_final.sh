# Round-4 validation on one GPU box: the GPU tests, smoke, the default bench
# line, the per-rank previews, rocprof kernel trace + PMC passes of config 3,
# and a kernel trace of the 8-rank strong preview.  Stops after a failure.
source tools/gpu_step.sh
TAIL=15 step pytest_gpu_r04 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
grep -qE "[0-9]+ failed|[0-9]+ error" gpurun_out/pytest_gpu_r04.log && { echo "GPU tests failed: stop"; exit 1; }
TAIL=5 step smoke_r04 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
grep -q "smoke ok" gpurun_out/smoke_r04.log || { echo "smoke failed: stop"; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_config3_r04.json 2> gpurun_out/bench_config3_r04.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_config3_r04.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_config3_r04.json')); print(d['ms_per_step'], d['parity'], d['roofline']['frac'], d.get('eq_path',{}).get('ms'), d.get('cpu_baseline',{}).get('value'))"
LEGS="strong_emu2 strong_emu4 strong_emu8 weak_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
bash profiles/run_rocprof.sh config3 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_emu8 -o trace --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --emulate-ranks 8 --no-parity > $REPO/gpurun_out/prof_emu8.log 2>&1
echo "rocprof emu8 rc=$?"
cd $REPO && python3 tools/trace_step.py gpurun_out/prof_trace classify2 > gpurun_out/config3_step.txt && python3 tools/trace_step.py gpurun_out/prof_emu8 classify2 > gpurun_out/emu8_step.txt && echo traces ok
