source tools/gpu_step.sh
TAIL=4 step pytest_step 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fake_rccl.py -q --timeout 300 --timeout-method thread
grep -q "failed" gpurun_out/pytest_step.log && { echo "step tests failed: stop"; exit 1; }
for r in 1 2; do LEGS="config3 strong_emu8" STEPS=20 bash tools/measure_quick.sh || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline off --no-e2e > gpurun_out/bench_ad.json 2> gpurun_out/bench_ad.err; echo "bench rc=$?"
python -c "import json; d=json.load(open('gpurun_out/bench_ad.json')); print(d['ms_per_step'], d['parity'], d['config']['columns_M'], d['config']['edges'], d['step_driver'])"
