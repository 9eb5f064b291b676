# Round-4 closing validation: the eq drop-in's new path first (tests + phases),
# then tools/run_r04_final.sh (all GPU tests, smoke, bench line, previews,
# rocprof trace + PMC, step traces).  Stops after a failure.
source tools/gpu_step.sh
TAIL=6 step pytest_eq 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_consumers.py tests/test_gpu_rearrange.py tests/test_gpu_ingest.py -q -k "eq" --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/pytest_eq.log && ! grep -q "failed" gpurun_out/pytest_eq.log || { echo "eq tests failed: stop"; exit 1; }
cd $REPO && timeout -k 10 300 python3 tools/eq_phases.py > gpurun_out/eq_phases9.json 2> gpurun_out/eq_phases9.err; echo "eq rc=$?"; cat gpurun_out/eq_phases9.json
bash tools/run_r04_final.sh
