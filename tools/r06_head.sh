#!/bin/bash
# Round 6 (re-entry): smoke, the records/deferred parity subset and the driver's bench command on the tree's build.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
O=gpurun_out/${R06_TAG:-r06v}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python tools/summarize_bench.py $O/bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --emulate-ranks 8 --cpu-baseline off --no-e2e > $O/emu8.json 2> $O/emu8.err || { echo "emu8 failed"; tail $O/emu8.err; exit 1; }
python -c "import json;d=json.load(open('$O/emu8.json'));print('emu8', d['ms_per_step'], d['single_batch_ms'], d.get('records_other',{}).get('ms_per_step'))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
