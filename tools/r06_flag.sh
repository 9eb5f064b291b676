#!/bin/bash
# Round 6: flagged records + rare-step replay: parity tests, then bench lines.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06f}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_configs.py tests/test_gpu_fake_rccl.py \
    -k "${PYK:-not config5}" -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('other', d.get('records_other'))"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --emulate-ranks 8 > $OUT/emu8.json 2> $OUT/emu8.err || { echo "emu8 failed"; tail -30 $OUT/emu8.err; exit 1; }
python tools/summarize_bench.py $OUT/emu8.json
python -c "import json;d=json.load(open('$OUT/emu8.json'));print('other', d.get('records_other'))"
