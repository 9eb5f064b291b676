#!/bin/bash
# Round 6 closing validation on one MI355X (the tree's build): every GPU test,
# smoke, the driver's bench command, the emulated-rank previews, config 5's
# per-GPU share, a rocprofv3 kernel trace + stats of the bench, and the
# FETCH_SIZE / WRITE_SIZE passes that profiles/pmc_traffic.json comes from.
#   tools/r06_final2.sh TAG  -> gpurun_out/TAG/
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06final2}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python tools/summarize_bench.py $OUT/bench.json
for w in 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --emulate-ranks $w --cpu-baseline off --no-e2e > $OUT/emu$w.json 2> $OUT/emu$w.err || { echo "emu$w failed"; tail $OUT/emu$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/emu$w.json'));print('emu$w', d['ms_per_step'], d['single_batch_ms'], d.get('records_other',{}).get('ms_per_step'))"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --weak --emulate-ranks 8 --cpu-baseline off --no-e2e > $OUT/weak8.json 2> $OUT/weak8.err || { echo "weak8 failed"; tail $OUT/weak8.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/weak8.json'));print('weak8', d['ms_per_step'], d.get('records_other',{}).get('ms_per_step'))"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --config config5 --cpu-baseline off --no-e2e > $OUT/config5.json 2> $OUT/config5.err || { echo "config5 failed"; tail $OUT/config5.err; exit 1; }
python tools/summarize_bench.py $OUT/config5.json | head -3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-other-format > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail $OUT/prof.log; exit 1; }
head -14 $OUT/prof/trace_kernel_stats.csv | cut -d, -f1-5
cd $REPO
PASSES="trace;FETCH_SIZE;WRITE_SIZE" tools/pmc_ab.sh $TAG/pmc3 "base:" > /dev/null 2>&1 || { echo "pmc3 failed"; exit 1; }
PASSES="trace;FETCH_SIZE;WRITE_SIZE" BENCH_ARGS="--emulate-ranks 8" tools/pmc_ab.sh $TAG/pmc8 "base:" > /dev/null 2>&1 || { echo "pmc8 failed"; exit 1; }
echo pmc done
