#!/bin/bash
# rocprofv3 trace + PMC passes of the default bench, then the per-kernel summaries (GPU box).
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
bash $REPO/profiles/run_rocprof.sh ${1:-config3} || { echo "rocprof failed"; exit 1; }
cd $REPO && python profiles/pmc_summary.py $OUT --json $OUT/pmc_summary.json > $OUT/prof_summary.txt && head -14 $OUT/prof_summary.txt
python tools/pmc_traffic.py $OUT/pmc_summary.json $OUT/pmc_traffic.json ${1:-config3}_n1 "rocprofv3 FETCH_SIZE/WRITE_SIZE passes of bench.py --config ${1:-config3}"
