#!/bin/bash
# rocprofv3 kernel trace + PMC passes of one bench.py workload under a list of
# environment settings (A/B), outputs under gpurun_out/TAG/<label>/.
#   tools/pmc_ab.sh TAG "label1:ENV=1 ENV2=0" "label2:" ...   (BENCH_ARGS: extra bench.py args)
# Counter passes are each a run of their own (never combined with other trace
# domains); each step under its own time limit; stop at the first failure.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 2 --cpu-baseline off --no-e2e --no-timing --no-parity --no-other-format ${BENCH_ARGS:-}"
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  OUT=$REPO/gpurun_out/$TAG/$label
  mkdir -p $OUT
  # PASSES: counter passes separated by ';' (default: the traffic and SQ passes below)
  IFS=';' read -ra PL <<< "${PASSES:-trace;FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY}"
  for pass in "${PL[@]}"; do
    if [ "$pass" = trace ]; then
      env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- \
          python3 $REPO/bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "$label trace failed"; tail -5 $OUT/trace.log; exit 1; }
    else
      name=$(echo $pass | cut -d' ' -f1)
      env $envs timeout -k 10 300 rocprofv3 --pmc $pass -d $OUT/pmc_$name -o pmc --output-format csv -- \
          python3 $REPO/bench.py $ARGS > $OUT/pmc_$name.log 2>&1 || { echo "$label pmc $name failed"; tail -5 $OUT/pmc_$name.log; exit 1; }
    fi
  done
  echo "$label done"
  python3 $REPO/tools/pmc_table.py $OUT
done
