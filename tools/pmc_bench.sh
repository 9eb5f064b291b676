#!/bin/bash
# SQ counters of every bench kernel (config3, sequential, 2 steps), one --pmc pass per group.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmcb
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export KARMA_OVERLAP=0
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o pmc --output-format csv -- python3 $REPO/bench.py --steps 2 --warmup 1 --cpu-baseline off --no-e2e --no-timing > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc $rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
