#!/bin/bash
# SQ counters of the graph kernels (tools/ablate.py, dbg 0), one --pmc pass per group.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmcg
mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o pmc --output-format csv -- python3 $REPO/tools/ablate.py 0 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc $rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
