#!/bin/bash
# SQ/TCC counters of the records -> pairs kernels (tools/ablate.py) for the base
# library and variants, one --pmc pass per group.  Usage (GPU box): tools/pmc_ab.sh name1 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmcab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$REPO/karma_amd/variants/libkarma_$v.so
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    KARMA_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/${v}_p$i -o pmc --output-format csv -- python3 $REPO/tools/ablate.py 0 > $OUT/${v}_p$i.log 2>&1
    rc=$?
    echo "$v pass $i rc $rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
exit 0
