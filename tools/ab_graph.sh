#!/bin/bash
# Graph-kernel variant check: records-graph parity tests on each library, then interleaved A/B bench.
# Usage (GPU box): tools/ab_graph.sh name1 name2 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $REPO/gpurun_out/ab
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$REPO/karma_amd/variants/libkarma_$v.so
  KARMA_LIB=$lib timeout -k 10 250 python -u -m pytest $REPO/tests/test_gpu_parity.py $REPO/tests/test_gpu_ingest.py -q -x -k "records or readset or update or sam or eq" --timeout 120 --timeout-method thread > $REPO/gpurun_out/ab/pytest_$v.log 2>&1
  rc=$?
  echo "pytest $v rc=$rc: $(tail -1 $REPO/gpurun_out/ab/pytest_$v.log)"
  [ $rc != 0 ] && { tail -30 $REPO/gpurun_out/ab/pytest_$v.log; exit 1; }
done
bash $REPO/tools/ab_bench.sh "$@"
