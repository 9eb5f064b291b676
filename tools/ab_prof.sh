#!/bin/bash
# Profile-kernel variant check: parity tests on each variant, then interleaved A/B bench.
# Usage (GPU box): tools/ab_prof.sh name1 name2 ...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $REPO/gpurun_out/ab
for v in "$@"; do
  KARMA_LIB=$REPO/karma_amd/variants/libkarma_$v.so timeout -k 10 200 python -u -m pytest $REPO/tests/test_gpu_parity.py -q -x -k profile --timeout 120 --timeout-method thread > $REPO/gpurun_out/ab/pytest_$v.log 2>&1 || { echo "pytest $v failed rc=$?"; tail -20 $REPO/gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "pytest $v ok: $(tail -1 $REPO/gpurun_out/ab/pytest_$v.log)"
done
timeout -k 10 200 python -u -m pytest $REPO/tests/test_gpu_parity.py -q -x -k profile --timeout 120 --timeout-method thread > $REPO/gpurun_out/ab/pytest_base.log 2>&1 || { echo "pytest base failed"; tail -20 $REPO/gpurun_out/ab/pytest_base.log; exit 1; }
echo "pytest base ok"
bash $REPO/tools/ab_bench.sh "$@"
