#!/bin/bash
# One parameterised GPU-box run (replaces the per-run tools/run_r04*.sh files).
#   tools/gpu_run.sh TAG ITEM...      outputs under gpurun_out/TAG/
# ITEM:
#   tests[=PYTEST_ARGS]   GPU tests (default: all of -m gpu); PYTEST_ARGS with ',' for ' '
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          bench.py line -> bench.json (ARGS with ',' for ' ')
#   ranks2                bench.py --gpus 2 self-launched on this one GPU (host-staged transport)
#   quick[=LEGS]          tools/measure_quick.sh legs (default: config3 strong_emu2/4/8 weak_emu8)
#   rocprof[=CFG]         profiles/run_rocprof.sh (kernel trace + PMC passes)
#   trace[=ARGS]          rocprofv3 kernel trace of bench.py ARGS -> trace_*.csv
# Every GPU step runs under its own time limit; the run stops after a fault,
# an abort, a segfault or a time limit (tools/gpu_step.sh).
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
source tools/gpu_step.sh
fail() { echo "$1: stop"; exit 1; }
for item in "$@"; do
  name=${item%%=*}; arg=""; [ "$name" != "$item" ] && arg=$(echo "${item#*=}" | tr ',' ' ')
  case $name in
    tests)
      TAIL=15 step $TAG/pytest 1500 python -u -m pytest ${arg:-tests} -m gpu -q --timeout 300 --timeout-method thread
      grep -qE "[0-9]+ failed|[0-9]+ error" $OUT/pytest.log && fail "GPU tests failed" ;;
    smoke)
      TAIL=5 step $TAG/smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
      grep -q "smoke ok" $OUT/smoke.log || fail "smoke failed" ;;
    bench)
      timeout -k 10 600 python bench.py $arg > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
      python tools/summarize_bench.py $OUT/bench.json ;;
    ranks2)
      KARMA_FORCE_DEVICE=0 KARMA_DIST_BACKEND=host timeout -k 10 600 python bench.py --gpus 2 --cpu-baseline off \
          --no-e2e --no-weak-leg $arg > $OUT/ranks2.json 2> $OUT/ranks2.err
      rc=$?; echo "ranks2 rc=$rc"; [ $rc -ne 0 ] && { tail -8 $OUT/ranks2.err; exit $rc; }
      python tools/summarize_bench.py $OUT/ranks2.json ;;
    quick)
      LEGS=${arg:-"config3 strong_emu2 strong_emu4 strong_emu8 weak_emu8"} QUICK_OUT=$OUT/quick STEPS=${STEPS:-40} \
          bash tools/measure_quick.sh || exit 1 ;;
    rocprof)
      PROF_OUT=$OUT bash profiles/run_rocprof.sh ${arg:-config3} || exit 1 ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace \
          --output-format csv -- python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e \
          --no-parity $arg > $OUT/trace.log 2>&1)
      rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
      python3 tools/trace_step.py $OUT/trace classify2 > $OUT/trace_step.txt && head -30 $OUT/trace_step.txt ;;
    *) echo "unknown item $item"; exit 2 ;;
  esac
done
echo "gpu_run $TAG done"
