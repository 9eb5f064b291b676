#!/bin/bash
# GPU box helper: run one step under its own time limit, log to gpurun_out/,
# print the log's tail, and stop the whole call after a fault, an abort, a
# segfault or a time limit (no further GPU step may start after those).
#   source tools/gpu_step.sh; step NAME SECONDS cmd...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $REPO/gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $REPO/gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -${TAIL:-12} $REPO/gpurun_out/$name.log
  case $rc in
    0|1) return 0 ;;  # pass / test failures: later steps may still run
    *) echo "stopping after $name (rc $rc)"; exit $rc ;;
  esac
}
