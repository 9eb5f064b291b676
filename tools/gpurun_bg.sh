#!/bin/bash
# Local (build container) wrapper: one gpurun call, tried again only when no
# box or slot is free (gpurun exit 3: nothing ran, nothing charged).
#   tools/gpurun_bg.sh NAME TIMEOUT_S COMMAND   -> gpurun_out/NAME.out
NAME=$1; T=$2; shift 2
OUT=gpurun_out/$NAME.out
: > $OUT
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" >> $OUT 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "[no box, waiting]" >> $OUT; sleep 90
done
echo "finished rc=$rc" >> $OUT
