#!/bin/bash
# Round 6: seg_read FETCH calibration + kernel traces of config 3 and the 8-rank
# strong preview (steps' timelines: tools/trace_step.py).  -> gpurun_out/TAG/
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06t}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $REPO/tools/micro/seg_read 7 > $OUT/seg_read.txt 2>&1 || { echo "seg_read failed"; exit 1; }
cat $OUT/seg_read.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $OUT/seg_pmc -o pmc --output-format csv -- $REPO/tools/micro/seg_read 7 > $OUT/seg_pmc.log 2>&1 || { echo "seg pmc failed"; tail $OUT/seg_pmc.log; exit 1; }
python3 - $OUT/seg_pmc <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    acc[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print("FETCH_SIZE", k, [round(x / 1024, 1) for x in v], "MiB per dispatch (KB units)")
PY
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr3 -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 8 --warmup 3 --cpu-baseline off --no-timing --no-e2e --no-parity > $OUT/tr3.log 2>&1 || { echo "trace3 failed"; tail $OUT/tr3.log; exit 1; }
python3 $REPO/tools/trace_step.py $OUT/tr3/trace classify2 2 > $OUT/config3_step.txt
tail -40 $OUT/config3_step.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr8 -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-timing --no-e2e --no-parity --emulate-ranks 8 > $OUT/tr8.log 2>&1 || { echo "trace8 failed"; tail $OUT/tr8.log; exit 1; }
python3 $REPO/tools/trace_step.py $OUT/tr8/trace classify2 4 > $OUT/emu8_step.txt
tail -60 $OUT/emu8_step.txt
