#!/bin/bash
# Round 6: kernel traces of the packed-staging build (which took the slower
# schedule in most runs) to check the dispatch race at the mark: does the
# final kernel start before the profile in the slow runs?
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
H=karma_amd/variants
O=gpurun_out/${R06_TAG:-r06race}
mkdir -p $O
for r in 1 2; do
  (cd /tmp && export TMPDIR=/tmp && KARMA_LIB=$REPO/$H/libkarma_pk.so KARMA_ALLOW_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/pk$r -o trace --output-format csv -- \
    python3 $REPO/bench.py --steps 20 --warmup 5 --cpu-baseline off --no-e2e --no-parity --no-other-format > $REPO/$O/pk$r.log 2>&1) || { echo "trace $r failed"; tail -5 $O/pk$r.log; exit 1; }
  python3 -c "import json; t=open('$O/pk$r.log').read(); i=t.rfind('{\"metric'); d=json.loads(t[i:t.index(chr(10),i)]); print('run $r', d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'))"
  python3 tools/trace_step.py $O/pk$r classify2 1 | tail -16
done
