# A/B: the timed loop's last batch deferred (default) or synchronous (KARMA_BENCH_LAST_SYNC=1)
for r in 1 2; do
  for st in 20 60; do
    echo "last=deferred steps=$st rep=$r"; LEGS="config3 strong_emu8" STEPS=$st bash tools/measure_quick.sh || exit 1
    echo "last=sync steps=$st rep=$r"; KARMA_BENCH_LAST_SYNC=1 LEGS="config3 strong_emu8" STEPS=$st bash tools/measure_quick.sh || exit 1
  done
done
