# A/B: where the profile may start (KARMA_MARK_AT) in config 3's deferred one-stream mode
for r in 1 2; do
  for m in 5 2 4 1; do
    echo "mark=$m rep=$r"
    KARMA_MARK_AT=$m LEGS="config3" STEPS=60 bash tools/measure_quick.sh || exit 1
  done
done
