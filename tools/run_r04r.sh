# A/B: where the side stream's profile may start (KARMA_MARK_AT) in the
# deferred two-stream mode (8-rank strong preview) and one-stream (config 3)
for r in 1 2; do
  for m in 5 3 1 4 0; do
    echo "mark=$m rep=$r"
    KARMA_MARK_AT=$m LEGS="strong_emu8 strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
  done
done
