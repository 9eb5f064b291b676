# A/B: profile beside classify from the start (KARMA_MARK_AT=3) in one-stream batches
for r in 1 2; do
  echo "mark=default rep=$r"; LEGS="config3 weak_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
  echo "mark=3 rep=$r"; KARMA_MARK_AT=3 LEGS="config3 weak_emu8" STEPS=40 bash tools/measure_quick.sh || exit 1
done
