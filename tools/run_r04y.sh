# A/B: KARMA_MARK_AT 2 (profile after the code partition) against 5, every leg,
# then the build's own choice (one main stream: 2; two: 5) with no override
for r in 1 2; do
  for m in 5 2; do
    echo "mark=$m rep=$r"
    KARMA_MARK_AT=$m LEGS="config3 strong_emu8 strong_emu4 weak_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  done
  echo "mark=default rep=$r"
  LEGS="config3 strong_emu8 strong_emu4 weak_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
