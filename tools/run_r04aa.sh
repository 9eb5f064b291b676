# A/B: side-stream priority (KARMA_STEP_SIDE_PRIO=1: as high as the main streams)
for r in 1 2; do
  echo "prio=normal rep=$r"; LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "prio=high rep=$r"; KARMA_STEP_SIDE_PRIO=1 LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
