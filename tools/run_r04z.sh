# A/B: one or two main streams (KARMA_STEP_STREAMS) at the 2- and 4-rank previews
for r in 1 2; do
  echo "streams=auto rep=$r"; LEGS="strong_emu2 strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "streams=2 rep=$r"; KARMA_STEP_STREAMS=2 LEGS="strong_emu2" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "streams=1 rep=$r"; KARMA_STEP_STREAMS=1 LEGS="strong_emu4" STEPS=60 bash tools/measure_quick.sh || exit 1
done
