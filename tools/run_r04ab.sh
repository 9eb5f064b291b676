# A/B: profile blocks per CU left free (KARMA_STEP_HEADROOM) in one-stream
# deferred batches, with the profile's start point (KARMA_MARK_AT)
for r in 1 2; do
  echo "h=0 mark=2 rep=$r"; LEGS="config3 weak_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "h=1 mark=2 rep=$r"; KARMA_STEP_HEADROOM=1 LEGS="config3 weak_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "h=1 mark=1 rep=$r"; KARMA_STEP_HEADROOM=1 KARMA_MARK_AT=1 LEGS="config3" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "h=1 mark=5 rep=$r"; KARMA_STEP_HEADROOM=1 KARMA_MARK_AT=5 LEGS="config3" STEPS=60 bash tools/measure_quick.sh || exit 1
done
