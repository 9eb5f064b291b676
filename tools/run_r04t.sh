# A/B: the records job's general-read branch on the spare main stream (default)
# or in order on the main stream (KARMA_FORK=0), config 3 and the 8-rank preview
for r in 1 2; do
  echo "fork=1 rep=$r"; LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "fork=0 rep=$r"; KARMA_FORK=0 LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
