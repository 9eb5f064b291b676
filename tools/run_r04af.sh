# fixed cost of the timed loop at the 8-rank preview: steps 10/20/40/80, one and two main streams
for st in 10 20 40 80; do
  echo "streams=auto steps=$st"; LEGS="strong_emu8" STEPS=$st bash tools/measure_quick.sh || exit 1
done
for st in 20 80; do
  echo "streams=1 steps=$st"; KARMA_STEP_STREAMS=1 LEGS="strong_emu8" STEPS=$st bash tools/measure_quick.sh || exit 1
done
for st in 10 40; do
  echo "config3 steps=$st"; LEGS="config3" STEPS=$st bash tools/measure_quick.sh || exit 1
done
