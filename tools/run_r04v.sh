# A/B: the process's hardware queues (HIP default 4) for the step's 5 streams
for r in 1 2; do
  echo "hwq=4 rep=$r"; LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
  echo "hwq=8 rep=$r"; GPU_MAX_HW_QUEUES=8 LEGS="config3 strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
done
