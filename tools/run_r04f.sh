source tools/gpu_step.sh
LEGS="strong_emu8 config3" STEPS=60 bash tools/measure_quick.sh || exit 1
KARMA_STEP_STREAMS=1 LEGS="strong_emu8" STEPS=60 bash tools/measure_quick.sh || exit 1
cd $REPO && timeout -k 10 200 tools/micro/write_bw7 > gpurun_out/write_bw7.txt 2>&1; echo "write_bw7 rc=$?"; cat gpurun_out/write_bw7.txt
