# C3 chain under a high-priority scan stream (GCSLAM_STREAM_PRIO=1) vs default, alternated
export O=gpurun_out/r07y
SWEEP="base1:-: prio1:-:GCSLAM_STREAM_PRIO=1 base2:-: prio2:-:GCSLAM_STREAM_PRIO=1" SWEEP_CONFIGS=c3 SWEEP_STEPS=40 bash tools/gpu.sh sweep
