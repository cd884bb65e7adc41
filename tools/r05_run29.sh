# the driver's bench command after warming the stamped path in the warm-up (twice)
export O=gpurun_out/r08f
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver1.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver2.log 2>&1
