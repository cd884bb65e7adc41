# C2 host prologue: budget launch on the worker (default) vs inline (GCSLAM_PUSH_THREAD=0), no RCCL
export O=gpurun_out/r08b
mkdir -p $O
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live --no-rccl > $O/def_$rep.log 2>&1 && \
GCSLAM_PUSH_THREAD=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live --no-rccl > $O/inline_$rep.log 2>&1 || exit 1
done
