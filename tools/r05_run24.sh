# C2 host split with and without the world-1 RCCL all-reduce in the step (alternated)
export O=gpurun_out/r08a
mkdir -p $O
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live > $O/rccl_$rep.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live --no-rccl > $O/norccl_$rep.log 2>&1 || exit 1
done
