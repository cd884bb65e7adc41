# association: prep + stage fused into one launch (A) vs two launches (B: GCSLAM_PREP_FUSED=0)
export O=gpurun_out/r08g
mkdir -p $O
PYTEST_K="association or live_chain or evidence or knob_paths" bash tools/gpu.sh tests && \
for rep in 1 2; do
timeout -k 10 200 python tools/assoc_bench.py 30 50,0 > $O/assoc_A$rep.txt 2>&1 && \
GCSLAM_PREP_FUSED=0 timeout -k 10 200 python tools/assoc_bench.py 30 50,0 > $O/assoc_B$rep.txt 2>&1 || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/assoc_bench.py 30 50 > $O/prof.log 2>&1
