# step 12b: dense-tile eviction shortcut; primitive-map tests, pmap bench, kernel trace
export O=gpurun_out/r08k
mkdir -p $O
PYTEST_K="primitive_map or live_chain or shared" bash tools/gpu.sh tests && \
timeout -k 10 300 python tools/pmap_bench.py 20 > $O/pmap_bench.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/pmap_bench.py 10 > $O/prof.log 2>&1
