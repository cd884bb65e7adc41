# association: candidate stats from the pool kernels; tests, timing, Sinkhorn phase probe, trace
export O=gpurun_out/r07r
mkdir -p $O
PYTEST_K="association or live_chain or evidence" bash tools/gpu.sh tests && \
timeout -k 10 200 python tools/assoc_bench.py 30 50,0 > $O/assoc_A.txt 2>&1 && \
GCSLAM_LIB=$PWD/gc-slam_amd/gcslam/libgcslam_hip_probe.so timeout -k 10 120 python tools/assoc_bench.py 3 0,50 > $O/probe.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/assoc_bench.py 30 50 > $O/prof.log 2>&1
