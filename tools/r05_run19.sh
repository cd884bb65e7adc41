# association closing measurement (one-barrier Sinkhorn default): tests, timing, probe, kernel trace
export O=gpurun_out/r07t
mkdir -p $O
PYTEST_K="association or live_chain or evidence or shared" bash tools/gpu.sh tests && \
timeout -k 10 200 python tools/assoc_bench.py 30 > $O/assoc_bench.txt 2>&1 && \
GCSLAM_LIB=$PWD/gc-slam_amd/gcslam/libgcslam_hip_probe.so timeout -k 10 120 python tools/assoc_bench.py 3 50 > $O/probe.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/assoc_bench.py 30 50 > $O/prof.log 2>&1
