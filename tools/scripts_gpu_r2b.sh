#!/bin/bash
# Direct buckets + k_budget on the worker: parity (bin path, full size, golden, association), the
# association timing, then same-box A/B at C2 and C3: base (direct), sorted (same library with
# GCSLAM_SORTED_BUCKETS=1) and prev (libgcslam_hip_prev.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b gpurun_out/assoc
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_association.py \
  > gpurun_out/r2b/pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/assoc_bench.py 30 > gpurun_out/assoc/bench.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/assoc/prof -o run --output-format csv -- python3 tools/assoc_bench.py 10 > gpurun_out/assoc/prof.log 2>&1 || exit 1
L=$PWD/gc-slam_amd/gcslam
for rep in 1 2; do
  for v in base sorted prev; do
    lib=$L/libgcslam_hip.so; env=""
    [ $v = prev ] && lib=$L/libgcslam_hip_prev.so
    [ $v = sorted ] && env="GCSLAM_SORTED_BUCKETS=1"
    env $env GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > gpurun_out/r2b/${v}_c2_$rep.log 2>&1 || exit 1
    env $env GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r2b/${v}_c3_$rep.log 2>&1 || exit 1
  done
done
