#!/bin/bash
# Parity suite on the default build, then a same-box A/B of k_points lane variants (C2, C3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
for rep in 1 2; do
for v in ${VARIANTS:-base lp1 lp2 lp4w0}; do
  lib=gc-slam_amd/gcslam/libgcslam_hip.so
  [ "$v" != base ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/var/${v}_c2_$rep.log 2>&1 || exit 1
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/var/${v}_c3_$rep.log 2>&1 || exit 1
done
done
