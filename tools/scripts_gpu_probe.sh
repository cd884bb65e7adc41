#!/bin/bash
# Same-box timing of kernel variants (no parity: probe builds drop work on purpose).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in ${VARIANTS:-base}; do
  lib=gc-slam_amd/gcslam/libgcslam_hip.so
  [ "$v" != base ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/var/${v}_c2.log 2>&1 || exit 1
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/var/${v}_c3.log 2>&1 || exit 1
done
