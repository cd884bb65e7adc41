#!/bin/bash
# C3 (and C2) A/B over kernel variants (VARIANTS, "base" = libgcslam_hip.so), REPS alternations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3var
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base prev}; do
    lib=gc-slam_amd/gcslam/libgcslam_hip.so
    [ "$v" != base ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
    GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/c3var/${v}_c3_$rep.log 2>&1 || exit 1
  done
done
