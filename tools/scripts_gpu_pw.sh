#!/bin/bash
# k_points register target A/B at C3 / C2 (compiler default vs 3 and 4 waves per SIMD, with spills).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pw
mkdir -p $O
L=$PWD/gc-slam_amd/gcslam
for v in base pw3 pw4; do
  lib=$L/libgcslam_hip.so
  [ $v != base ] && lib=$L/libgcslam_hip_$v.so
  GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_$v.log 2>&1 || exit 1
  GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > $O/c2_$v.log 2>&1 || exit 1
done
