#!/bin/bash
# Same-box A/B of two builds of the library (bench C2 and C3, alternating): A = libgcslam_hip.so,
# B = libgcslam_hip_$B.so (default prev).  Host speed differs between boxes by ~10 %, so only
# same-call comparisons are meaningful.  REPS (default 2) alternations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
B=${B:-prev}
for rep in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    lib=gc-slam_amd/gcslam/libgcslam_hip.so; [ $v = B ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$B.so
    GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > gpurun_out/ab/${v}_c2_$rep.log 2>&1 || exit 1
    GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab/${v}_c3_$rep.log 2>&1 || exit 1
  done
done
