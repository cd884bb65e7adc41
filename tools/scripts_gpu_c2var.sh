#!/bin/bash
# C2 A/B over kernel variants (VARIANTS, "base" = libgcslam_hip.so), REPS alternations, then a
# rocprof kernel summary of the base build at C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c2var
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base prev}; do
    lib=gc-slam_amd/gcslam/libgcslam_hip.so
    [ "$v" != base ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
    GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > gpurun_out/c2var/${v}_$rep.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2var/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > gpurun_out/c2var/prof.log 2>&1
