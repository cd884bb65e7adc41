#!/bin/bash
# Same-box A/B of the bins fold width at C2 (1,563 partial rows): 1024 (default), 512, 256 threads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/foldab
mkdir -p $O
L=$PWD/gc-slam_amd/gcslam
for rep in 1 2; do
  for v in base fold512 fold256; do
    lib=$L/libgcslam_hip.so
    [ $v != base ] && lib=$L/libgcslam_hip_$v.so
    GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > $O/${v}_$rep.log 2>&1 || exit 1
  done
done
GCSLAM_LIB=$L/libgcslam_hip_fold256.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_256 -o run \
    --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > $O/prof_256.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_base -o run \
    --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > $O/prof_base.log 2>&1 || exit 1
