#!/bin/bash
# R_mf polar iteration: f32 scaling / exact polish (default) vs the round-4 form vs a no-polar probe;
# C2 bench + kernel stats per library, alternated; then the host/GPU tests touching R_mf
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r09}; mkdir -p "$O"
for r in 1 2; do
  for v in fast oldpolar nopolar; do
    L=""; [ "$v" != fast ] && L="gc-slam_amd/gcslam/libgcslam_hip_$v.so"
    GCSLAM_LIB=${L:-gc-slam_amd/gcslam/libgcslam_hip.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$r -o run --output-format csv -- \
      python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live > $O/bench_${v}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_trajectory.py > $O/pytest.log 2>&1
