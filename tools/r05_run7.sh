#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05i}; mkdir -p "$O"
O=$O SWEEP_STEPS=60 SWEEP="base:-:GCSLAM_BENCH_STRIDE=60 pw3:pw3:GCSLAM_BENCH_STRIDE=60 pw4:pw4:GCSLAM_BENCH_STRIDE=60 base2:-:GCSLAM_BENCH_STRIDE=60" bash tools/gpu.sh sweep || exit $?
O=$O SWEEP_CONFIGS=c2 SWEEP_STEPS=60 SWEEP="st_fence:-:GCSLAM_BENCH_STRIDE=1 st_default:-:GCSLAM_BENCH_STRIDE=1,GCSLAM_STAMP_EVENT=default st_device:-:GCSLAM_BENCH_STRIDE=1,GCSLAM_STAMP_EVENT=device st_none:-:GCSLAM_BENCH_STRIDE=60" bash tools/gpu.sh sweep
