#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05j}; mkdir -p "$O"
O=$O SWEEP_STEPS=60 SWEEP="base:-:GCSLAM_BENCH_STRIDE=4 cu4:-:GCSLAM_BENCH_STRIDE=4,GCSLAM_PUSH_CU_SKIP=4 cu8:-:GCSLAM_BENCH_STRIDE=4,GCSLAM_PUSH_CU_SKIP=8 cu2:-:GCSLAM_BENCH_STRIDE=4,GCSLAM_PUSH_CU_SKIP=2 base2:-:GCSLAM_BENCH_STRIDE=4" bash tools/gpu.sh sweep
