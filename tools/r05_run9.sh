#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05k}; mkdir -p "$O"
O=$O SWEEP_CONFIGS=c3 SWEEP_STEPS=40 SWEEP="base:-:GCSLAM_BENCH_STRIDE=2 s384:s384:GCSLAM_BENCH_STRIDE=2 pipe1:pipe1:GCSLAM_BENCH_STRIDE=2 nobal:nobal:GCSLAM_BENCH_STRIDE=2 mapv0:mapv0:GCSLAM_BENCH_STRIDE=2 base2:-:GCSLAM_BENCH_STRIDE=2" bash tools/gpu.sh sweep
