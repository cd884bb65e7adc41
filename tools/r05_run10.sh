#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05l}; mkdir -p "$O"
O=$O SWEEP_CONFIGS="c3 c2" SWEEP_STEPS=40 SWEEP="base:-:GCSLAM_BENCH_STRIDE=2 pipe4:pipe4:GCSLAM_BENCH_STRIDE=2 pipe4w4:pipe4w4:GCSLAM_BENCH_STRIDE=2 base2:-:GCSLAM_BENCH_STRIDE=2" bash tools/gpu.sh sweep
