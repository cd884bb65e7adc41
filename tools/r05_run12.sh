#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05n}; mkdir -p "$O"
O=$O PYTEST_K="golden or determinism or fullsize or planar or pipeline" bash tools/gpu.sh tests || exit $?
O=$O SWEEP_CONFIGS="c3 c2" SWEEP_STEPS=40 SWEEP="hoist:-:GCSLAM_BENCH_STRIDE=40 hoist2:-:GCSLAM_BENCH_STRIDE=40" bash tools/gpu.sh sweep
