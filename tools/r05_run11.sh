#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05m}; mkdir -p "$O"
O=$O SWEEP_CONFIGS="c3 c2" SWEEP_STEPS=40 SWEEP="pt1024:-:GCSLAM_BENCH_STRIDE=40 pt2048:-:GCSLAM_BENCH_STRIDE=40,GCSLAM_PT_BLOCKS=2048 pt4096:-:GCSLAM_BENCH_STRIDE=40,GCSLAM_PT_BLOCKS=4096 pt1024b:-:GCSLAM_BENCH_STRIDE=40" bash tools/gpu.sh sweep
