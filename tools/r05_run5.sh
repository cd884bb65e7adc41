#!/bin/bash
# round-5 GPU step: the world-1 all-reduce inside the pipeline, A/B of its stream priority and of the
# pushforward's launch thread
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05g}; mkdir -p "$O"
O=$O REPS=2 STEPS=100 VARIANTS="base|GCSLAM_BENCH_STRIDE=100|;;prio|GCSLAM_BENCH_STRIDE=100 GCSLAM_COMBINE_PRIO=1|;;pushinline|GCSLAM_BENCH_STRIDE=100 GCSLAM_PUSH_THREAD=0|;;prio_inline|GCSLAM_BENCH_STRIDE=100 GCSLAM_COMBINE_PRIO=1 GCSLAM_PUSH_THREAD=0|" bash tools/ab_bench.sh
