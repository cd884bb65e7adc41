#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05h}; mkdir -p "$O"
for v in "stamped|" "query|GCSLAM_COMBINE_OUT=query"; do
  n=${v%%|*}; e=${v#*|}
  env $e timeout -k 10 120 python tools/combine_bench.py 2000 > "$O/combine_$n.json" 2>&1 || exit $?
done
O=$O REPS=2 STEPS=100 VARIANTS="stamped|GCSLAM_BENCH_STRIDE=100|;;query|GCSLAM_BENCH_STRIDE=100 GCSLAM_COMBINE_OUT=query|" bash tools/ab_bench.sh
