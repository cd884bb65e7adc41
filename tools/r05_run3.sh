#!/bin/bash
# round-5 GPU step: armed all-reduce chain tests + latency, stamping stride A/B with fence-free events
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05e}; mkdir -p "$O"
O=$O PYTEST_K="distributed or determinism" bash tools/gpu.sh tests || exit $?
for v in "armed|" "direct|GCSLAM_COMBINE_ARMED=0"; do
  n=${v%%|*}; e=${v#*|}
  env $e timeout -k 10 120 python tools/combine_bench.py 2000 > "$O/combine_$n.json" 2>&1 || exit $?
done
O=$O/ab REPS=2 STEPS=20 VARIANTS="s8|GCSLAM_BENCH_STRIDE=8|;;s1|GCSLAM_BENCH_STRIDE=1|;;norccl|GCSLAM_BENCH_STRIDE=1|--no-rccl" bash tools/ab_bench.sh
