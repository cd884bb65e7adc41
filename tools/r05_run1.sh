#!/bin/bash
# round-5 GPU step: parity subset, combine latency variants, balanced-gather A/B, phase clocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05c}; mkdir -p "$O"
O=$O PYTEST_K="parity or fullsize or golden or determinism or trajectory or distributed" bash tools/gpu.sh tests || exit $?
for v in "graph|" "direct|GCSLAM_COMBINE_GRAPH=0" "noccl|GCSLAM_COMBINE_PROBE=noccl"; do
  n=${v%%|*}; e=${v#*|}
  env $e timeout -k 10 120 python tools/combine_bench.py 2000 > "$O/combine_$n.json" 2>&1 || exit $?
done
O=$O B=nobal REPS=2 bash tools/gpu.sh ab phase
