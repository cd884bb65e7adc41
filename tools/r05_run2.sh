#!/bin/bash
# round-5 GPU step: combine latency variants and the roofline stamping stride A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05d}; mkdir -p "$O"
for v in "graph|" "main|GCSLAM_COMBINE_STREAM=main GCSLAM_COMBINE_GRAPH=0" "sendhost|GCSLAM_COMBINE_SEND=host" \
         "main_sendhost|GCSLAM_COMBINE_STREAM=main GCSLAM_COMBINE_SEND=host GCSLAM_COMBINE_GRAPH=0" \
         "probe_outonly|GCSLAM_COMBINE_PROBE=noccl GCSLAM_COMBINE_SEND=host" \
         "probe_outonly_main|GCSLAM_COMBINE_PROBE=noccl GCSLAM_COMBINE_SEND=host GCSLAM_COMBINE_STREAM=main GCSLAM_COMBINE_GRAPH=0"; do
  n=${v%%|*}; e=${v#*|}
  env $e timeout -k 10 120 python tools/combine_bench.py 2000 > "$O/combine_$n.json" 2>&1 || exit $?
done
O=$O/ab REPS=2 STEPS=20 VARIANTS="s8|GCSLAM_BENCH_STRIDE=8|--no-rccl;;s1|GCSLAM_BENCH_STRIDE=1|--no-rccl" bash tools/ab_bench.sh
