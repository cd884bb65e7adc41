#!/bin/bash
# round-5 GPU step: the whole GPU suite, smoke, the driver-shaped bench line and a 100-step line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r05f}; mkdir -p "$O"
O=$O bash tools/gpu.sh tests smoke || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live > "$O/bench_c2_100.log" 2>&1 || exit $?
