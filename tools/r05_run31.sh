#!/bin/bash
# round-5 closing check on the final code: full GPU suite, smoke, the driver's command (default: CPU
# baseline included), association / primitive-map C-ABI timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
export O=${O:-gpurun_out/r08j}; mkdir -p "$O"
bash tools/gpu.sh tests smoke || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || exit $?
bash tools/gpu.sh assoc pmap || exit $?
