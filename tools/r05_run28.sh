#!/bin/bash
# round-5 closing measurement: full GPU suite, smoke, the driver's bench command, rocprof C2 / C3,
# association and primitive-map C-ABI timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
export O=${O:-gpurun_out/r08e}; mkdir -p "$O"
bash tools/gpu.sh tests smoke || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || exit $?
bash tools/gpu.sh prof2 prof3 assoc pmap || exit $?
