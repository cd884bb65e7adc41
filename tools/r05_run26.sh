#!/bin/bash
# live path after the association / step-12b work: timing, host phase stamps, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r08c}; mkdir -p "$O"
timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench.json" 2> "$O/live_bench.err" && GCSLAM_LIVE_STAMPS=1 timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_stamps.json" 2>> "$O/live_bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_bench.py 30 > "$O/liveprof.log" 2>&1 || exit $?
