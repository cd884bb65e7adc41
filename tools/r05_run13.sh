#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r05o}; mkdir -p "$O"
timeout -k 10 300 python tools/live_prof.py 30 > "$O/live_prof.txt" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_prof.py 30 > "$O/liveprof.log" 2>&1 || exit $?
