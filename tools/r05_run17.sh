#!/bin/bash
# round 5: association and step-12b C-ABI timings (verdict item 6) with their kernel splits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r05y}; mkdir -p "$O"
timeout -k 10 300 python tools/assoc_bench.py 30 > "$O/assoc_bench.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/pmap_bench.py > "$O/pmap_bench.txt" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/assocprof" -o run --output-format csv -- python3 tools/assoc_bench.py 30 50 > "$O/assocprof.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/pmapprof" -o run --output-format csv -- python3 tools/pmap_bench.py > "$O/pmapprof.log" 2>&1 || exit $?
