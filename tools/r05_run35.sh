#!/bin/bash
# sparse top-k: batched key gathers per bitmap word; primitive-map + live tests, pmap bench, live bench
# and kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r09e}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "primitive or live or pmap or view" tests/ \
  > "$O/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python tools/pmap_bench.py 20 > "$O/pmap_bench.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench.json" 2> "$O/live_bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_bench.py 30 > "$O/liveprof.log" 2>&1
