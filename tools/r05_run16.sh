#!/bin/bash
# round 5: surfel LDS sort (keys on the grid, sort in one workgroup); live chain parity + timing + trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r06a}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_live_path.py tests/test_gpu_live_shared.py tests/test_gpu_primitive_path.py \
  tests/test_gpu_live_chain.py > "$O/tests.log" 2>&1 || exit $?
timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench.json" 2> "$O/live_bench.err" && GCSLAM_LIVE_STAMPS=1 timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_stamps.json" 2>> "$O/live_bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_bench.py 30 > "$O/liveprof.log" 2>&1 || exit $?
