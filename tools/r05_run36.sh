#!/bin/bash
# surfels: bucket fill folded into k_sf_moments; surfel + live tests, live bench, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r09k}; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_surfels.py \
  tests/test_gpu_live_chain.py tests/test_gpu_live_path.py tests/test_gpu_live_shared.py tests/test_gpu_primitive_path.py > "$O/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench.json" 2> "$O/live_bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_bench.py 30 > "$O/liveprof.log" 2>&1
