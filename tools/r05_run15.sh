#!/bin/bash
# round 5: LDS key sort for the surfels, begin through the point fold's mirror; live chain parity + timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r05q}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_surfels.py \
  tests/test_gpu_live_chain.py tests/test_gpu_live_path.py tests/test_gpu_live_shared.py tests/test_gpu_primitive_path.py \
  > "$O/tests.log" 2>&1 || exit $?
timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench.json" 2> "$O/live_bench.err" || exit $?
GCSLAM_BEGIN_MIRROR=0 GCSLAM_SF_LDS_SORT=0 timeout -k 10 300 python tools/live_bench.py 30 > "$O/live_bench_old.json" 2>> "$O/live_bench.err" || exit $?
timeout -k 10 300 python tools/live_prof.py 30 > "$O/live_prof.txt" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/liveprof" -o run --output-format csv -- python3 tools/live_bench.py 30 > "$O/liveprof.log" 2>&1 || exit $?
