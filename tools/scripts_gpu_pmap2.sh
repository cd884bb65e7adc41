#!/bin/bash
# Primitive map parity (map + evidence), then its timing at the reference sizes with rocprof stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmap2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_primitive_map.py tests/test_gpu_primitive_evidence.py tests/test_gpu_primitive_path.py > $O/pytest_pmap.log 2>&1 || exit 1
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/bench.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 tools/pmap_bench.py 10 > $O/prof.log 2>&1 || exit 1
