#!/bin/bash
# Per-tile radix select (k_pm_select) vs the full per-tile radix sort in the primitive map: parity of
# the primitive tests, then the reference-size timing of both paths and a rocprof split of the new one.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/select
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitive_map.py tests/test_gpu_primitive_path.py tests/test_gpu_primitive_evidence.py tests/test_gpu_surfels.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 180 python tools/pmap_bench.py 30 > $O/bench_select.txt 2>&1 || exit 1
GCSLAM_PM_FULLSORT=1 timeout -k 10 180 python tools/pmap_bench.py 30 > $O/bench_fullsort.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/pmap_bench.py 30 > $O/prof.log 2>&1 || exit 1
