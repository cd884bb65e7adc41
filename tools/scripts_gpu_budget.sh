#!/bin/bash
# Vectorised k_budget clears: bin-path parity, C2 / C3 benches, rocprof kernel stats at C3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/budget
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_trajectory.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > $O/c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- \
    python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_c3.log 2>&1 || exit 1
