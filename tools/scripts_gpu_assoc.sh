#!/bin/bash
# Association operator: GPU parity tests, timing, rocprof kernel summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/assoc
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_association.py > gpurun_out/assoc/pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/assoc_bench.py 30 > gpurun_out/assoc/bench.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/assoc/prof -o run --output-format csv -- python3 tools/assoc_bench.py 10 > gpurun_out/assoc/prof.log 2>&1
