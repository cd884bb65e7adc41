#!/bin/bash
# Surfel extraction parity tests on the GPU, then a rocprof kernel summary of one extraction loop.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_surfels.py \
  > gpurun_out/pytest_surfels.log 2>&1 || exit 1
timeout -k 10 200 python tools/surfel_bench.py > gpurun_out/surfel_bench.txt 2>&1
