#!/bin/bash
# Primitive map parity on the GPU, then the whole GPU suite + smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmap
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_primitive_map.py tests/test_gpu_primitive_evidence.py > $O/pytest_pmap.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -v -rA --timeout 120 --timeout-method thread -m gpu tests \
  > $O/pytest_all.log 2>&1 || exit 1
