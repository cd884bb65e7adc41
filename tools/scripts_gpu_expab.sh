#!/bin/bash
# Whole GPU suite on the current build, then same-box A/B against libgcslam_hip_prev.so.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/pytest_gpu.log 2>&1 || exit 1
REPS=2 bash tools/scripts_gpu_ab.sh
