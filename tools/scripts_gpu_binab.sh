#!/bin/bash
# Bin-kernel change check: parity tests of the bin kernel, same-box A/B against the previous
# build (libgcslam_hip_prev.so), then the phase profiles of the new build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py > gpurun_out/pytest_new.log 2>&1 || exit 1
REPS=${REPS:-2} bash tools/scripts_gpu_ab.sh || exit 1
timeout -k 10 200 python tools/phase_prof.py c3 > gpurun_out/phase_c3_new.txt 2>&1 || exit 1
timeout -k 10 200 python tools/phase_prof.py c2 > gpurun_out/phase_c2_new.txt 2>&1
