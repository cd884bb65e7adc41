#!/bin/bash
# Deflation start A/B (Frobenius-norm start vs Gershgorin alone): bin-path parity, then same-box C3
# and C2 benches, twice each, and the C3 phase clocks of the new start.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/frob
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py > $O/pytest.log 2>&1 || exit 1
L=$PWD/gc-slam_amd/gcslam
for rep in 1 2; do
  for v in base frob0; do
    lib=$L/libgcslam_hip.so
    [ $v != base ] && lib=$L/libgcslam_hip_$v.so
    GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_${v}_$rep.log 2>&1 || exit 1
    GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > $O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
