#!/bin/bash
# Index staging for direct-bucket tiles over their record stage: bin-path parity (direct vs sorted
# bitwise includes dense 2,000-bin scans), then A/B with 32-bin tiles (whose C2 tiles overflow the
# 256-record stage) and the default C2 / C3 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/idx
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py > $O/pytest.log 2>&1 || exit 1
L=$PWD/gc-slam_amd/gcslam
for v in base idx0; do
  lib=$L/libgcslam_hip.so
  [ $v != base ] && lib=$L/libgcslam_hip_$v.so
  GCSLAM_BIN_TILE=32 GCSLAM_LIB=$lib timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > $O/c2_t32_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/c2_base.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_base.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_primitive_map.py tests/test_gpu_primitive_evidence.py tests/test_gpu_primitive_path.py > $O/pytest_pmap.log 2>&1 || exit 1
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/pmap_bench.txt 2>&1 || exit 1
