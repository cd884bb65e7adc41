#!/bin/bash
# Bin-kernel tile shape A/B: parity (bin path, full size, golden), then same-box C2 bench with the
# default tile (32 bins x 8 lanes at C2) and GCSLAM_BIN_TILE=64, twice each, C3 once, and the
# per-phase clocks of both shapes at C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tile
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for tb in 32 64; do
    GCSLAM_BIN_TILE=$tb timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 > $O/c2_${tb}_$rep.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
for tb in 32 64; do
  GCSLAM_BIN_TILE=$tb timeout -k 10 180 python tools/phase_prof.py c2 > $O/phase_c2_$tb.txt 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > $O/prof_c2.log 2>&1 || exit 1
