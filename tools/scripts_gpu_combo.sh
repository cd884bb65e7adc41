#!/bin/bash
# Deflation start A/B at C3 / C2 (same box) + bin-path parity, then the primitive map's parity and
# timing after the one-pass block fuse of step 12b.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/scripts_gpu_frob.sh || exit 1
O=gpurun_out/pmap3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_primitive_map.py tests/test_gpu_primitive_evidence.py tests/test_gpu_primitive_path.py > $O/pytest_pmap.log 2>&1 || exit 1
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/bench.txt 2>&1 || exit 1
