#!/bin/bash
# Closing check of the per-tile select: the whole GPU suite + smoke, then the primitive-map timing of
# the select and the full-sort paths.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/selfin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 180 python tools/pmap_bench.py 30 > $O/bench_select.txt 2>&1 || exit 1
GCSLAM_PM_FULLSORT=1 timeout -k 10 180 python tools/pmap_bench.py 30 > $O/bench_fullsort.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/pmap_bench.py 30 > $O/prof.log 2>&1 || exit 1
