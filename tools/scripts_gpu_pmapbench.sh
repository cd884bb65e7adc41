#!/bin/bash
# Primitive map timing at the reference sizes + rocprof kernel stats of the same run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmapbench
mkdir -p $O
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/bench.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 tools/pmap_bench.py 10 > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python tools/assoc_bench.py 30 > $O/assoc.txt 2>&1 || exit 1
