#!/bin/bash
# rocprof kernel summary of the surfel extraction loop (tools/surfel_bench.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/surfprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/surfprof -o run --output-format csv -- \
  python3 tools/surfel_bench.py > gpurun_out/surfprof/bench.txt 2>&1
