#!/bin/bash
# GPU check: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > "$OUT/bench_c2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1 || exit $?
exit $rc
