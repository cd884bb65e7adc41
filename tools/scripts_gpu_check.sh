#!/bin/bash
# GPU check: parity tests, smoke, bench (C2 headline line incl. C3 roofline + CPU baseline), and
# rocprofv3 kernel traces of C2 and C3.  Each GPU step has its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py > "$OUT/bench_c2.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_c3.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > "$OUT/prof_c2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv -- \
    python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/prof_c3.log" 2>&1 || exit $?
exit 0
