#!/bin/bash
# GPU parity suite + smoke (each step under its own limit; stops at the first failure).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
