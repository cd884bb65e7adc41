#!/bin/bash
# Same-box A/B of an environment knob on one build: A = default, B = $ENVB (e.g. GCSLAM_PUSH_MAIN=1),
# bench C2 and C3 alternating, REPS (default 2) times.  Optionally the whole GPU suite first (TESTS=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/envab
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_gpu.log 2>&1 || exit 1
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    e=""; [ $v = B ] && e="$ENVB"
    env $e timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c3 > gpurun_out/envab/${v}_c2_$rep.log 2>&1 || exit 1
    env $e timeout -k 10 300 python bench.py --config c3 --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/envab/${v}_c3_$rep.log 2>&1 || exit 1
  done
done
