cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 120 python tools/phase_prof.py c2 > gpurun_out/phase_c2.txt 2>&1 || exit 1
timeout -k 10 180 python tools/phase_prof.py c3 > gpurun_out/phase_c3.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit 1
