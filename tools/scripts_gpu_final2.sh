#!/bin/bash
# Round-2 closing evidence on HEAD: the whole GPU suite + smoke, bench C2 (headline line with the C3
# roofline pass and the CPU baseline) and C3, rocprof kernel stats of both, PMC FETCH/WRITE passes of
# the hot kernels, per-phase clocks of the bin kernel, the primitive-map timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 > $O/prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- \
    python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_c3.log 2>&1 || exit 1
bash tools/scripts_pmc.sh || exit 1
timeout -k 10 180 python tools/phase_prof.py c2 > $O/phase_c2.txt 2>&1 || exit 1
timeout -k 10 180 python tools/phase_prof.py c3 > $O/phase_c3.txt 2>&1 || exit 1
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/pmap_bench.txt 2>&1 || exit 1
