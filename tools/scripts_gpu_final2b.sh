#!/bin/bash
# The closing evidence's last steps (after the instrumented library rebuild): per-phase clocks of the
# bin kernel at C2 / C3 and the primitive-map timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 180 python tools/phase_prof.py c2 > $O/phase_c2.txt 2>&1 || exit 1
timeout -k 10 180 python tools/phase_prof.py c3 > $O/phase_c3.txt 2>&1 || exit 1
timeout -k 10 300 python tools/pmap_bench.py 30 > $O/pmap_bench.txt 2>&1 || exit 1
