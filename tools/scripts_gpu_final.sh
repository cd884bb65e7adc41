#!/bin/bash
# Round-end evidence: parity suite + smoke + bench (C2, C3) + rocprof kernel stats (scripts_gpu_check.sh),
# PMC FETCH/WRITE passes (scripts_pmc.sh), then the per-phase clocks of the bin kernel (prof build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/scripts_gpu_check.sh || exit $?
bash tools/scripts_pmc.sh || exit $?
timeout -k 10 180 python tools/phase_prof.py c2 > gpurun_out/phase_c2.txt 2>&1 || exit $?
timeout -k 10 180 python tools/phase_prof.py c3 > gpurun_out/phase_c3.txt 2>&1 || exit $?
