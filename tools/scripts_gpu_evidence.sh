#!/bin/bash
# Round evidence: the GPU check (tests, smoke, bench C2 + C3, rocprof kernel stats), the PMC
# FETCH/WRITE passes of the roofline kernel, and the bin kernel's phase clocks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/scripts_gpu_check.sh || exit $?
bash tools/scripts_pmc.sh || exit $?
timeout -k 10 200 python tools/phase_prof.py c3 > gpurun_out/phase_c3.txt 2>&1 || exit $?
timeout -k 10 200 python tools/phase_prof.py c2 > gpurun_out/phase_c2.txt 2>&1
