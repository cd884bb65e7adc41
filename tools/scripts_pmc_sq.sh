#!/bin/bash
# SQ counter pass (instruction mix / wave states) for the bin kernel, C2 and C3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/pmc"
mkdir -p "$OUT"
for cfg in c2 c3; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY \
    --kernel-include-regex 'k_bins_scale|k_points|k_pushforward' -d "$OUT/${cfg}_sq" -o run --output-format csv -- \
    python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${cfg}_sq.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex 'k_bins_scale|k_points|k_pushforward' -d "$OUT/${cfg}_sq2" -o run --output-format csv -- \
    python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${cfg}_sq2.log" 2>&1 || exit $?
done
