#!/bin/bash
# PMC passes (counters only, no traces) for the hot kernels; each pass has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/pmc"
mkdir -p "$OUT"
RE='k_bins_scale|k_points|k_pt|k_pushforward|k_budget'
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -d "$OUT/$name" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES || exit $?
run hit TCC_HIT_sum TCC_MISS_sum || exit $?
