#!/bin/bash
# PMC passes (counters only, no traces) for the hot kernels, C2 and C3; one pass per run, each
# with its own time limit (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/pmc"
mkdir -p "$OUT"
RE='k_bins_scale|k_points|k_pt|k_pushforward'
run() {  # config, name, counters...
  local cfg=$1 name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -d "$OUT/${cfg}_$name" -o run \
    --output-format csv -- python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline --no-c3 \
    > "$OUT/${cfg}_$name.log" 2>&1
}
for cfg in ${PMC_CONFIGS:-c2 c3}; do
  run "$cfg" fetch FETCH_SIZE || exit $?
  run "$cfg" write WRITE_SIZE || exit $?
done
exit 0
