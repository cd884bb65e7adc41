#!/bin/bash
# One entry point for the GPU-box steps (run through gpurun from the repo root):
#   bash tools/gpu.sh STEP [STEP ...]
# Steps (each under its own time limit, stopping at the first failure; outputs under $O):
#   tests        pytest -m gpu (the parity suite)          smoke      __graft_entry__.smoke()
#   bench        bench.py C2 headline line (+ C3 roofline + live path + CPU baseline)
#   live         bench.py C2, short, with the live primitive path's timing (live_path)
#   bench3       bench.py --config c3        benchshared  bench.py --map-mode shared (a follower's scan)
#   hostbench    host 22-D numerics micro-benchmark (gc-slam_amd/build/host_bench)
#   prof2/prof3  rocprofv3 --kernel-trace --stats of bench at C2 / C3
#   pmc          FETCH_SIZE / WRITE_SIZE passes (one counter per run) at C2 and C3 (PMC_CONFIGS)
#   sq           SQ instruction-mix / wave-state passes of the hot kernels
#   phase        per-phase clocks of the bin kernel (needs `make -C gc-slam_amd prof`)
#   pmap         primitive-map timing (tools/pmap_bench.py)    assoc   association timing
#   pmapprof     rocprofv3 --kernel-trace --stats of tools/pmap_bench.py (assocprof: of tools/assoc_bench.py)
#   assocsq / assocpmc   SQ passes / FETCH, WRITE, L2 hit and TCP passes of the association kernels
#   ab           same-box A/B of two builds: A = libgcslam_hip.so, B = libgcslam_hip_$B.so
#   envab        same-box A/B of an environment knob: B runs with $ENVB
#   io / ioprof  IMU / odometry branch timing, host vs device (tools/io_bench.py) / its rocprofv3 kernel stats
#   graphab      hipGraph vs stream launches of a six-kernel chain (tools/graph_ab, built in-tree)
#   gaps         device idle gaps per kernel from prof2's trace (tools/trace_gaps.py)
#   sweep        bench C2 + C3 per entry of SWEEP="name:lib_suffix:ENV=V,... ..." (library variants / knobs)
# Env: O (output dir, default gpurun_out/run), REPS (A/B alternations), PYTEST_K (pytest -k filter).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/run}
mkdir -p "$O"
RE='k_bins_scale|k_points|k_budget|k_pt|k_pushforward|k_final|k_fold'

step() {
  case "$1" in
    tests)
      local k=(); [ -n "$PYTEST_K" ] && k=(-k "$PYTEST_K")
      # test failures (pytest exit 1) are in the log and do not stop the later steps; anything else does
      timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail="${MAXFAIL:-8}" -v -rA --timeout 120 --timeout-method thread "${k[@]}" \
        > "$O/pytest_gpu.log" 2>&1; local rc=$?; [ $rc -eq 1 ] && { echo "[gpu.sh] tests: failures, see $O/pytest_gpu.log"; return 0; }; return $rc ;;
    smoke) timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    snapprev)  # the same snapshot with the A/B library (libgcslam_hip_$B.so)
      GCSLAM_LIB=$PWD/gc-slam_amd/gcslam/libgcslam_hip_${B:-prev}.so timeout -k 10 300 python -u tools/bitwise_snapshot.py \
        save "$O/snap_prev.npz" > "$O/snap_prev.log" 2>&1 ;;
    snapenv)  # the same snapshot with $ENVB set (an environment knob)
      env $ENVB timeout -k 10 300 python -u tools/bitwise_snapshot.py save "$O/snap_env.npz" > "$O/snap_env.log" 2>&1 ;;
    snap)  # bitwise snapshot of the bin path (tools/bitwise_snapshot.py), compared with $SNAP_BASE if set
      timeout -k 10 300 python -u tools/bitwise_snapshot.py save "$O/snap.npz" > "$O/snap.log" 2>&1 || return $?
      [ -n "$SNAP_BASE" ] && python tools/bitwise_snapshot.py compare "$SNAP_BASE" "$O/snap.npz" > "$O/snap_cmp.txt" 2>&1
      return 0 ;;
    bench) timeout -k 10 400 python bench.py > "$O/bench_c2.log" 2>&1 ;;
    driver) timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 ;;
    live) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 > "$O/bench_live.log" 2>&1 ;;
    benchshared) timeout -k 10 300 python bench.py --map-mode shared --no-cpu-baseline --no-c3 --no-live > "$O/bench_shared.log" 2>&1 ;;
    hostbench) timeout -k 10 120 ./tools/host_bench tools/host_bench_in.bin > "$O/host_bench.txt" 2>&1 ;;
    bench3) timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline --no-live \
              > "$O/bench_c3.log" 2>&1 ;;
    prof2) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o run --output-format csv -- \
             python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-live > "$O/prof_c2.log" 2>&1 ;;
    prof3) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- \
             python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-live > "$O/prof_c3.log" 2>&1 ;;
    pmc)
      for cfg in ${PMC_CONFIGS:-c2 c3}; do
        for ctr in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" -d "$O/pmc/${cfg}_$ctr" -o run \
            --output-format csv -- python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline --no-c3 --no-live \
            > "$O/pmc_${cfg}_$ctr.log" 2>&1 || return $?
        done
      done ;;
    sq)
      for cfg in c2 c3; do
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES \
          SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$RE" -d "$O/sq/${cfg}" -o run \
          --output-format csv -- python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline --no-c3 --no-live \
          > "$O/sq_$cfg.log" 2>&1 || return $?
      done ;;
    assocsq)  # SQ instruction mix / wave states of the association kernels
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES \
        SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-include-regex "k_as_" -d "$O/assocsq" -o run \
        --output-format csv -- python3 tools/assoc_bench.py 5 > "$O/assocsq.log" 2>&1 ;;
    assocpmc)  # HBM fetch / write and L2 hit counts of the association kernels, one pass each
      for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
        local nm=${ctr// /_}
        timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "k_as_" -d "$O/assocpmc/$nm" -o run \
          --output-format csv -- python3 tools/assoc_bench.py 5 50 > "$O/assocpmc_$nm.log" 2>&1 || return $?
      done ;;
    phasev)  # the phase clocks with PHASE_LIB (a GCS_PHASE_PROF variant: libgcslam_hip_<PHASE_LIB>.so), C3
      GCSLAM_LIB=$PWD/gc-slam_amd/gcslam/libgcslam_hip_${PHASE_LIB}.so timeout -k 10 180 python tools/phase_prof.py c3 \
        > "$O/phase_${PHASE_LIB}_c3.txt" 2>&1 ;;
    phase) for cfg in c2 c3; do timeout -k 10 180 python tools/phase_prof.py $cfg > "$O/phase_$cfg.txt" 2>&1 || return $?; done ;;
    pmap) timeout -k 10 300 python tools/pmap_bench.py 30 > "$O/pmap_bench.txt" 2>&1 ;;
    pmapprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/pmap_prof" -o run --output-format csv -- \
                python3 tools/pmap_bench.py 10 > "$O/pmap_prof.log" 2>&1 ;;
    assoc) timeout -k 10 300 python tools/assoc_bench.py > "$O/assoc_bench.txt" 2>&1 ;;
    assocab) for v in A B; do  # association timing, default library vs libgcslam_hip_$B.so
               lib=gc-slam_amd/gcslam/libgcslam_hip.so; [ $v = B ] && lib=gc-slam_amd/gcslam/libgcslam_hip_${B:-prev}.so
               GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python tools/assoc_bench.py > "$O/assocab_$v.txt" 2>&1 || return $?
             done ;;
    assocprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/assoc_prof" -o run --output-format csv -- \
                 python3 tools/assoc_bench.py 30 ${ASSOC_ITERS:-50,0,10} > "$O/assoc_prof.log" 2>&1 ;;
    ab)
      for rep in $(seq 1 "${REPS:-2}"); do
        for v in A B; do
          lib=gc-slam_amd/gcslam/libgcslam_hip.so; [ $v = B ] && lib=gc-slam_amd/gcslam/libgcslam_hip_${B:-prev}.so
          GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live \
            > "$O/ab_${v}_c2_$rep.log" 2>&1 || return $?
          GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline --no-live \
            > "$O/ab_${v}_c3_$rep.log" 2>&1 || return $?
        done
      done ;;
    envab)
      for rep in $(seq 1 "${REPS:-2}"); do
        for v in A B; do
          e=""; [ $v = B ] && e="$ENVB"
          env $e timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c3 --no-live \
            > "$O/envab_${v}_c2_$rep.log" 2>&1 || return $?
          env $e timeout -k 10 300 python bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline --no-live \
            > "$O/envab_${v}_c3_$rep.log" 2>&1 || return $?
        done
      done ;;
    sweep)  # SWEEP="name:lib_suffix:ENV=V,ENV2=V2 ..." (lib_suffix '-' = the default library)
      for spec in $SWEEP; do
        IFS=: read -r name suf envs <<< "$spec"
        lib=gc-slam_amd/gcslam/libgcslam_hip.so; [ "$suf" != "-" ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$suf.so
        e="GCSLAM_LIB=$PWD/$lib ${envs//,/ }"
        for cfg in ${SWEEP_CONFIGS:-c2 c3}; do
          env $e timeout -k 10 300 python bench.py --config $cfg --steps ${SWEEP_STEPS:-60} --warmup 5 --no-cpu-baseline --no-c3 --no-live > "$O/sweep_${name}_$cfg.log" 2>&1 || return $?
        done
      done ;;
    io) timeout -k 10 120 python tools/io_bench.py > "$O/io_bench.txt" 2>&1 ;;
    ioprof) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$O/io_prof" -o run --output-format csv -- \
              python3 tools/io_bench.py 100 > "$O/io_prof.log" 2>&1 ;;
    ioprobe)  # the IMU kernels' time per probe variant (IOPROBE="- io1 io2 ...": libgcslam_hip_<v>.so; - = default)
      for v in ${IOPROBE:-- io1 io2 io4 io7}; do
        lib=gc-slam_amd/gcslam/libgcslam_hip.so; [ "$v" != "-" ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
        GCSLAM_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/ioprobe_${v/-/base}" -o run \
          --output-format csv -- python3 tools/io_bench.py 50 > "$O/ioprobe_${v/-/base}.log" 2>&1 || return $?
      done ;;
    longrun) for cfg in ${LONG_CONFIGS:-c3}; do  # tools/long_run.py: a long cycled sequence's per-scan diagnostics
        timeout -k 10 240 python tools/long_run.py $cfg ${LONG_SCANS:-400} > "$O/long_run_$cfg.txt" 2>&1 || return $?
      done ;;
    tests2)  # the same pytest selection a second time into pytest_gpu_2.log (a flakiness check; failures do not stop)
      local k2=(); [ -n "$PYTEST_K" ] && k2=(-k "$PYTEST_K")
      timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail="${MAXFAIL:-8}" -v -rA --timeout 120 --timeout-method thread "${k2[@]}" \
        > "$O/pytest_gpu_2.log" 2>&1; local rc=$?; [ $rc -le 1 ] && return 0; return $rc ;;
    det) timeout -k 10 600 python -u tools/determinism_check.py ${DET_REPS:-12} > "$O/det.txt" 2>&1 ;;
    repeat)  # REPEAT="tests/file.py test_name N": one test function N times in one process
      timeout -k 10 600 python -u tools/repeat_test.py $REPEAT > "$O/repeat.log" 2>&1 ;;
    graphab) timeout -k 10 120 ./tools/graph_ab 2000 > "$O/graph_ab.json" 2>&1 ;;
    gaps)  # device idle gaps of the C2 step, from prof2's kernel trace
      local tr; tr=$(find "$O/prof_c2" -name '*kernel_trace.csv' | head -1)
      [ -n "$tr" ] && python3 tools/trace_gaps.py "$tr" --json "$O/gaps_c2.json" > "$O/gaps_c2.txt" 2>&1 ;;
    *) echo "unknown step $1" >&2; return 2 ;;
  esac
}

for s in "$@"; do
  echo "[gpu.sh] $s $(date +%T)"
  step "$s" || { rc=$?; echo "[gpu.sh] step $s failed rc=$rc"; exit $rc; }
done
