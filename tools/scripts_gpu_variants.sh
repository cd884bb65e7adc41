#!/bin/bash
# A/B of kernel variants (gc-slam_amd/Makefile "variant"): bench C2 and C3 per library, then one
# LDS-counter pass on the default build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in ${VARIANTS:-base pad swz}; do
  lib=gc-slam_amd/gcslam/libgcslam_hip.so
  [ "$v" != base ] && lib=gc-slam_amd/gcslam/libgcslam_hip_$v.so
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/var/${v}_c2.log 2>&1 || exit 1
  GCSLAM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/var/${v}_c3.log 2>&1 || exit 1
done
for cfg in c2 c3; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex 'k_bins_scale' -d gpurun_out/var/pmc_${cfg} -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var/pmc_${cfg}.log 2>&1 || exit 1
done
