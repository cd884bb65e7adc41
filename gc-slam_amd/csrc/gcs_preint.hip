// IMU window weights + preintegration -> deskew twist on gfx950:
// smooth_window_weights and preintegrate_imu_relative_pose_jax, FS/backend/operators/
// imu_preintegration.py:20-43, 47-147, as the pipeline uses them for the deskew twist
// (pipeline.py:432-483).  The host restatement is gcs_host.cpp preintegrate_imu.
//
// The reference runs a sequential lax.scan over the 512-sample window.  Here the carry is split
// into its associative parts and one workgroup of 512 lanes (one sample per lane) scans them:
//   R_i   = R0 dR_0 ... dR_{i-1}                  prefix PRODUCT of the per-sample Exp((w-bg) w dt)
//   v_i   = sum_{j<i} a_j dte_j                   prefix SUM, a_j = R_j (acc_j - ab) + g
//   p_end = sum_j (v_j dte_j + 1/2 a_j dte_j^2)   a reduction over the exclusive v prefix
// Each scan is a 64-lane shuffle scan per wave, then the 8 wave totals through LDS; windows longer
// than 512 samples run in chunks with the carry (R, v, p) in registers.  Only the association of
// the products / sums differs from the sequential form (rounding level, tested against the oracle
// at 1e-12).  The tail (R0^T R_end, so3_log, se3_log, rotation-only) runs on lane 0.
//
// Inputs arrive through pinned host memory written by the scan prologue (zero-copy reads, no copy
// engine op in the stream); the twist goes to a device word k_points reads (PointKernelArgs.xi_dev)
// and, with ess and the delta pose, to a pinned host record the scan tail reads after its sync.
#include <hip/hip_runtime.h>

#include <math.h>

#include "gcs_kernels.h"
#include "gcs_math.h"
#include "gcs_preint_scan.h"

namespace gcs {
namespace {

__global__ __launch_bounds__(preint::kPreintThreads) void k_preint(PreintArgs a) {
  const int tid = (int)threadIdx.x;
  const int m = a.m;
  const double* stamps = a.imu;
  const double* gyro = a.imu + m;
  const double* accel = a.imu + 4 * m;
  double Pc[9], vc[3], pc[3], ess;
  const double t0 = a.t0, t1 = a.t1, sg = a.sigma;
  preint::window_carry(stamps, gyro, accel, m, [=](int, double t) { return smooth_window(t, t0, t1, sg); }, a.rotvec,
                       a.gb, a.ab, a.g, Pc, vc, pc, ess);
  double R0[9];
  so3_exp(a.rotvec, R0);
  if (tid != 0) return;
  // the trimmed run of repeated trailing stamps (the window's padding): zero steps, weight only
  if (a.n_tail > 0) ess += (double)a.n_tail * smooth_window(a.tail_stamp, a.t0, a.t1, a.sigma);
  // the tail (imu_preintegration.py:130-142): R_end = R0 Pc, dR = R0^T R_end
  double Re[9], dR[9], dpose[6], dvel[3], xi[6];
  preint::mat3_mul_inplace(R0, Pc, Re);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dR[3 * i + j] = R0[i] * Re[j] + R0[3 + i] * Re[3 + j] + R0[6 + i] * Re[6 + j];
  for (int i = 0; i < 3; ++i) dpose[i] = R0[i] * pc[0] + R0[3 + i] * pc[1] + R0[6 + i] * pc[2];
  for (int i = 0; i < 3; ++i) dvel[i] = R0[i] * vc[0] + R0[3 + i] * vc[1] + R0[6 + i] * vc[2];
  so3_log(dR, dpose + 3);
  se3_log_hd(dpose, xi);
  if (a.rotation_only) xi[0] = xi[1] = xi[2] = 0.0;
  for (int k = 0; k < 6; ++k) a.xi_dev[k] = xi[k];
  if (a.host_out) {  // [xi 6, ess, delta_pose 6, delta_v 3]
    for (int k = 0; k < 6; ++k) a.host_out[k] = xi[k];
    a.host_out[6] = ess;
    for (int k = 0; k < 6; ++k) a.host_out[7 + k] = dpose[k];
    for (int k = 0; k < 3; ++k) a.host_out[13 + k] = dvel[k];
  }
}

}  // namespace

hipError_t launch_preint(const PreintArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_preint, dim3(1), dim3(preint::kPreintThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace gcs
