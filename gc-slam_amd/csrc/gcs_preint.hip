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

namespace gcs {
namespace {

constexpr int kPreintThreads = 512;
constexpr int kPreintWaves = kPreintThreads / 64;

__device__ __forceinline__ void mat3_id(double* M) {
#pragma unroll
  for (int k = 0; k < 9; ++k) M[k] = (k % 4 == 0) ? 1.0 : 0.0;
}

// C = A B (A, B may alias C)
__device__ __forceinline__ void mat3_mul_inplace(const double* A, const double* B, double* C) {
  double t[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int k = 0; k < 9; ++k) C[k] = t[k];
}

// inclusive left-to-right product scan over one wave: M_lane := M_0 ... M_lane
__device__ __forceinline__ void wave_prod_scan(double* M, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double L[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) L[k] = __shfl_up(M[k], o, 64);
    if (lane >= o) mat3_mul_inplace(L, M, M);
  }
}

template <int NV>
__device__ __forceinline__ void wave_sum_scan(double* v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const double u = __shfl_up(v[k], o, 64);
      if (lane >= o) v[k] += u;
    }
  }
}

template <int NV>
__device__ __forceinline__ void wave_sum(double* v) {
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], sh, 64);
}

__global__ __launch_bounds__(kPreintThreads) void k_preint(PreintArgs a) {
  __shared__ double s_mat[kPreintWaves][9];
  __shared__ double s_vec[kPreintWaves][4];
  __shared__ double s_red[kPreintWaves][4];
  const int tid = (int)threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m = a.m;
  const double* stamps = a.imu;
  const double* gyro = a.imu + m;
  const double* accel = a.imu + 4 * m;
  double R0[9];
  so3_exp(a.rotvec, R0);
  double Pc[9];  // the carry: dR_0 ... dR_{last chunk's end}
  mat3_id(Pc);
  double vc[3] = {0.0, 0.0, 0.0}, pc[3] = {0.0, 0.0, 0.0}, ess = 0.0;
  for (int base = 0; base < m; base += kPreintThreads) {
    const int i = base + tid;
    const bool live = i < m;
    double w = 0.0, dte = 0.0, om[3] = {0.0, 0.0, 0.0}, ab[3] = {0.0, 0.0, 0.0};
    if (live) {
      const double t = stamps[i];
      w = smooth_window(t, a.t0, a.t1, a.sigma);
      double dt = i + 1 < m ? stamps[i + 1] - t : 0.0;
      dt = dt > 0.0 ? dt : 0.0;
      dte = w * dt;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        om[k] = (gyro[3 * i + k] - a.gb[k]) * dte;
        ab[k] = accel[3 * i + k] - a.ab[k];
      }
    }
    // ess: the window's full weight sum (padding included, as the reference's sum over the window)
    double e1[1] = {w};
    wave_sum<1>(e1);
    // 1) dR_i, inclusive product within the chunk
    double P[9];
    if (dte == 0.0) mat3_id(P); else so3_exp(om, P);  // dte == 0: the host's exact identity step
    wave_prod_scan(P, lane);
    if (lane == 63) {
#pragma unroll
      for (int k = 0; k < 9; ++k) s_mat[wid][k] = P[k];
    }
    if (lane == 0) s_red[wid][0] = e1[0];
    __syncthreads();
    double W[9];  // Pc * (totals of the waves before this one)
#pragma unroll
    for (int k = 0; k < 9; ++k) W[k] = Pc[k];
    for (int q = 0; q < wid; ++q) mat3_mul_inplace(W, s_mat[q], W);
    // exclusive prefix at this lane: W * (inclusive product at lane - 1) (W itself at lane 0)
    double X[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const double u = __shfl_up(P[k], 1, 64);
      X[k] = lane == 0 ? (k % 4 == 0 ? 1.0 : 0.0) : u;
    }
    mat3_mul_inplace(W, X, X);
    double Rb[9];
    mat3_mul_inplace(R0, X, Rb);  // R before sample i
    // 2) a_world dte, inclusive sum within the chunk
    double aw[3], dv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      aw[r] = Rb[3 * r] * ab[0] + Rb[3 * r + 1] * ab[1] + Rb[3 * r + 2] * ab[2] + a.g[r];
      dv[r] = aw[r] * dte;
    }
    double V[3] = {dv[0], dv[1], dv[2]};
    wave_sum_scan<3>(V, lane);
    if (lane == 63) {
#pragma unroll
      for (int k = 0; k < 3; ++k) s_vec[wid][k] = V[k];
    }
    __syncthreads();
    double Vw[3] = {vc[0], vc[1], vc[2]};
    for (int q = 0; q < wid; ++q)
#pragma unroll
      for (int k = 0; k < 3; ++k) Vw[k] += s_vec[q][k];
    double vb[3];  // v before sample i: carry + waves before + exclusive lane prefix
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double u = __shfl_up(V[k], 1, 64);
      vb[k] = Vw[k] + (lane == 0 ? 0.0 : u);
    }
    // 3) p increments, reduced over the chunk
    double dp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) dp[k] = vb[k] * dte + 0.5 * aw[k] * (dte * dte);
    wave_sum<3>(dp);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) s_red[wid][1 + k] = dp[k];
    }
    __syncthreads();
    // the carry for the next chunk: Pc * (all 8 wave totals); every lane keeps it (uniform across the workgroup, same fixed order everywhere)
    for (int q = 0; q < kPreintWaves; ++q) {
      mat3_mul_inplace(Pc, s_mat[q], Pc);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        vc[k] += s_vec[q][k];
        pc[k] += s_red[q][1 + k];
      }
      ess += s_red[q][0];
    }
    __syncthreads();  // s_* are rewritten by the next chunk
  }
  if (tid != 0) return;
  // the trimmed run of repeated trailing stamps (the window's padding): zero steps, weight only
  if (a.n_tail > 0) ess += (double)a.n_tail * smooth_window(a.tail_stamp, a.t0, a.t1, a.sigma);
  // the tail (imu_preintegration.py:130-142): R_end = R0 Pc, dR = R0^T R_end
  double Re[9], dR[9], dpose[6], dvel[3], xi[6];
  mat3_mul_inplace(R0, Pc, Re);
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
  hipLaunchKernelGGL(k_preint, dim3(1), dim3(kPreintThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace gcs
