// The IMU preintegration's carry as parallel scans over one workgroup (imu_preintegration.py:47-147):
// shared by k_preint (the deskew twist, gcs_preint.hip) and k_imu_odom (the scan-to-scan window of the
// IMU / odometry evidence, gcs_imu_odom.hip).  One sample per lane, windows longer than the workgroup in
// chunks with the carry in registers:
//   R_i   = R0 dR_0 ... dR_{i-1}                  prefix PRODUCT of the per-sample Exp((w-bg) w dt)
//   v_i   = sum_{j<i} a_j dte_j                   prefix SUM, a_j = R_j (acc_j - ab) + g
//   p_end = sum_j (v_j dte_j + 1/2 a_j dte_j^2)   a reduction over the exclusive v prefix
// Only the association of the products / sums differs from the sequential form (rounding level).
#pragma once
#include <hip/hip_runtime.h>

#include "gcs_math.h"

namespace gcs {
namespace preint {

constexpr int kPreintThreads = 512;  // the scan's workgroup
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


// The carry over the whole window: Pc = dR_0 ... dR_{m-1}, vc = v_end, pc = p_end (world frame, from
// R0 = Exp(rotvec)), ess = the sum of the weights.  weight(i, t) gives sample i's weight; every lane of
// the kPreintThreads-lane workgroup calls it and gets the same carry (uniform, fixed order).
template <class Weight>
__device__ void window_carry(const double* stamps, const double* gyro, const double* accel, int m, Weight weight,
                             const double* rotvec, const double* gbias, const double* abias, const double* grav,
                             double* Pc, double* vc, double* pc, double& ess) {
  __shared__ double s_mat[kPreintWaves][9];
  __shared__ double s_vec[kPreintWaves][4];
  __shared__ double s_red[kPreintWaves][4];
  const int tid = (int)threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double R0[9];
  so3_exp(rotvec, R0);
  mat3_id(Pc);  // the carry: dR_0 ... dR_{last chunk's end}
  for (int k = 0; k < 3; ++k) vc[k] = pc[k] = 0.0;
  ess = 0.0;
  for (int base = 0; base < m; base += kPreintThreads) {
    const int i = base + tid;
    const bool live = i < m;
    double w = 0.0, dte = 0.0, om[3] = {0.0, 0.0, 0.0}, ab[3] = {0.0, 0.0, 0.0};
    if (live) {
      const double t = stamps[i];
      w = weight(i, t);
      double dt = i + 1 < m ? stamps[i + 1] - t : 0.0;
      dt = dt > 0.0 ? dt : 0.0;
      dte = w * dt;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        om[k] = (gyro[3 * i + k] - gbias[k]) * dte;
        ab[k] = accel[3 * i + k] - abias[k];
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
      aw[r] = Rb[3 * r] * ab[0] + Rb[3 * r + 1] * ab[1] + Rb[3 * r + 2] * ab[2] + grav[r];
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
}

}  // namespace preint
}  // namespace gcs
