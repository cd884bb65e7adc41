// LiDAR surfel extraction on gfx950 -- the first operator of the live primitive path
// (SURVEY.md 8(f) rank 2): extract_lidar_surfels, FS/backend/operators/lidar_surfel_extraction.py:
// 339-431, with the MA-hex 3D bucketing of FS/common/ma_hex_web.py:221-303 and the LiDAR slice of
// FS/backend/structures/measurement_batch.py:272-381.
//
//   k_sf_partials   weighted centre partial sums (sentinel mask, :259-266), fixed-order block trees;
//                   also clears the per-cell run bounds
//   k_sf_keys       every block folds the partials in the same fixed tree (the centre), then per
//                   point the hash-grid cell of the centred point (masked points -> key n_cells)
//   radix sort      stable (rocPRIM LSD radix sort on the cell key, point index as value): the
//                   reference's stable argsort by (masked, cell) (ma_hex_web.py:276-280)
//   k_sf_bounds     per sorted point: the first / last position of each cell's run
//   k_sf_cells      per cell: the first max_occupants indices, the clipped count (:284-303)
//   k_sf_moments    one wave per occupied cell: weight, centroid, time and scatter sums over the
//                   occupants in fixed xor trees (lidar_surfel_extraction.py:113-126)
//   k_sf_fit        one lane per cell: eigh, normal, in-plane variances, Wishart-regularised
//                   covariance, kappa, validity (:126-163)
//   k_sf_slots      one workgroup: valid cells in cell-id order -> slots (:297-305)
//   k_sf_write      one lane per slot: the surfel rows and the information form of the LiDAR
//                   slice (:307-321, measurement_batch.py:298-331), padding past n_valid
// Everything is fixed-order (no floating-point atomics): results are bitwise reproducible.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "gcs_math.h"
#include "gcslam_hip.h"
#include "gcs_live.h"

namespace gcs {
namespace {

constexpr int kSfThreads = 256;
constexpr int kSfMaxPartials = 256;
constexpr int kSelThreads = 1024;
constexpr double kSentinelBound = 0.1 * 1e6;       // 0.1 * GC_NONFINITE_SENTINEL (:261)
constexpr double kSqrt3Half = 0.8660254037844386;  // sqrt(3.0) * 0.5 in f64 (ma_hex_web.py:235)
constexpr double kFitEps = 1e-12;                  // eps of _fit_one_cell / _normalize
constexpr int kFitFields = 18;                     // centroid 3 | Sigma_reg 9 | normal 3 | kappa | w | t

struct SfParams {
  int n_cells, n1, n2, nz, max_occ, min_points, n_surfel;
  double h, sensor_var, wishart_nu, wishart_psi, kappa_scale, kappa_min, kappa_max, eig_min, eps_lift;
};

__device__ __forceinline__ bool sf_mask(double x, double y, double z) {
  return fabs(x) < kSentinelBound && fabs(y) < kSentinelBound && fabs(z) < kSentinelBound;
}

// per block: sum over its grid-stride points of (x w_eff, y w_eff, z w_eff, w_eff), w_eff = w * mask
__global__ __launch_bounds__(kSfThreads) void k_sf_partials(const double* __restrict__ p,
                                                             const double* __restrict__ w, int n,
                                                             double* __restrict__ partials, int32_t* __restrict__ run,
                                                             int n_run) {
  __shared__ double lds[kSfThreads / 64][4];
  for (int j = blockIdx.x * kSfThreads + threadIdx.x; j < n_run; j += gridDim.x * kSfThreads) run[j] = 0;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = blockIdx.x * kSfThreads + threadIdx.x; i < n; i += gridDim.x * kSfThreads) {
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    const double we = w[i] * (sf_mask(x, y, z) ? 1.0 : 0.0);
    v[0] += x * we;
    v[1] += y * we;
    v[2] += z * we;
    v[3] += we;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += __shfl_xor(v[k], off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) lds[wid][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double s = lds[0][k];
      for (int q = 1; q < kSfThreads / 64; ++q) s += lds[q][k];
      partials[4 * blockIdx.x + k] = s;
    }
}

// cell key of every point around the weighted centre (hex_cell_3d_batch + bin_points_3d's wrap,
// linear index and mask); numpy's operation order, no contraction
__global__ __launch_bounds__(kSfThreads) void k_sf_keys(const double* __restrict__ p, int n,
                                                         const double* __restrict__ partials, int nblk,
                                                         SfParams a, uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals, double* __restrict__ center_out,
                                                         double* __restrict__ center_host) {
#pragma clang fp contract(off)
  __shared__ double s_c[3];
  __shared__ double lds[kSfThreads / 64][4];
  {  // the partial rows in one fixed tree (row t on thread t, nblk <= kSfThreads), same in every block
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if ((int)threadIdx.x < nblk)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = partials[4 * threadIdx.x + k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += __shfl_xor(v[k], off, 64);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) lds[threadIdx.x >> 6][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      double sm[4];
      for (int k = 0; k < 4; ++k) {
        sm[k] = lds[0][k];
        for (int q = 1; q < kSfThreads / 64; ++q) sm[k] += lds[q][k];
      }
      const double ws = sm[3] + a.eig_min;
      for (int k = 0; k < 3; ++k) s_c[k] = sm[k] / ws;
      if (blockIdx.x == 0)
        for (int k = 0; k < 3; ++k) {
          center_out[k] = s_c[k];
          center_host[k] = s_c[k];
        }
    }
    __syncthreads();
  }
  const double cx = s_c[0], cy = s_c[1], cz = s_c[2];
  for (int i = blockIdx.x * kSfThreads + threadIdx.x; i < n; i += gridDim.x * kSfThreads) {
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    uint32_t key = (uint32_t)a.n_cells;
    if (sf_mask(x, y, z)) {
      const double px = x - cx, py = y - cy, pz = z - cz;
      const double s2 = px * 0.5 + py * kSqrt3Half;
      long long c1 = (long long)floor(px / a.h), c2 = (long long)floor(s2 / a.h), c3 = (long long)floor(pz / a.h);
      c1 = ((c1 % a.n1) + a.n1) % a.n1;
      c2 = ((c2 % a.n2) + a.n2) % a.n2;
      c3 = ((c3 % a.nz) + a.nz) % a.nz;
      key = (uint32_t)(c1 * (a.n2 * a.nz) + c2 * a.nz + c3);
    }
    keys[i] = key;
    vals[i] = (uint32_t)i;
  }
}

// run bounds of every cell in the sorted keys: start and end (one past), 0/0 = empty
__global__ __launch_bounds__(kSfThreads) void k_sf_bounds(const uint32_t* __restrict__ keys_s, int n, int n_cells,
                                                           int32_t* __restrict__ run) {
  const int q = blockIdx.x * kSfThreads + threadIdx.x;
  if (q >= n) return;
  const uint32_t k = keys_s[q];
  if (k >= (uint32_t)n_cells) return;  // masked points sort last
  if (q == 0 || keys_s[q - 1] != k) run[2 * k] = q;
  if (q == n - 1 || keys_s[q + 1] != k) run[2 * k + 1] = q + 1;
}

// per (cell, occupant slot): the first max_occ point indices of the cell's run (stable: index
// order) and the clipped count -- one thread per bucket entry, so an occupied cell's entries cost one
// dependent round trip (run bounds, then the index), not one per occupant
__global__ __launch_bounds__(kSfThreads) void k_sf_cells(const int32_t* __restrict__ run,
                                                          const uint32_t* __restrict__ vals_s, SfParams a,
                                                          int32_t* __restrict__ bucket, int32_t* __restrict__ count) {
  const long j = (long)blockIdx.x * kSfThreads + threadIdx.x;
  if (j >= (long)a.n_cells * a.max_occ) return;
  const int k = (int)(j / a.max_occ), r = (int)(j - (long)k * a.max_occ);
  const int s = run[2 * k], e = run[2 * k + 1];
  const int c = min(e - s, a.max_occ);
  if (r == 0) count[k] = c;
  bucket[j] = r < c ? (int32_t)vals_s[s + r] : -1;
}

__device__ __forceinline__ void normalize3(double* v) {
  const double nr = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) + kFitEps;
  v[0] /= nr; v[1] /= nr; v[2] /= nr;
}

__device__ __forceinline__ void sym_plus_diag(double* M, double d) {
  const double m01 = 0.5 * (M[1] + M[3]), m02 = 0.5 * (M[2] + M[6]), m12 = 0.5 * (M[5] + M[7]);
  M[1] = M[3] = m01; M[2] = M[6] = m02; M[5] = M[7] = m12;
  M[0] += d; M[4] += d; M[8] += d;
}

template <int NV>
__device__ __forceinline__ void sf_wave_sum(double (&v)[NV]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], off, 64);
}

// Occupant sums of one cell per wave (lidar_surfel_extraction.py:113-126; absent slots carry zero
// weight in the reference and add exact zeros): lane r holds occupant r, the sums meet in fixed
// xor trees.  Moment row = sum w, centroid (3), sum t, sum w d d^T (xx xy xz yy yz zz).
constexpr int kMomFields = 11;
constexpr int kCellsPerBlock = kSfThreads / 64;
// run / vals_s (may be null: the bucket rows of k_sf_cells are read instead): the wave also writes its
// cell's bucket row and clipped count from the sorted run (k_sf_cells folded in: one launch fewer,
// the same rows) and reads the occupants from the run
__global__ __launch_bounds__(kSfThreads) void k_sf_moments(const double* __restrict__ p, const double* __restrict__ t,
                                                            const double* __restrict__ w,
                                                            const double* __restrict__ center,
                                                            int32_t* __restrict__ bucket,
                                                            int32_t* __restrict__ count, SfParams a,
                                                            double* __restrict__ mom, const int32_t* __restrict__ run,
                                                            const uint32_t* __restrict__ vals_s) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * kCellsPerBlock + (threadIdx.x >> 6);
  if (k >= a.n_cells) return;  // wave-uniform
  int c;
  const int32_t* row;
  if (run) {
    const int s0 = run[2 * k], e0 = run[2 * k + 1];
    c = min(e0 - s0, a.max_occ);
    int32_t* brow = bucket + (size_t)k * a.max_occ;
    for (int r = lane; r < a.max_occ; r += 64) brow[r] = r < c ? (int32_t)vals_s[s0 + r] : -1;
    if (lane == 0) count[k] = c;
    row = reinterpret_cast<const int32_t*>(vals_s + s0);
  } else {
    c = count[k];
    row = bucket + (size_t)k * a.max_occ;
  }
  if (c == 0) return;          // k_sf_fit does not read the row of an empty cell
  const double cx = center[0], cy = center[1], cz = center[2];
  double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // w, w x, w y, w z, t
  double px[2] = {0.0, 0.0}, py[2] = {0.0, 0.0}, pz[2] = {0.0, 0.0}, pw[2] = {0.0, 0.0};
  for (int r = lane, u = 0; r < c; r += 64, ++u) {
    const int i = row[r];
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    const double we = w[i];  // occupants are unmasked points: w_eff = w * 1
    s5[0] += we;
    s5[1] += (x - cx) * we;
    s5[2] += (y - cy) * we;
    s5[3] += (z - cz) * we;
    s5[4] += t[i];
    if (u < 2) { px[u] = x - cx; py[u] = y - cy; pz[u] = z - cz; pw[u] = we; }
  }
  sf_wave_sum<5>(s5);
  const double wsum = s5[0] + kFitEps;
  const double m[3] = {s5[1] / wsum, s5[2] / wsum, s5[3] / wsum};
  double c6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int r = lane, u = 0; r < c; r += 64, ++u) {
    double x, y, z, we;
    if (u < 2) { x = px[u]; y = py[u]; z = pz[u]; we = pw[u]; }
    else {
      const int i = row[r];
      x = p[3 * (size_t)i] - cx; y = p[3 * (size_t)i + 1] - cy; z = p[3 * (size_t)i + 2] - cz;
      we = w[i];
    }
    const double d0 = x - m[0], d1 = y - m[1], d2 = z - m[2];
    c6[0] += d0 * we * d0; c6[1] += d0 * we * d1; c6[2] += d0 * we * d2;
    c6[3] += d1 * we * d1; c6[4] += d1 * we * d2; c6[5] += d2 * we * d2;
  }
  sf_wave_sum<6>(c6);
  double f = 0.0;
  if (lane == 0) f = s5[0];
  else if (lane < 4) f = m[lane - 1];
  else if (lane == 4) f = s5[4];
  else if (lane < 11) f = c6[lane - 5];
  if (lane < kMomFields) mom[(size_t)k * kMomFields + lane] = f;
}

// The rest of _fit_one_cell (:126-163), one lane per cell.  The in-plane variances are the
// quadratic forms e^T (sum w d d^T) e / w_sum (the reference sums w (d.e)^2 point by point: equal
// up to rounding).  Fit row = centroid (+ centre) | Sigma_reg | normal | kappa | w_surfel | t_surfel.
__global__ __launch_bounds__(kSfThreads) void k_sf_fit(const double* __restrict__ mom,
                                                        const double* __restrict__ center,
                                                        const int32_t* __restrict__ count, SfParams a,
                                                        double* __restrict__ fit, uint8_t* __restrict__ valid) {
  const int k = blockIdx.x * kSfThreads + threadIdx.x;
  if (k >= a.n_cells) return;
  const int c = count[k];
  if (c == 0) {  // never valid (w_surfel = 0): the fit row is not read
    valid[k] = 0;
    return;
  }
  const double* mo = mom + (size_t)k * kMomFields;
  const double ws = mo[0], wsum = ws + kFitEps;
  const double m[3] = {mo[1], mo[2], mo[3]};
  const double* c6 = mo + 5;
  double C[9] = {c6[0] / wsum, c6[1] / wsum, c6[2] / wsum, c6[1] / wsum, c6[3] / wsum,
                 c6[4] / wsum, c6[2] / wsum, c6[4] / wsum, c6[5] / wsum};
  sym_plus_diag(C, a.eig_min);
  double ev[3], V[9];
  eigh3_jacobi(C, ev, V);
  int im = 0;
  if (ev[1] < ev[im]) im = 1;
  if (ev[2] < ev[im]) im = 2;
  double nrm[3] = {V[im], V[3 + im], V[6 + im]};
  if (nrm[2] < 0.0) { nrm[0] = -nrm[0]; nrm[1] = -nrm[1]; nrm[2] = -nrm[2]; }
  normalize3(nrm);
  // _orthonormal_basis_from_normal (:72-81)
  double n2[3] = {nrm[0], nrm[1], nrm[2]};
  normalize3(n2);
  double e1[3];
  if (fabs(n2[2]) < 0.9) { e1[0] = -n2[1]; e1[1] = n2[0]; e1[2] = 0.0; }
  else { e1[0] = -n2[2]; e1[1] = 0.0; e1[2] = n2[0]; }
  normalize3(e1);
  double e2[3];
  cross3(n2, e1, e2);
  normalize3(e2);
  const double S6[9] = {c6[0], c6[1], c6[2], c6[1], c6[3], c6[4], c6[2], c6[4], c6[5]};
  auto quad = [&](const double* e) {
    double q = 0.0;
#pragma unroll
    for (int u = 0; u < 3; ++u) q += e[u] * (S6[3 * u] * e[0] + S6[3 * u + 1] * e[1] + S6[3 * u + 2] * e[2]);
    return q;
  };
  const double var_e1 = quad(e1) / wsum + a.sensor_var, var_e2 = quad(e2) / wsum + a.sensor_var;
  const double sps = fmax(ev[im], a.eig_min);
  const double var_perp = sps + a.sensor_var;
  const double D[3] = {fmax(var_e1, a.eig_min), fmax(var_e2, a.eig_min), fmax(var_perp, a.eig_min)};
  const double Bm[9] = {e1[0], e2[0], nrm[0], e1[1], e2[1], nrm[1], e1[2], e2[2], nrm[2]};  // columns e1 e2 n
  double Sg[9];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int v = 0; v < 3; ++v)
      Sg[3 * u + v] = Bm[3 * u] * D[0] * Bm[3 * v] + Bm[3 * u + 1] * D[1] * Bm[3 * v + 1] + Bm[3 * u + 2] * D[2] * Bm[3 * v + 2];
  sym_plus_diag(Sg, a.eig_min);
  double A[9], Lam[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) A[q] = Sg[q];
  A[0] += a.eig_min; A[4] += a.eig_min; A[8] += a.eig_min;
  inv3(A, Lam);
  sym_plus_diag(Lam, 0.0);
  const double psi = fmax(a.wishart_psi, kFitEps);
  const double nu_psi = a.wishart_nu / psi;
  Lam[0] += nu_psi; Lam[4] += nu_psi; Lam[8] += nu_psi;
  sym_plus_diag(Lam, a.eig_min);
  double Sr[9];
  inv3(Lam, Sr);
  sym_plus_diag(Sr, a.eig_min);
  double kap = a.kappa_scale / sqrt(fmax(sps, a.eig_min));
  kap = fmin(fmax(kap, a.kappa_min), a.kappa_max);
  double* out = fit + (size_t)k * kFitFields;
  out[0] = m[0] + center[0];
  out[1] = m[1] + center[1];
  out[2] = m[2] + center[2];
#pragma unroll
  for (int q = 0; q < 9; ++q) out[3 + q] = Sr[q];
  out[12] = nrm[0]; out[13] = nrm[1]; out[14] = nrm[2];
  out[15] = kap;
  out[16] = ws;
  out[17] = mo[4] / wsum;
  valid[k] = (c >= a.min_points && ws > 0.0) ? 1 : 0;
}

struct SelOut {
  double *positions, *covariances, *normals, *kappas, *weights, *timestamps;
  double *Lambdas, *thetas, *etas, *colors;
  uint8_t* valid_mask;
  int32_t *source_indices, *cell_ids, *sources;
};

// one workgroup: valid cells in cell-id order -> slot_cell[slot], n_valid (device + mapped host)
__global__ __launch_bounds__(kSelThreads) void k_sf_slots(const uint8_t* __restrict__ valid, SfParams a,
                                                           int32_t* __restrict__ slot_cell, int32_t* __restrict__ nv_dev,
                                                           int32_t* __restrict__ nv_host) {
  __shared__ int s_wsum[kSelThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int per = (a.n_cells + kSelThreads - 1) / kSelThreads;
  const int k0 = min(a.n_cells, t * per), k1 = min(a.n_cells, k0 + per);
  // the thread's first kSelBatch flags loaded together (one round trip for grids up to
  // kSelBatch x kSelThreads cells), the rest one by one
  constexpr int kSelBatch = 16;
  uint8_t vb[kSelBatch];
#pragma unroll
  for (int u = 0; u < kSelBatch; ++u) vb[u] = k0 + u < k1 ? valid[k0 + u] : (uint8_t)0;
  int mine = 0;
#pragma unroll
  for (int u = 0; u < kSelBatch; ++u) mine += vb[u];
  for (int k = k0 + kSelBatch; k < k1; ++k) mine += valid[k];
  int x = mine;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  int run = x - mine;
  for (int q = 0; q < wid; ++q) run += s_wsum[q];
#pragma unroll
  for (int u = 0; u < kSelBatch; ++u)
    if (vb[u] && run < a.n_surfel) slot_cell[run++] = k0 + u;
  for (int k = k0 + kSelBatch; k < k1 && run < a.n_surfel; ++k)
    if (valid[k]) slot_cell[run++] = k;
  if (t == kSelThreads - 1) {
    int tot = 0;
    for (int q = 0; q < kSelThreads / 64; ++q) tot += s_wsum[q];
    const int nv = min(tot, a.n_surfel);
    *nv_dev = nv;
    *nv_host = nv;
  }
}

// one lane per slot: the surfel row of its cell and the LiDAR slice in information form, or the
// reference's padding past n_valid
__global__ __launch_bounds__(kSfThreads) void k_sf_write(const double* __restrict__ fit,
                                                          const int32_t* __restrict__ slot_cell,
                                                          const int32_t* __restrict__ nv_dev, SfParams a, SelOut o) {
  const int s = blockIdx.x * kSfThreads + threadIdx.x;
  if (s >= a.n_surfel) return;
  if (s >= *nv_dev) {
    if (o.positions) for (int q = 0; q < 3; ++q) o.positions[3 * s + q] = 0.0;
    if (o.covariances) for (int q = 0; q < 9; ++q) o.covariances[9 * s + q] = (q % 4 == 0) ? 1.0 : 0.0;
    if (o.normals) for (int q = 0; q < 3; ++q) o.normals[3 * s + q] = 0.0;
    if (o.kappas) o.kappas[s] = 0.0;
    if (o.weights) o.weights[s] = 0.0;
    if (o.timestamps) o.timestamps[s] = 0.0;
    if (o.cell_ids) o.cell_ids[s] = -1;
    if (o.Lambdas) for (int q = 0; q < 9; ++q) o.Lambdas[9 * s + q] = 0.0;
    if (o.thetas) for (int q = 0; q < 3; ++q) o.thetas[3 * s + q] = 0.0;
    if (o.etas) for (int q = 0; q < 9; ++q) o.etas[9 * s + q] = 0.0;
    if (o.colors) for (int q = 0; q < 3; ++q) o.colors[3 * s + q] = 0.0;
    if (o.valid_mask) o.valid_mask[s] = 0;
    if (o.source_indices) o.source_indices[s] = 0;
    return;
  }
  const int k = slot_cell[s];
  const double* f = fit + (size_t)k * kFitFields;
  double pos[3], S[9], nrm[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) { pos[q] = f[q]; nrm[q] = f[12 + q]; }
#pragma unroll
  for (int q = 0; q < 9; ++q) S[q] = f[3 + q];
  const double kap = f[15];
  if (o.positions) for (int q = 0; q < 3; ++q) o.positions[3 * s + q] = pos[q];
  if (o.covariances) for (int q = 0; q < 9; ++q) o.covariances[9 * s + q] = S[q];
  if (o.normals) for (int q = 0; q < 3; ++q) o.normals[3 * s + q] = nrm[q];
  if (o.kappas) o.kappas[s] = kap;
  if (o.weights) o.weights[s] = f[16];
  if (o.timestamps) o.timestamps[s] = f[17];
  if (o.cell_ids) o.cell_ids[s] = k;
  // measurement_batch_add_lidar_surfels (measurement_batch.py:298-312)
  double A[9], L[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) A[q] = S[q];
  A[0] += a.eps_lift; A[4] += a.eps_lift; A[8] += a.eps_lift;
  inv3(A, L);
  if (o.Lambdas) for (int q = 0; q < 9; ++q) o.Lambdas[9 * s + q] = L[q];
  if (o.thetas)
    for (int q = 0; q < 3; ++q) o.thetas[3 * s + q] = L[3 * q] * pos[0] + L[3 * q + 1] * pos[1] + L[3 * q + 2] * pos[2];
  if (o.etas)
    for (int q = 0; q < 9; ++q) o.etas[9 * s + q] = q < 3 ? kap * nrm[q] : 0.0;
  if (o.colors) {
    const double nz = fmin(fmax(nrm[2], -1.0), 1.0);
    const double g = 0.25 + 0.5 * (nz + 1.0) / 2.0;
    for (int q = 0; q < 3; ++q) o.colors[3 * s + q] = g;
  }
  if (o.valid_mask) o.valid_mask[s] = 1;
  if (o.source_indices) o.source_indices[s] = s;
  if (o.sources) o.sources[s] = 1;  // measurement_batch_add_lidar_surfels: LiDAR rows
}

// One workgroup for clouds of up to kSortMax points: the stable sort of k_sf_keys' (key, point index)
// pairs by key and k_sf_bounds' run bounds, in LDS (replaces the rocPRIM radix sort's kernels and
// k_sf_bounds: the same permutation, as both sorts are stable on the key with the points in index
// order).  Each key is packed above its IDXB-bit index and sorted by LSD passes of 7-bit digits: per
// wave a contiguous segment in 64-lane steps, equal digits found by ballots, ranks from per-(wave,
// digit) offsets (digit-major, then wave order).  IDXB 13: up to 8,192 points (the reference's
// N_POINTS_CAP; 64 KB of LDS); IDXB 14: up to 16,384 (twice it; 128 KB of the CU's 160 KB).
constexpr int kSortThreads = 1024;
constexpr int kSortIdxBits = 13;
constexpr int kSortMax = 1 << kSortIdxBits;
constexpr int kSortMaxWide = 2 * kSortMax;
constexpr int kSortDigitBits = 7;
constexpr int kSortDigits = 1 << kSortDigitBits;
constexpr int kSortWaves = kSortThreads / 64;

template <int IDXB>
__global__ __launch_bounds__(kSortThreads) void k_sf_sort_lds(const uint32_t* __restrict__ keys, int n, SfParams a,
                                                               int end_bit, uint32_t* __restrict__ vals_s,
                                                               int32_t* __restrict__ run) {
  constexpr int kSortMax = 1 << IDXB, kSortIdxBits = IDXB;
  constexpr int kSortSeg = kSortMax / kSortWaves;  // entries per wave
  static_assert(kSortThreads <= 1024 && kSortSeg % 64 == 0, "sort shape");
  __shared__ uint32_t s_buf[2][kSortMax];
  __shared__ uint32_t s_off[kSortWaves][kSortDigits];
  __shared__ uint32_t s_tot[kSortDigits], s_dsum[kSortDigits / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  {  // every key load issued before the first LDS store (one round trip, not one per key)
    constexpr int KPT = kSortMax / kSortThreads;
    uint32_t kv[KPT];
#pragma unroll
    for (int u = 0; u < KPT; ++u) kv[u] = t + u * kSortThreads < n ? keys[t + u * kSortThreads] : 0u;
#pragma unroll
    for (int u = 0; u < KPT; ++u)
      if (t + u * kSortThreads < n) s_buf[0][t + u * kSortThreads] = (kv[u] << kSortIdxBits) | (uint32_t)(t + u * kSortThreads);
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int npass = (end_bit + kSortDigitBits - 1) / kSortDigitBits;
  for (int pass = 0; pass < npass; ++pass) {
    const uint32_t* src = s_buf[pass & 1];
    uint32_t* dst = s_buf[(pass + 1) & 1];
    const int shift = kSortIdxBits + pass * kSortDigitBits;
    for (int q = t; q < kSortWaves * kSortDigits; q += kSortThreads) (&s_off[0][0])[q] = 0u;
    __syncthreads();
    // per (wave, digit) counts.  Each entry's word, digit and peer mask (the wave's lanes with the same
    // digit) are kept in registers for the scatter.  The peer mask is the AND over the digit's bits of
    // the bit's ballot or its complement, as ~(ballot ^ -bit): a few VALU ops per bit (the pass is
    // VALU-bound: 16 waves on one CU).
    constexpr int kIt = kSortSeg / 64;
    uint32_t xv[kIt], dv[kIt];
    uint64_t pv[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int e = wid * kSortSeg + it * 64 + lane;
      xv[it] = dv[it] = 0u;
      pv[it] = 0ull;
      if (wid * kSortSeg + it * 64 >= n) continue;  // wave-uniform: no entry in this step
      const bool ok = e < n;
      const uint32_t x = ok ? src[e] : 0u;
      const uint32_t d = (x >> shift) & (kSortDigits - 1);
      uint64_t peers = __builtin_amdgcn_ballot_w64(ok);
#pragma unroll
      for (int b = 0; b < kSortDigitBits; ++b) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t m = __builtin_amdgcn_ballot_w64(bit != 0u);
        peers &= ~(m ^ (0ull - (uint64_t)bit));
      }
      if (!ok) peers = 0ull;
      xv[it] = x;
      dv[it] = d;
      pv[it] = peers;
      if (ok && (peers & lt) == 0ull) s_off[wid][d] += (uint32_t)__popcll(peers);  // the group's first lane
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // offsets: digit-major, then wave order (thread d owns digit d)
    if (t < kSortDigits) {
      uint32_t tot = 0;
      for (int w = 0; w < kSortWaves; ++w) tot += s_off[w][t];
      uint32_t x = tot;  // inclusive scan over the digits: per wave, then the waves in order
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) s_dsum[wid] = x;
      s_tot[t] = x - tot;  // exclusive within the wave
    }
    __syncthreads();
    if (t < kSortDigits) {
      uint32_t r = s_tot[t];
      for (int w = 0; w < wid; ++w) r += s_dsum[w];
      for (int w = 0; w < kSortWaves; ++w) {
        const uint32_t c = s_off[w][t];
        s_off[w][t] = r;
        r += c;
      }
    }
    __syncthreads();
    // scatter: each wave's entries in order, equal digits by lane order
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const uint64_t peers = pv[it];
      const uint32_t d = dv[it];
      if (peers) dst[s_off[wid][d] + (uint32_t)__popcll(peers & lt)] = xv[it];
      __builtin_amdgcn_wave_barrier();
      if (peers && (peers & lt) == 0ull) s_off[wid][d] += (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
  }
  // sorted point indices and k_sf_bounds' runs (run[] zeroed by k_sf_partials)
  const uint32_t* srt = s_buf[npass & 1];
  for (int q = t; q < n; q += kSortThreads) {
    const uint32_t x = srt[q];
    vals_s[q] = x & (kSortMax - 1);
    const uint32_t k = x >> kSortIdxBits;
    if (k >= (uint32_t)a.n_cells) continue;  // masked points sort last
    if (q == 0 || (srt[q - 1] >> kSortIdxBits) != k) run[2 * k] = q;
    if (q == n - 1 || (srt[q + 1] >> kSortIdxBits) != k) run[2 * k + 1] = q + 1;
  }
}

}  // namespace
}  // namespace gcs

using namespace gcs;

struct gcs_surfel_ctx {
  gcs_surfel_config cfg{};
  SfParams prm{};
  std::string err;
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  double* d_partials = nullptr;
  uint32_t *d_keys = nullptr, *d_vals = nullptr, *d_keys_s = nullptr, *d_vals_s = nullptr;
  void* d_temp = nullptr;
  size_t temp_bytes = 0;
  unsigned end_bit = 1;
  bool lds_sort = true;  // k_sf_sort_lds for clouds of <= kSortMaxWide points (GCSLAM_SF_LDS_SORT=0: rocPRIM)
  bool fold_cells = true;  // k_sf_moments writes the bucket rows (GCSLAM_SF_FOLD_CELLS=0: k_sf_cells)
  int32_t *d_bucket = nullptr, *d_count = nullptr, *d_run = nullptr, *d_slot_cell = nullptr;
  double *d_mom = nullptr, *d_fit = nullptr;
  uint8_t* d_valid = nullptr;
  double* d_scal = nullptr;   // device: center[3], n_valid (int32 in the 4th slot)
  double* h_scal = nullptr;   // pinned, mapped: the same, written by the kernels (no copy)
  double* h_scal_dev = nullptr;
};

namespace {
int sf_fail(gcs_surfel_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}
#define SFCHK(ctx, expr)                                                                          \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return sf_fail((ctx), GCS_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)
}  // namespace

extern "C" {

int gcs_surfel_config_defaults(gcs_surfel_config* c) {
  if (!c) return GCS_ERR_ARG;
  memset(c, 0, sizeof(*c));
  c->n_surfel = 1024;   // GC_N_SURFEL, constants.py:353
  c->n_feat = 512;      // GC_N_FEAT, constants.py:350
  c->voxel_size_m = 0.1;
  c->num_cells_1 = 32;
  c->num_cells_2 = 32;
  c->num_cells_z = 8;
  c->max_occupants = 32;
  c->min_points_per_voxel = 3;
  c->sensor_noise_var_per_axis = 1e-6;
  c->wishart_nu = 5.0;
  c->wishart_psi_scale = 0.1;
  c->kappa_main_scale = 10.0;
  c->kappa_min = 0.1;
  c->kappa_max = 100.0;
  c->eig_min = 1e-12;
  c->eps_lift = 1e-9;   // GC_EPS_LIFT, constants.py:71
  c->max_points = 65536;
  c->device = 0;
  return GCS_OK;
}

const char* gcs_surfel_last_error(const gcs_surfel_ctx* c) { return c ? c->err.c_str() : "null surfel context"; }

int gcs_surfel_ctx_destroy(gcs_surfel_ctx* c) {
  if (!c) return GCS_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_partials, c->d_keys, c->d_vals, c->d_keys_s, c->d_vals_s, c->d_temp,
                  c->d_bucket, c->d_count, c->d_run, c->d_slot_cell, c->d_mom, c->d_fit, c->d_valid, c->d_scal};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->h_scal) (void)hipHostFree(c->h_scal);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return GCS_OK;
}

int gcs_surfel_ctx_create(const gcs_surfel_config* cfg, gcs_surfel_ctx** out) {
  if (!cfg || !out) return GCS_ERR_ARG;
  *out = nullptr;
  const long n_cells = (long)cfg->num_cells_1 * cfg->num_cells_2 * cfg->num_cells_z;
  if (cfg->num_cells_1 < 1 || cfg->num_cells_2 < 1 || cfg->num_cells_z < 1 || n_cells > (1L << 24) ||
      cfg->max_occupants < 1 || cfg->max_occupants > 1024 || cfg->n_surfel < 1 || cfg->n_surfel > n_cells ||
      cfg->n_feat < 0 || cfg->max_points < 1 || !(cfg->voxel_size_m > 0.0) || cfg->min_points_per_voxel < 0)
    return GCS_ERR_ARG;  // n_surfel <= n_cells: the reference takes n_surfel of the cell order (:302)
  auto* c = new gcs_surfel_ctx();
  c->cfg = *cfg;
  c->device = cfg->device;
  SfParams& a = c->prm;
  a.n_cells = (int)n_cells;
  a.n1 = cfg->num_cells_1; a.n2 = cfg->num_cells_2; a.nz = cfg->num_cells_z;
  a.max_occ = cfg->max_occupants;
  a.min_points = cfg->min_points_per_voxel;
  a.n_surfel = cfg->n_surfel;
  a.h = std::max(cfg->voxel_size_m, 1e-12);
  a.sensor_var = cfg->sensor_noise_var_per_axis;
  a.wishart_nu = cfg->wishart_nu;
  a.wishart_psi = cfg->wishart_psi_scale;
  a.kappa_scale = cfg->kappa_main_scale;
  a.kappa_min = cfg->kappa_min;
  a.kappa_max = cfg->kappa_max;
  a.eig_min = cfg->eig_min;
  a.eps_lift = cfg->eps_lift;
  while ((1UL << c->end_bit) <= (unsigned long)n_cells) ++c->end_bit;  // keys 0..n_cells
  if (const char* e = getenv("GCSLAM_SF_LDS_SORT")) c->lds_sort = atoi(e) != 0;
  if (const char* e = getenv("GCSLAM_SF_FOLD_CELLS")) c->fold_cells = atoi(e) != 0;
  auto bad = [&](hipError_t e) { return e != hipSuccess; };
  const size_t N = (size_t)cfg->max_points;
  if (bad(hipSetDevice(cfg->device)) || bad(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) ||
      bad(hipMalloc(&c->d_partials, kSfMaxPartials * 4 * sizeof(double))) ||
      bad(hipMalloc(&c->d_keys, N * 4)) || bad(hipMalloc(&c->d_vals, N * 4)) ||
      bad(hipMalloc(&c->d_keys_s, N * 4)) || bad(hipMalloc(&c->d_vals_s, N * 4)) ||
      bad(hipMalloc(&c->d_bucket, (size_t)n_cells * a.max_occ * 4)) || bad(hipMalloc(&c->d_count, n_cells * 4)) ||
      bad(hipMalloc(&c->d_fit, (size_t)n_cells * kFitFields * sizeof(double))) ||
      bad(hipMalloc(&c->d_valid, n_cells)) || bad(hipMalloc(&c->d_scal, 4 * sizeof(double))) ||
      bad(hipMalloc(&c->d_run, (size_t)n_cells * 2 * 4)) || bad(hipMalloc(&c->d_slot_cell, (size_t)cfg->n_surfel * 4)) ||
      bad(hipMalloc(&c->d_mom, (size_t)n_cells * kMomFields * sizeof(double))) ||
      bad(hipHostMalloc(&c->h_scal, 4 * sizeof(double), hipHostMallocMapped)) ||
      bad(hipHostGetDevicePointer((void**)&c->h_scal_dev, c->h_scal, 0))) {
    gcs_surfel_ctx_destroy(c);
    return GCS_ERR_HIP;
  }
  c->stream = c->own;
  size_t tb = 0;
  if (bad(rocprim::radix_sort_pairs(nullptr, tb, c->d_keys, c->d_keys_s, c->d_vals, c->d_vals_s, (unsigned)N, 0u,
                                    c->end_bit, c->stream)) ||
      bad(hipMalloc(&c->d_temp, std::max<size_t>(tb, 16)))) {
    gcs_surfel_ctx_destroy(c);
    return GCS_ERR_HIP;
  }
  c->temp_bytes = std::max<size_t>(tb, 16);
  *out = c;
  return GCS_OK;
}

int gcs_surfel_ctx_set_stream(gcs_surfel_ctx* c, void* stream) {
  if (!c) return GCS_ERR_ARG;
  hipStream_t ns = stream ? (hipStream_t)stream : c->own;
  if (ns == c->stream) return GCS_OK;
  SFCHK(c, hipSetDevice(c->device));
  SFCHK(c, hipStreamSynchronize(c->stream));  // work queued on the old stream completes first
  c->stream = ns;
  return GCS_OK;
}

}  // extern "C"

namespace gcs {
namespace live {
int surfel_bind_stream(gcs_surfel_ctx* c, void* s) {
  if ((hipStream_t)s == c->stream) return GCS_OK;
  SFCHK(c, hipSetDevice(c->device));
  SFCHK(c, hipStreamSynchronize(c->stream));
  c->stream = (hipStream_t)s;
  return GCS_OK;
}

int surfel_launch(gcs_surfel_ctx* c, const double* points, const double* timestamps, const double* weights,
                  int32_t n, gcs_surfel_outputs* o) {
  if (!c || !o) return GCS_ERR_ARG;
  if (n < 0 || n > c->cfg.max_points) return sf_fail(c, GCS_ERR_ARG, "n exceeds max_points");
  if (n > 0 && (!points || !timestamps || !weights)) return sf_fail(c, GCS_ERR_ARG, "null input");
  SFCHK(c, hipSetDevice(c->device));
  const SfParams& a = c->prm;
  hipStream_t s = c->stream;
  const int nblk = std::max(1, std::min(kSfMaxPartials, (n + kSfThreads - 1) / kSfThreads));
  hipLaunchKernelGGL(k_sf_partials, dim3(nblk), dim3(kSfThreads), 0, s, points, weights, n, c->d_partials, c->d_run,
                     2 * a.n_cells);
  hipLaunchKernelGGL(k_sf_keys, dim3(nblk), dim3(kSfThreads), 0, s, points, n, (const double*)c->d_partials, nblk, a,
                     c->d_keys, c->d_vals, c->d_scal, c->h_scal_dev);
  if (n > 0 && c->lds_sort && n <= kSortMax && c->end_bit + kSortIdxBits <= 32) {
    hipLaunchKernelGGL(k_sf_sort_lds<kSortIdxBits>, dim3(1), dim3(kSortThreads), 0, s, (const uint32_t*)c->d_keys, n,
                       a, (int)c->end_bit, c->d_vals_s, c->d_run);
  } else if (n > 0 && c->lds_sort && n <= kSortMaxWide && c->end_bit + kSortIdxBits + 1 <= 32) {
    hipLaunchKernelGGL(k_sf_sort_lds<kSortIdxBits + 1>, dim3(1), dim3(kSortThreads), 0, s, (const uint32_t*)c->d_keys,
                       n, a, (int)c->end_bit, c->d_vals_s, c->d_run);
  } else if (n > 0) {
    size_t tb = c->temp_bytes;
    SFCHK(c, rocprim::radix_sort_pairs(c->d_temp, tb, c->d_keys, c->d_keys_s, c->d_vals, c->d_vals_s, (unsigned)n, 0u,
                                       c->end_bit, s));
    hipLaunchKernelGGL(k_sf_bounds, dim3((n + kSfThreads - 1) / kSfThreads), dim3(kSfThreads), 0, s,
                       (const uint32_t*)c->d_keys_s, n, a.n_cells, c->d_run);
  }
  const int cblk = (a.n_cells + kSfThreads - 1) / kSfThreads;
  if (c->fold_cells) {  // the bucket rows and counts written by k_sf_moments' waves
    hipLaunchKernelGGL(k_sf_moments, dim3((a.n_cells + kCellsPerBlock - 1) / kCellsPerBlock), dim3(kSfThreads), 0, s,
                       points, timestamps, weights, (const double*)c->d_scal, c->d_bucket, c->d_count, a, c->d_mom,
                       (const int32_t*)c->d_run, (const uint32_t*)c->d_vals_s);
  } else {
    const long n_entries = (long)a.n_cells * a.max_occ;
    hipLaunchKernelGGL(k_sf_cells, dim3((unsigned)((n_entries + kSfThreads - 1) / kSfThreads)), dim3(kSfThreads), 0, s,
                       (const int32_t*)c->d_run, (const uint32_t*)c->d_vals_s, a, c->d_bucket, c->d_count);
    hipLaunchKernelGGL(k_sf_moments, dim3((a.n_cells + kCellsPerBlock - 1) / kCellsPerBlock), dim3(kSfThreads), 0, s,
                       points, timestamps, weights, (const double*)c->d_scal, c->d_bucket, c->d_count, a, c->d_mom,
                       (const int32_t*)nullptr, (const uint32_t*)nullptr);
  }
  hipLaunchKernelGGL(k_sf_fit, dim3(cblk), dim3(kSfThreads), 0, s, (const double*)c->d_mom, (const double*)c->d_scal,
                     (const int32_t*)c->d_count, a, c->d_fit, c->d_valid);
  hipLaunchKernelGGL(k_sf_slots, dim3(1), dim3(kSelThreads), 0, s, (const uint8_t*)c->d_valid, a, c->d_slot_cell,
                     (int32_t*)(c->d_scal + 3), (int32_t*)(c->h_scal_dev + 3));
  SelOut so{o->positions, o->covariances, o->normals, o->kappas, o->weights, o->timestamps, o->Lambdas, o->thetas,
            o->etas, o->colors, o->valid_mask, o->source_indices, o->cell_ids, o->sources};
  hipLaunchKernelGGL(k_sf_write, dim3((a.n_surfel + kSfThreads - 1) / kSfThreads), dim3(kSfThreads), 0, s,
                     (const double*)c->d_fit, (const int32_t*)c->d_slot_cell, (const int32_t*)(c->d_scal + 3), a, so);
  SFCHK(c, hipGetLastError());
  if (o->bucket)
    SFCHK(c, hipMemcpyAsync(o->bucket, c->d_bucket, (size_t)a.n_cells * a.max_occ * 4, hipMemcpyDeviceToDevice, s));
  if (o->count) SFCHK(c, hipMemcpyAsync(o->count, c->d_count, (size_t)a.n_cells * 4, hipMemcpyDeviceToDevice, s));
  return GCS_OK;
}

const int32_t* surfel_nvalid_dev(gcs_surfel_ctx* c) { return (const int32_t*)(c->d_scal + 3); }

void surfel_collect(gcs_surfel_ctx* c, gcs_surfel_outputs* o) {
  for (int k = 0; k < 3; ++k) o->center[k] = c->h_scal[k];
  int32_t nv;
  memcpy(&nv, c->h_scal + 3, sizeof(nv));
  o->n_valid = nv;
  o->cert[0] = (double)nv;
  o->cert[1] = (double)nv / (double)std::max(c->cfg.n_surfel, 1);
}
}  // namespace live
}  // namespace gcs

extern "C" {
int gcs_extract_lidar_surfels(gcs_surfel_ctx* c, const double* points, const double* timestamps,
                              const double* weights, int32_t n, gcs_surfel_outputs* o) {
  if (int rc = gcs::live::surfel_launch(c, points, timestamps, weights, n, o)) return rc;
  SFCHK(c, hipStreamSynchronize(c->stream));
  gcs::live::surfel_collect(c, o);
  return GCS_OK;
}
}  // extern "C"
