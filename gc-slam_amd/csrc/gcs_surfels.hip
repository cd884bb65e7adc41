// LiDAR surfel extraction on gfx950 -- the first operator of the live primitive path
// (SURVEY.md 8(f) rank 2): extract_lidar_surfels, FS/backend/operators/lidar_surfel_extraction.py:
// 339-431, with the MA-hex 3D bucketing of FS/common/ma_hex_web.py:221-303 and the LiDAR slice of
// FS/backend/structures/measurement_batch.py:272-381.
//
//   k_sf_partials   weighted centre partial sums (sentinel mask, :259-266), fixed-order block trees
//   k_sf_keys       every block folds the partials in the same order (the centre), then per point
//                   the hash-grid cell of the centred point (masked points -> key n_cells)
//   radix sort      stable (rocPRIM LSD radix sort on the cell key, point index as value): the
//                   reference's stable argsort by (masked, cell) (ma_hex_web.py:276-280)
//   k_sf_cells      per cell: run bounds by binary search, the first max_occupants indices, the
//                   clipped count (:284-303)
//   k_sf_fit        per cell: weighted plane fit, eigh, Wishart-regularised covariance, kappa
//                   (lidar_surfel_extraction.py:84-163)
//   k_sf_select     one workgroup: valid cells in cell-id order into n_surfel slots (:297-321),
//                   the information form of the LiDAR slice (measurement_batch.py:298-331)
// Everything is fixed-order (no floating-point atomics): results are bitwise reproducible.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "gcs_math.h"
#include "gcslam_hip.h"

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
                                                             double* __restrict__ partials) {
  __shared__ double lds[kSfThreads / 64][4];
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
                                                         uint32_t* __restrict__ vals, double* __restrict__ center_out) {
#pragma clang fp contract(off)
  __shared__ double s_c[3];
  if (threadIdx.x == 0) {
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = 0; b < nblk; ++b)
      for (int k = 0; k < 4; ++k) s[k] += partials[4 * b + k];
    const double ws = s[3] + a.eig_min;
    for (int k = 0; k < 3; ++k) s_c[k] = s[k] / ws;
    if (blockIdx.x == 0)
      for (int k = 0; k < 3; ++k) center_out[k] = s_c[k];
  }
  __syncthreads();
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

__device__ __forceinline__ int lower_bound_u32(const uint32_t* __restrict__ a, int n, uint32_t v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// per cell: its run in the sorted keys, the first max_occ point indices, the clipped count
__global__ __launch_bounds__(kSfThreads) void k_sf_cells(const uint32_t* __restrict__ keys_s,
                                                          const uint32_t* __restrict__ vals_s, int n, SfParams a,
                                                          int32_t* __restrict__ bucket, int32_t* __restrict__ count) {
  const int k = blockIdx.x * kSfThreads + threadIdx.x;
  if (k >= a.n_cells) return;
  const int s = lower_bound_u32(keys_s, n, (uint32_t)k);
  const int e = lower_bound_u32(keys_s, n, (uint32_t)k + 1u);
  const int c = min(e - s, a.max_occ);
  count[k] = c;
  int32_t* row = bucket + (size_t)k * a.max_occ;
  for (int r = 0; r < a.max_occ; ++r) row[r] = r < c ? (int32_t)vals_s[s + r] : -1;
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

// _fit_one_cell (lidar_surfel_extraction.py:84-163) on the cell's present slots (absent slots carry
// zero weight in the reference and add exact zeros); fit row = centroid (+ centre) | Sigma_reg |
// normal | kappa | w_surfel | t_surfel
__global__ __launch_bounds__(kSfThreads) void k_sf_fit(const double* __restrict__ p, const double* __restrict__ t,
                                                        const double* __restrict__ w, const double* __restrict__ center,
                                                        const int32_t* __restrict__ bucket,
                                                        const int32_t* __restrict__ count, SfParams a,
                                                        double* __restrict__ fit, uint8_t* __restrict__ valid) {
  const int k = blockIdx.x * kSfThreads + threadIdx.x;
  if (k >= a.n_cells) return;
  const int c = count[k];
  double* out = fit + (size_t)k * kFitFields;
  if (c == 0) {  // never valid (w_surfel = 0): the row is not read
    valid[k] = 0;
    return;
  }
  const int32_t* row = bucket + (size_t)k * a.max_occ;
  const double cx = center[0], cy = center[1], cz = center[2];
  double ws = 0.0, sx = 0.0, sy = 0.0, sz = 0.0, st = 0.0;
  for (int r = 0; r < c; ++r) {
    const int i = row[r];
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    const double we = w[i] * (sf_mask(x, y, z) ? 1.0 : 0.0);
    ws += we;
    sx += (x - cx) * we;
    sy += (y - cy) * we;
    sz += (z - cz) * we;
    st += t[i];
  }
  const double wsum = ws + kFitEps;
  const double m[3] = {sx / wsum, sy / wsum, sz / wsum};
  double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < c; ++r) {
    const int i = row[r];
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    const double we = w[i] * (sf_mask(x, y, z) ? 1.0 : 0.0);
    const double d[3] = {(x - cx) - m[0], (y - cy) - m[1], (z - cz) - m[2]};
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int v = 0; v < 3; ++v) C[3 * u + v] += d[u] * we * d[v];
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) C[q] /= wsum;
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
  double v1 = 0.0, v2 = 0.0;
  for (int r = 0; r < c; ++r) {
    const int i = row[r];
    const double x = p[3 * (size_t)i], y = p[3 * (size_t)i + 1], z = p[3 * (size_t)i + 2];
    const double we = w[i] * (sf_mask(x, y, z) ? 1.0 : 0.0);
    const double d[3] = {(x - cx) - m[0], (y - cy) - m[1], (z - cz) - m[2]};
    const double q1 = d[0] * e1[0] + d[1] * e1[1] + d[2] * e1[2];
    const double q2 = d[0] * e2[0] + d[1] * e2[1] + d[2] * e2[2];
    v1 += we * (q1 * q1);
    v2 += we * (q2 * q2);
  }
  const double var_e1 = v1 / wsum + a.sensor_var, var_e2 = v2 / wsum + a.sensor_var;
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
  out[0] = m[0] + cx;
  out[1] = m[1] + cy;
  out[2] = m[2] + cz;
#pragma unroll
  for (int q = 0; q < 9; ++q) out[3 + q] = Sr[q];
  out[12] = nrm[0]; out[13] = nrm[1]; out[14] = nrm[2];
  out[15] = kap;
  out[16] = ws;
  out[17] = st / wsum;
  valid[k] = (c >= a.min_points && ws > 0.0) ? 1 : 0;
}

struct SelOut {
  double *positions, *covariances, *normals, *kappas, *weights, *timestamps;
  double *Lambdas, *thetas, *etas, *colors;
  uint8_t* valid_mask;
  int32_t *source_indices, *cell_ids;
  int32_t* n_valid;  // device scalar
};

// one workgroup: valid cells (cell-id order) -> slots, then the padded tail
__global__ __launch_bounds__(kSelThreads) void k_sf_select(const double* __restrict__ fit,
                                                            const uint8_t* __restrict__ valid, SfParams a, SelOut o) {
  __shared__ int s_wsum[kSelThreads / 64];
  __shared__ int s_total;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int per = (a.n_cells + kSelThreads - 1) / kSelThreads;
  const int k0 = min(a.n_cells, t * per), k1 = min(a.n_cells, k0 + per);
  int mine = 0;
  for (int k = k0; k < k1; ++k) mine += valid[k];
  int x = mine;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  int run = x - mine;
  for (int q = 0; q < wid; ++q) run += s_wsum[q];
  if (t == kSelThreads - 1) s_total = run + mine;
  for (int k = k0; k < k1; ++k) {
    if (!valid[k]) continue;
    const int s = run++;
    if (s >= a.n_surfel) break;
    const double* f = fit + (size_t)k * kFitFields;
    const double* pos = f;
    const double* S = f + 3;
    const double* nrm = f + 12;
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
  }
  __syncthreads();
  const int nv = min(s_total, a.n_surfel);
  if (t == 0) *o.n_valid = nv;
  for (int s = nv + t; s < a.n_surfel; s += kSelThreads) {  // the reference's padding
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
  int32_t *d_bucket = nullptr, *d_count = nullptr;
  double* d_fit = nullptr;
  uint8_t* d_valid = nullptr;
  double* d_scal = nullptr;   // center[3], n_valid (as int32 in the 4th slot)
  double* h_scal = nullptr;   // pinned
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
                  c->d_bucket, c->d_count, c->d_fit, c->d_valid, c->d_scal};
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
  auto bad = [&](hipError_t e) { return e != hipSuccess; };
  const size_t N = (size_t)cfg->max_points;
  if (bad(hipSetDevice(cfg->device)) || bad(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) ||
      bad(hipMalloc(&c->d_partials, kSfMaxPartials * 4 * sizeof(double))) ||
      bad(hipMalloc(&c->d_keys, N * 4)) || bad(hipMalloc(&c->d_vals, N * 4)) ||
      bad(hipMalloc(&c->d_keys_s, N * 4)) || bad(hipMalloc(&c->d_vals_s, N * 4)) ||
      bad(hipMalloc(&c->d_bucket, (size_t)n_cells * a.max_occ * 4)) || bad(hipMalloc(&c->d_count, n_cells * 4)) ||
      bad(hipMalloc(&c->d_fit, (size_t)n_cells * kFitFields * sizeof(double))) ||
      bad(hipMalloc(&c->d_valid, n_cells)) || bad(hipMalloc(&c->d_scal, 4 * sizeof(double))) ||
      bad(hipHostMalloc(&c->h_scal, 4 * sizeof(double), hipHostMallocDefault))) {
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
  SFCHK(c, hipSetDevice(c->device));
  SFCHK(c, hipStreamSynchronize(c->stream));  // work queued on the old stream completes first
  c->stream = stream ? (hipStream_t)stream : c->own;
  return GCS_OK;
}

int gcs_extract_lidar_surfels(gcs_surfel_ctx* c, const double* points, const double* timestamps,
                              const double* weights, int32_t n, gcs_surfel_outputs* o) {
  if (!c || !o) return GCS_ERR_ARG;
  if (n < 0 || n > c->cfg.max_points) return sf_fail(c, GCS_ERR_ARG, "n exceeds max_points");
  if (n > 0 && (!points || !timestamps || !weights)) return sf_fail(c, GCS_ERR_ARG, "null input");
  SFCHK(c, hipSetDevice(c->device));
  const SfParams& a = c->prm;
  hipStream_t s = c->stream;
  const int nblk = std::max(1, std::min(kSfMaxPartials, (n + kSfThreads - 1) / kSfThreads));
  hipLaunchKernelGGL(k_sf_partials, dim3(nblk), dim3(kSfThreads), 0, s, points, weights, n, c->d_partials);
  hipLaunchKernelGGL(k_sf_keys, dim3(nblk), dim3(kSfThreads), 0, s, points, n, (const double*)c->d_partials, nblk, a,
                     c->d_keys, c->d_vals, c->d_scal);
  if (n > 0) {
    size_t tb = c->temp_bytes;
    SFCHK(c, rocprim::radix_sort_pairs(c->d_temp, tb, c->d_keys, c->d_keys_s, c->d_vals, c->d_vals_s, (unsigned)n, 0u,
                                       c->end_bit, s));
  }
  const int cblk = (a.n_cells + kSfThreads - 1) / kSfThreads;
  hipLaunchKernelGGL(k_sf_cells, dim3(cblk), dim3(kSfThreads), 0, s, (const uint32_t*)c->d_keys_s,
                     (const uint32_t*)c->d_vals_s, n, a, c->d_bucket, c->d_count);
  hipLaunchKernelGGL(k_sf_fit, dim3(cblk), dim3(kSfThreads), 0, s, points, timestamps, weights,
                     (const double*)c->d_scal, (const int32_t*)c->d_bucket, (const int32_t*)c->d_count, a, c->d_fit,
                     c->d_valid);
  SelOut so{o->positions, o->covariances, o->normals, o->kappas, o->weights, o->timestamps, o->Lambdas, o->thetas,
            o->etas, o->colors, o->valid_mask, o->source_indices, o->cell_ids, (int32_t*)(c->d_scal + 3)};
  hipLaunchKernelGGL(k_sf_select, dim3(1), dim3(kSelThreads), 0, s, (const double*)c->d_fit,
                     (const uint8_t*)c->d_valid, a, so);
  SFCHK(c, hipGetLastError());
  if (o->bucket)
    SFCHK(c, hipMemcpyAsync(o->bucket, c->d_bucket, (size_t)a.n_cells * a.max_occ * 4, hipMemcpyDeviceToDevice, s));
  if (o->count) SFCHK(c, hipMemcpyAsync(o->count, c->d_count, (size_t)a.n_cells * 4, hipMemcpyDeviceToDevice, s));
  SFCHK(c, hipMemcpyAsync(c->h_scal, c->d_scal, 4 * sizeof(double), hipMemcpyDeviceToHost, s));
  SFCHK(c, hipStreamSynchronize(s));
  for (int k = 0; k < 3; ++k) o->center[k] = c->h_scal[k];
  int32_t nv;
  memcpy(&nv, c->h_scal + 3, sizeof(nv));
  o->n_valid = nv;
  o->cert[0] = (double)nv;
  o->cert[1] = (double)nv / (double)std::max(c->cfg.n_surfel, 1);
  return GCS_OK;
}

}  // extern "C"
