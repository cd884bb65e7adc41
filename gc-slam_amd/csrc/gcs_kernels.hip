// HIP kernels for the GC-SLAM bin-path hot path on gfx950 (MI355X).
//
//   k_budget_*      PointBudgetResample mass sums   point_budget.py:50-109
//   k_points        budget gather + DeskewConstantTwist + ray direction + nearest bin +
//                   K-candidate softmax normaliser (BinSoftAssign, scale mode) or dense
//                   softmax normaliser, and the per-point certificate partials
//                   deskew_constant_twist.py:31-69, pipeline.py:589-593, binning.py:56-76
//   k_scan_*, k_place, k_bucket_*   deterministic bucketing of points by nearest bin
//   k_bins_scale    bin-centric gather: ScanBinMomentMatch + Kappa, finalize + write
//                   binning.py:139-209, kappa.py:130-169
//   k_dense_*       the reference's dense N x B form (legacy B=48)
//   k_mf_*          MatrixFisherRotation bin reduction + device 3x3 SVD
//                   matrix_fisher_evidence.py:155-256
//   k_pt_*          PlanarTranslationEvidence bin reduction   matrix_fisher_evidence.py:413-499
//   k_pushforward   PoseCovInflationPushforward + forgetting + derived map stats
//                   (declared; bin_atlas.py:137-257)
//
// All reductions are fixed-shape (fixed grid, fixed lane/LDS trees, fixed-order final pass),
// so results are bitwise reproducible run to run (docs/GC_SLAM.md:1150).  No float atomics.
#include <hip/hip_runtime.h>


#include "gcs_kernels.h"
#include "gcs_layout.h"
#include "gcs_math.h"

namespace gcs {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// ---------------------------------------------------------------- reductions
template <int NV>
__device__ __forceinline__ void wave_sum(double (&v)[NV]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], off, 64);
  }
}

// Block sum of NV doubles; result valid in thread 0.  lds must hold kWaves*NV doubles.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* lds) {
  wave_sum<NV>(v);
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[wid * NV + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = lds[k];
      for (int w = 1; w < kWaves; ++w) s += lds[w * NV + k];
      v[k] = s;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double block_max(double v, double* lds) {
  v = wave_max(v);
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = lds[0];
    for (int w = 1; w < kWaves; ++w) m = fmax(m, lds[w]);
    v = m;
  }
  __syncthreads();
  return v;
}

// Final pass over per-block partials: one block, thread t sums partials t, t+256, ... in order,
// then a fixed tree.  Bit k of MAXMASK selects max instead of sum for component k.
template <int NV, unsigned MAXMASK>
__global__ __launch_bounds__(kBlock) void k_partials_final(const double* __restrict__ partials, int nblocks,
                                                           double* out, int out_off) {
  __shared__ double lds[kWaves * NV];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = ((MAXMASK >> k) & 1u) ? -INFINITY : 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double x = partials[(size_t)b * NV + k];
      v[k] = ((MAXMASK >> k) & 1u) ? fmax(v[k], x) : v[k] + x;
    }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if ((MAXMASK >> k) & 1u) {
      v[k] = wave_max(v[k]);
    } else {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    }
  }
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[wid * NV + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < NV; ++k) {
      double s = lds[k];
      for (int w = 1; w < kWaves; ++w) s = ((MAXMASK >> k) & 1u) ? fmax(s, lds[w * NV + k]) : s + lds[w * NV + k];
      out[out_off + k] = s;
    }
  }
}

// ---------------------------------------------------------------- row 1: budget mass sums
__global__ __launch_bounds__(kBlock) void k_budget_partial(const double* __restrict__ w, int n_raw, int stride,
                                                           double* partials) {
  __shared__ double lds[kWaves * 2];
  double v[2] = {0.0, 0.0};
  for (int j = blockIdx.x * kBlock + threadIdx.x; j < n_raw; j += gridDim.x * kBlock) {
    double x = w[j];
    v[0] += x;
    if (j % stride == 0) v[1] += x;
  }
  block_sum<2>(v, lds);
  if (threadIdx.x == 0) {
    partials[blockIdx.x * 2] = v[0];
    partials[blockIdx.x * 2 + 1] = v[1];
  }
}

__global__ __launch_bounds__(kBlock) void k_budget_final(const double* __restrict__ partials, int nblocks,
                                                         double* scalars) {
  __shared__ double lds[kWaves * 2];
  double v[2] = {0.0, 0.0};
  for (int b = threadIdx.x; b < nblocks; b += kBlock) { v[0] += partials[2 * b]; v[1] += partials[2 * b + 1]; }
  block_sum<2>(v, lds);
  if (threadIdx.x == 0) {
    scalars[SC_MASS_IN] = v[0];
    scalars[SC_MASS_SEL] = v[1];
    // mass_scale = total_mass_in / (total_mass_selected + eps_mass)   point_budget.py:80-84
    scalars[SC_MASS_SCALE] = v[0] / (v[1] + kEpsMass);
  }
}

// ---------------------------------------------------------------- cube-map cell of a direction
__device__ __forceinline__ int cube_cell(double dx, double dy, double dz, int G) {
  double ax = fabs(dx), ay = fabs(dy), az = fabs(dz);
  int face;
  double m, u, v;
  if (ax >= ay && ax >= az) { face = dx >= 0.0 ? 0 : 1; m = ax; u = dy; v = dz; }
  else if (ay >= az) { face = dy >= 0.0 ? 2 : 3; m = ay; u = dx; v = dz; }
  else { face = dz >= 0.0 ? 4 : 5; m = az; u = dx; v = dy; }
  if (!(m > 0.0)) return 0;
  double fu = (u / m + 1.0) * 0.5 * (double)G;
  double fv = (v / m + 1.0) * 0.5 * (double)G;
  int iu = (int)floor(fu), iv = (int)floor(fv);
  iu = iu < 0 ? 0 : (iu >= G ? G - 1 : iu);
  iv = iv < 0 ? 0 : (iv >= G ? G - 1 : iv);
  return (face * G + iu) * G + iv;
}

__device__ __forceinline__ void ray_dir(double px, double py, double pz, const double* o, double* d) {
  double rx = px - o[0], ry = py - o[1], rz = pz - o[2];
  double nrm = sqrt(dot3_exact(rx, ry, rz, rx, ry, rz));
  double den = nrm + kEpsMass;
  d[0] = rx / den; d[1] = ry / den; d[2] = rz / den;
}

// ---------------------------------------------------------------- row 1+3+5: the point kernel
// One thread per budget output slot i in [0, cap).  SCALE = candidate-restricted softmax.
template <bool SCALE, int KC>
__global__ __launch_bounds__(kBlock) void k_points(PointKernelArgs a, double* partials) {
  __shared__ double lds[kWaves * 5];
  const double mass_scale = a.scalars[SC_MASS_SCALE];
  const double mass_in = a.scalars[SC_MASS_IN];
  const double denom = a.t1 - a.t0 > 1e-12 ? a.t1 - a.t0 : 1e-12;
  const double inv_tau = 1.0 / a.tau;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sum w_budget, sum wn^2, sum w_out, sum H
  double rmax = -INFINITY;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < a.cap; i += gridDim.x * kBlock) {
    double p[3] = {0.0, 0.0, 0.0}, t = 0.0, wb = 0.0;
    bool valid = i < a.n_sel;
    if (valid) {
      size_t src = (size_t)i * (size_t)a.stride;
      const float* rec = (const float*)(a.xyz + src * (size_t)a.point_step);
      p[0] = (double)rec[0]; p[1] = (double)rec[1]; p[2] = (double)rec[2];
      t = a.timestamps[src];
      wb = a.weights[src] * mass_scale;
    }
    double alpha = (t - a.t0) / denom;
    double p0[3];
    deskew_point(alpha, a.xi, p, p0);
    double wout = wb * smooth_window(t, a.t0, a.t1, kTimeWarpSigmaFrac * denom);
    double d[3];
    ray_dir(p0[0], p0[1], p0[2], a.origin, d);
    double m = -INFINITY, Z = 0.0, H = 0.0, rm = 0.0;
    int nearest = 0;
    if (SCALE) {
      // exact nearest atlas bin: pool of the direction's cube cell, ascending ids, strict '>'
      bool zero = (d[0] == 0.0 && d[1] == 0.0 && d[2] == 0.0);
      if (!zero) {
        const int4* pool = (const int4*)(a.pools + (size_t)cube_cell(d[0], d[1], d[2], a.grid) * a.pool_width);
        double best = -INFINITY;
        for (int q = 0; q < (a.pool_width >> 2); ++q) {
          int4 id4 = pool[q];
          int ids[4] = {id4.x, id4.y, id4.z, id4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (ids[u] >= 0) {
              const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)ids[u]);
              double s = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
              if (s > best) { best = s; nearest = ids[u]; }
            }
          }
          if (id4.w < 0) break;
        }
      }
      const int* cand = a.knn + (size_t)nearest * KC;
      double sims[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)cand[k]);
        sims[k] = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
        m = fmax(m, sims[k]);
      }
#pragma unroll
      for (int k = 0; k < KC; ++k) Z += exp((sims[k] - m) * inv_tau);
      double iz = 1.0 / Z;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        double r = exp((sims[k] - m) * inv_tau) * iz;
        H -= r * log(r + kEpsMass);
        rm = fmax(rm, r);
      }
      uint32_t key = (uint32_t)a.n_bins;
      if (valid) {
        // bucket slot: arrival order only (reordered by point index in k_bucket_order)
        uint32_t slot = atomicAdd(a.counts + nearest, 1u);
        a.slots[i] = slot;
        key = (uint32_t)nearest;
        if (slot == 0) {  // first arrival marks the bucket's candidate bins active
#pragma unroll
          for (int k = 0; k < KC; ++k) a.flags[cand[k]] = 1;
        }
      }
      a.keys[i] = key;
      Z = iz;
    } else {
      for (int b = 0; b < a.n_bins; ++b) {
        const double* bd = a.bin_dirs + 4 * (size_t)b;
        m = fmax(m, dot3_exact(d[0], d[1], d[2], bd[0], bd[1], bd[2]));
      }
      for (int b = 0; b < a.n_bins; ++b) {
        const double* bd = a.bin_dirs + 4 * (size_t)b;
        Z += exp((dot3_exact(d[0], d[1], d[2], bd[0], bd[1], bd[2]) - m) * inv_tau);
      }
      double iz = 1.0 / Z;
      for (int b = 0; b < a.n_bins; ++b) {
        const double* bd = a.bin_dirs + 4 * (size_t)b;
        double r = exp((dot3_exact(d[0], d[1], d[2], bd[0], bd[1], bd[2]) - m) * inv_tau) * iz;
        H -= r * log(r + kEpsMass);
        rm = fmax(rm, r);
      }
      Z = iz;
    }
    PointRec pr;
    pr.x = p0[0]; pr.y = p0[1]; pr.z = p0[2];
    pr.dx = d[0]; pr.dy = d[1]; pr.dz = d[2];
    pr.w = wout; pr.m = m; pr.iz = Z; pr.pad = 0.0;
    a.recs[i] = pr;
    if (a.p0_out) { a.p0_out[3 * (size_t)i] = p0[0]; a.p0_out[3 * (size_t)i + 1] = p0[1]; a.p0_out[3 * (size_t)i + 2] = p0[2]; }
    if (a.w_out) a.w_out[i] = wout;
    if (a.w_budget_out) a.w_budget_out[i] = wb;
    if (a.nearest_out) a.nearest_out[i] = nearest;
    double wn = wb / (mass_in + kEpsMass);
    acc[0] += wb;
    acc[1] += wn * wn;
    acc[2] += wout;
    acc[3] += H;
    rmax = fmax(rmax, rm);
  }
  block_sum<4>(acc, lds);
  rmax = block_max(rmax, lds);
  if (threadIdx.x == 0) {
    double* pp = partials + blockIdx.x * 5;
    pp[0] = acc[0]; pp[1] = acc[1]; pp[2] = acc[2]; pp[3] = acc[3]; pp[4] = rmax;
  }
}

// ---------------------------------------------------------------- deterministic bucketing by nearest bin
// counts[] were filled by atomic slots in k_points.  start[] = exclusive scan of counts in two
// passes over 4096-bucket tiles; points are placed at start+slot, then every bucket is reordered
// by ascending point index (insertion sort up to 64 entries, an in-order compaction over all
// keys for larger buckets), so the bin gather sees a scheduling-independent order.
constexpr int kScanTile = 4096;
__global__ __launch_bounds__(kBlock) void k_scan_tiles(const uint32_t* __restrict__ counts, int n, uint32_t* tile_sums) {
  __shared__ uint32_t ws[kWaves];
  int base = blockIdx.x * kScanTile;
  uint32_t s = 0;
  for (int i = base + threadIdx.x; i < min(base + kScanTile, n); i += kBlock) s += counts[i];
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(kBlock) void k_scan_apply(const uint32_t* __restrict__ counts, int n,
                                                       const uint32_t* __restrict__ tile_sums, uint32_t* start) {
  __shared__ uint32_t wsum[kWaves];
  __shared__ uint32_t carry;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) {
    uint32_t c = 0;
    for (int b = 0; b < (int)blockIdx.x; ++b) c += tile_sums[b];
    carry = c;
  }
  __syncthreads();
  int base = blockIdx.x * kScanTile;
  for (int c0 = base; c0 < min(base + kScanTile, n); c0 += kBlock) {
    int i = c0 + t;
    uint32_t v = i < n ? counts[i] : 0u;
    uint32_t x = v;  // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t pre = carry;
    for (int w = 0; w < wid; ++w) pre += wsum[w];
    if (i < n) start[i] = pre + x - v;
    __syncthreads();
    if (t == kBlock - 1) carry = pre + x;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_place(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ slots,
                                                  const uint32_t* __restrict__ start, int n, int n_bins,
                                                  uint32_t* sorted) {
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    uint32_t key = keys[i];
    if (key < (uint32_t)n_bins) sorted[start[key] + slots[i]] = (uint32_t)i;
  }
}

constexpr int kSmallBucket = 64;
__global__ __launch_bounds__(kBlock) void k_bucket_order(const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ start, int n_bins,
                                                         uint32_t* sorted, uint32_t* big_list, uint32_t* big_n) {
  for (int a = blockIdx.x * kBlock + threadIdx.x; a < n_bins; a += gridDim.x * kBlock) {
    uint32_t c = counts[a];
    if (c < 2) continue;
    if (c > (uint32_t)kSmallBucket) {
      big_list[atomicAdd(big_n, 1u)] = (uint32_t)a;
      continue;
    }
    uint32_t* v = sorted + start[a];
    for (uint32_t j = 1; j < c; ++j) {
      uint32_t x = v[j];
      int q = (int)j - 1;
      while (q >= 0 && v[q] > x) { v[q + 1] = v[q]; --q; }
      v[q + 1] = x;
    }
  }
}

// big buckets: one block rebuilds the bucket by an in-order compaction over all keys
__global__ __launch_bounds__(kBlock) void k_bucket_big(const uint32_t* __restrict__ keys, int n,
                                                       const uint32_t* __restrict__ start,
                                                       const uint32_t* __restrict__ big_list,
                                                       const uint32_t* __restrict__ big_n, uint32_t* sorted) {
  __shared__ uint32_t wcnt[kWaves];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint32_t nb = *big_n;
  for (uint32_t j = blockIdx.x; j < nb; j += gridDim.x) {
    uint32_t a = big_list[j];
    uint32_t pos = start[a];
    for (int c0 = 0; c0 < n; c0 += kBlock) {
      int i = c0 + t;
      bool hit = i < n && keys[i] == a;
      unsigned long long m = __ballot(hit);
      if (lane == 0) wcnt[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t pre = pos;
      for (int w = 0; w < wid; ++w) pre += wcnt[w];
      if (hit) sorted[pre + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
      pos += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- bin finalize (shared)
// Raw sums layout (19): N, sd[3], S[xx,xy,xz,yy,yz,zz], sp[3], spp[xx,xy,xz,yy,yz,zz]
__device__ __forceinline__ void finalize_bin(const double* r, double* __restrict__ scan, int B, int b,
                                             double* cert /*5*/) {
  double N = r[0];
  double den = N + kEpsMass + kF64Eps;          // inv_mass_core, primitives.py:195-212
  double invN = 1.0 / den;
  double epsr = kEpsMass / den;
  double pb[3] = {r[10] * invN, r[11] * invN, r[12] * invN};
  const double* q = r + 13;
  double sc[9];
  sc[0] = q[0] * invN - pb[0] * pb[0];
  sc[1] = q[1] * invN - pb[0] * pb[1];
  sc[2] = q[2] * invN - pb[0] * pb[2];
  sc[3] = q[1] * invN - pb[1] * pb[0];
  sc[4] = q[3] * invN - pb[1] * pb[1];
  sc[5] = q[4] * invN - pb[1] * pb[2];
  sc[6] = q[2] * invN - pb[2] * pb[0];
  sc[7] = q[4] * invN - pb[2] * pb[1];
  sc[8] = q[5] * invN - pb[2] * pb[2];
  double sig[9];
  double delta = psd_project3(sc, sig);
  double sn = sqrt(dot3_exact(r[1], r[2], r[3], r[1], r[2], r[3]));
  double kap = kappa_from_rbar(sn * invN);
  size_t Bs = (size_t)B;
  scan[SF_N * Bs + b] = N;
  scan[(SF_SD + 0) * Bs + b] = r[1];
  scan[(SF_SD + 1) * Bs + b] = r[2];
  scan[(SF_SD + 2) * Bs + b] = r[3];
  const double* s6 = r + 4;
  double S9[9] = {s6[0], s6[1], s6[2], s6[1], s6[3], s6[4], s6[2], s6[4], s6[5]};
#pragma unroll
  for (int k = 0; k < 9; ++k) scan[(SF_S + k) * Bs + b] = S9[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) scan[(SF_PB + k) * Bs + b] = pb[k];
#pragma unroll
  for (int k = 0; k < 9; ++k) scan[(SF_SIG + k) * Bs + b] = sig[k];
  scan[SF_KAPPA * Bs + b] = kap;
  cert[0] += N;
  cert[1] += N * N;
  cert[2] += N / (N + kEpsMass);
  cert[3] += delta;
  cert[4] = fmax(cert[4], epsr);
}

__device__ __forceinline__ void add_contrib(double* acc, double wr, const double* d, const double* p) {
  acc[0] += wr;
  double wd0 = wr * d[0], wd1 = wr * d[1], wd2 = wr * d[2];
  acc[1] += wd0; acc[2] += wd1; acc[3] += wd2;
  acc[4] += wd0 * d[0]; acc[5] += wd0 * d[1]; acc[6] += wd0 * d[2];
  acc[7] += wd1 * d[1]; acc[8] += wd1 * d[2]; acc[9] += wd2 * d[2];
  double wp0 = wr * p[0], wp1 = wr * p[1], wp2 = wr * p[2];
  acc[10] += wp0; acc[11] += wp1; acc[12] += wp2;
  acc[13] += wp0 * p[0]; acc[14] += wp0 * p[1]; acc[15] += wp0 * p[2];
  acc[16] += wp1 * p[1]; acc[17] += wp1 * p[2]; acc[18] += wp2 * p[2];
}

__device__ __forceinline__ void write_bin_cert(double* cert, double* lds, double* partials) {
  double v[4] = {cert[0], cert[1], cert[2], cert[3]};
  block_sum<4>(v, lds);
  double mx = block_max(cert[4], lds);
  if (threadIdx.x == 0) {
    double* pp = partials + blockIdx.x * 5;
    pp[0] = v[0]; pp[1] = v[1]; pp[2] = v[2]; pp[3] = v[3]; pp[4] = mx;
  }
}

// ---------------------------------------------------------------- row 5+6 scale mode: bin-centric
// One 256-thread workgroup per tile of 64 consecutive bins.  Phase 1 compacts the tile's active
// bins (ballot, wave order).  Phase 2: a 16-lane group per active bin; lane l owns the bin's
// reverse-kNN buckets l, l+16, ... (fixed order) and walks each bucket's points in ascending
// point index (stable sort), so each lane's dependent chain is one bucket deep and the 16
// buckets are fetched concurrently; the 16 lane sums meet in a fixed xor tree.  Phase 3: the
// first wave finalizes the 64 bins (PSD, kappa) and streams the 26 field-major outputs.
constexpr int kTile = 64;
constexpr int kGroup = 16;
__global__ __launch_bounds__(kBlock) void k_bins_scale(BinKernelArgs a, double* partials) {
  __shared__ double sums[19 * kTile];
  __shared__ int active[kTile];
  __shared__ int n_active;
  __shared__ double lds[kWaves * 4];
  const int t = threadIdx.x;
  const int b0 = blockIdx.x * kTile;
  for (int i = t; i < 19 * kTile; i += kBlock) sums[i] = 0.0;
  if (t < 64) {
    int b = b0 + t;
    bool act = (b < a.n_bins) && a.flags[b];
    unsigned long long mask = __ballot(act);
    if (act) active[__popcll(mask & ((1ull << t) - 1ull))] = t;
    if (t == 0) n_active = __popcll(mask);
  }
  __syncthreads();
  const int g = t / kGroup, l = t % kGroup;
  const double inv_tau = 1.0 / a.tau;
  for (int j = g; j < n_active; j += kBlock / kGroup) {
    int lb = active[j];
    int bb = b0 + lb;
    const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)bb);
    double acc[19];
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = 0.0;
    const int q0 = a.rknn_off[bb], q1 = a.rknn_off[bb + 1];
    // reverse-kNN buckets in chunks of 16 (one per lane); contributions flattened over the
    // group in (bucket order, ascending point index) and dealt to lanes round-robin
    for (int qc = q0; qc < q1; qc += kGroup) {
      int q = qc + l;
      uint32_t st = 0, ct = 0;
      if (q < q1) {
        int src = a.rknn[q];
        st = a.starts[src];
        ct = a.counts[src];
      }
      uint32_t x = ct;  // inclusive scan over the 16 lanes of the group
#pragma unroll
      for (int off = 1; off < kGroup; off <<= 1) {
        uint32_t y = __shfl_up(x, off, kGroup);
        if (l >= off) x += y;
      }
      const uint32_t pre = x - ct;
      const uint32_t tot = __shfl(x, kGroup - 1, kGroup);
      for (uint32_t r0 = 0; r0 < tot; r0 += kGroup) {
        uint32_t jj = r0 + (uint32_t)l;
        // source lane = last lane whose exclusive prefix <= jj (binary search over the group)
        int s = 0;
#pragma unroll
        for (int step = kGroup / 2; step >= 1; step >>= 1) {
          uint32_t ps = __shfl(pre, s + step, kGroup);
          if (ps <= jj && s + step < kGroup) s += step;
        }
        uint32_t s_st = __shfl(st, s, kGroup);
        uint32_t s_pre = __shfl(pre, s, kGroup);
        if (jj < tot) {
          const PointRec pr = a.recs[a.sorted_vals[s_st + (jj - s_pre)]];
          double d[3] = {pr.dx, pr.dy, pr.dz};
          double p[3] = {pr.x, pr.y, pr.z};
          double sim = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
          double r = exp((sim - pr.m) * inv_tau) * pr.iz;
          add_contrib(acc, pr.w * r, d, p);
        }
      }
    }
#pragma unroll
    for (int off = kGroup / 2; off >= 1; off >>= 1)
#pragma unroll
      for (int f = 0; f < 19; ++f) acc[f] += __shfl_xor(acc[f], off, 64);
    if (l == 0)
#pragma unroll
      for (int f = 0; f < 19; ++f) sums[f * kTile + lb] = acc[f];
  }
  __syncthreads();
  double cert[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
  if (t < kTile && b0 + t < a.n_bins) {
    double r[19];
#pragma unroll
    for (int f = 0; f < 19; ++f) r[f] = sums[f * kTile + t];
    finalize_bin(r, a.scan, a.n_bins, b0 + t, cert);
  }
  write_bin_cert(cert, lds, partials);
}

// ---------------------------------------------------------------- row 5+6 dense mode (B small)
// Block = chunk of 256 points staged in LDS; each thread owns bins t, t+256, ... and
// accumulates the chunk in point order.  Partials[f][block][bin] are reduced in block order.
__global__ __launch_bounds__(kBlock) void k_dense_accum(BinKernelArgs a, double* bin_partials) {
  __shared__ PointRec pts[kBlock];
  __shared__ double dirs[kBlock * 3];
  const int t = threadIdx.x;
  const int i = blockIdx.x * kBlock + t;
  if (i < a.cap) {
    PointRec pr = a.recs[i];
    pts[t] = pr;
    dirs[3 * t] = pr.dx; dirs[3 * t + 1] = pr.dy; dirs[3 * t + 2] = pr.dz;
  }
  __syncthreads();
  int np = a.cap - blockIdx.x * kBlock;
  np = np > kBlock ? kBlock : np;
  const double inv_tau = 1.0 / a.tau;
  for (int b = t; b < a.n_bins; b += kBlock) {
    const double* bd = a.bin_dirs + 4 * (size_t)b;
    double acc[19];
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = 0.0;
    for (int j = 0; j < np; ++j) {
      const double* d = dirs + 3 * j;
      double s = dot3_exact(d[0], d[1], d[2], bd[0], bd[1], bd[2]);
      double r = exp((s - pts[j].m) * inv_tau) * pts[j].iz;
      double p[3] = {pts[j].x, pts[j].y, pts[j].z};
      add_contrib(acc, pts[j].w * r, d, p);
    }
    size_t nb = gridDim.x;
#pragma unroll
    for (int f = 0; f < 19; ++f) bin_partials[((size_t)f * nb + blockIdx.x) * a.n_bins + b] = acc[f];
  }
}

__global__ __launch_bounds__(kBlock) void k_dense_finalize(BinKernelArgs a, const double* __restrict__ bin_partials,
                                                           int nchunks, double* partials) {
  __shared__ double lds[kWaves * 4];
  int b = blockIdx.x * kBlock + threadIdx.x;
  double cert[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
  if (b < a.n_bins) {
    double r[19];
    for (int f = 0; f < 19; ++f) {
      double s = 0.0;
      for (int c = 0; c < nchunks; ++c) s += bin_partials[((size_t)f * nchunks + c) * a.n_bins + b];
      r[f] = s;
    }
    finalize_bin(r, a.scan, a.n_bins, b, cert);
  }
  write_bin_cert(cert, lds, partials);
}

// ---------------------------------------------------------------- row 7: Matrix-Fisher reduction
// Per bin (matrix_fisher_evidence.py:181-211): w_b = sqrt(N_s N_m + eps), u = S/(|S|+eps),
// conf = Rbar_s Rbar_m, H += w_b conf u_map u_scan^T.  Also sum map S_dir_scatter / N_dir
// (z precision in planar evidence, :572-587) and sum scan N.
constexpr int kMfNV = 22;
__global__ __launch_bounds__(kBlock) void k_mf_partial(const double* __restrict__ scan, const double* __restrict__ map,
                                                       int B, double* partials) {
  __shared__ double lds[kWaves * kMfNV];
  double v[kMfNV];
#pragma unroll
  for (int k = 0; k < kMfNV; ++k) v[k] = 0.0;
  size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    double Ns = scan[SF_N * Bs + b];
    double sx = scan[(SF_SD) * Bs + b], sy = scan[(SF_SD + 1) * Bs + b], sz = scan[(SF_SD + 2) * Bs + b];
    double Nm = map[MF_ND * Bs + b];
    double mx = map[(MF_SD) * Bs + b], my = map[(MF_SD + 1) * Bs + b], mz = map[(MF_SD + 2) * Bs + b];
    double wb = sqrt(Ns * Nm + kEpsMass);
    double sn = sqrt(dot3_exact(sx, sy, sz, sx, sy, sz));
    double mn = sqrt(dot3_exact(mx, my, mz, mx, my, mz));
    double us[3] = {sx / (sn + kEpsMass), sy / (sn + kEpsMass), sz / (sn + kEpsMass)};
    double um[3] = {mx / (mn + kEpsMass), my / (mn + kEpsMass), mz / (mn + kEpsMass)};
    double conf = (sn * (1.0 / (Ns + kEpsMass))) * (mn * (1.0 / (Nm + kEpsMass)));
    double wf = wb * conf;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) v[3 * i + j] += wf * um[i] * us[j];
    v[9] += wf;
#pragma unroll
    for (int k = 0; k < 9; ++k) v[10 + k] += map[(MF_S + k) * Bs + b];
    v[19] += Nm;
    v[20] += Ns;
  }
  block_sum<kMfNV>(v, lds);
  if (threadIdx.x == 0)
    for (int k = 0; k < kMfNV; ++k) partials[(size_t)blockIdx.x * kMfNV + k] = v[k];
}

// final MF: reduce partials (fixed order) then 3x3 SVD and the det-fixed R_mf on one thread.
__global__ __launch_bounds__(kBlock) void k_mf_final(const double* __restrict__ partials, int nblocks, double* scalars) {
  __shared__ double lds[kWaves * kMfNV];
  double v[kMfNV];
#pragma unroll
  for (int k = 0; k < kMfNV; ++k) v[k] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock)
#pragma unroll
    for (int k = 0; k < kMfNV; ++k) v[k] += partials[(size_t)b * kMfNV + k];
  block_sum<kMfNV>(v, lds);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 9; ++k) scalars[SC_MF_H + k] = v[k];
    scalars[SC_MF_NEFF] = v[9];
    for (int k = 0; k < 9; ++k) scalars[SC_MF_MAPSCAT + k] = v[10 + k];
    scalars[SC_MF_MAPND] = v[19];
    scalars[SC_MF_SCANN] = v[20];
    double U[9], s[3], V[9];
    svd3(v, U, s, V);
    // det fix of U's last column, matrix_fisher_evidence.py:217-222
    double UVt[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) UVt[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
    double dt = det3(UVt);
    double sg = dt > 0.0 ? 1.0 : (dt < 0.0 ? -1.0 : 0.0);
    U[2] *= sg; U[5] *= sg; U[8] *= sg;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        scalars[SC_MF_R + 3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
    for (int k = 0; k < 3; ++k) scalars[SC_MF_S + k] = s[k];
    for (int k = 0; k < 9; ++k) scalars[SC_MF_V + k] = V[k];
  }
}

// ---------------------------------------------------------------- row 8: planar translation
// Per bin (matrix_fisher_evidence.py:442-475): t_b = c_map - R p_scan,
// S_b = Sigma_map + R Sigma_scan R^T, W_b = w_b inv(S_b + eps I); L += W_b, h += W_b t_b.
constexpr int kPtNV = 13;
__global__ __launch_bounds__(kBlock) void k_pt_partial(const double* __restrict__ scan, const double* __restrict__ map,
                                                       const double* __restrict__ derived, int B,
                                                       const double* __restrict__ scalars, double* partials) {
  __shared__ double lds[kWaves * kPtNV];
  double R[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = scalars[SC_MF_R + k];
  double v[kPtNV];
#pragma unroll
  for (int k = 0; k < kPtNV; ++k) v[k] = 0.0;
  size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    double Ns = scan[SF_N * Bs + b];
    double Nm = map[MF_NP * Bs + b];
    double pb[3], Sp[9], c[3], Sc[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) { pb[k] = scan[(SF_PB + k) * Bs + b]; c[k] = derived[(MD_C + k) * Bs + b]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) { Sp[k] = scan[(SF_SIG + k) * Bs + b]; Sc[k] = derived[(MD_SIG + k) * Bs + b]; }
    double tb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) tb[i] = c[i] - (R[3 * i] * pb[0] + R[3 * i + 1] * pb[1] + R[3 * i + 2] * pb[2]);
    double RS[9], S[9];
    mat3_mul(R, Sp, RS);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        S[3 * i + j] = Sc[3 * i + j] + (RS[3 * i] * R[3 * j] + RS[3 * i + 1] * R[3 * j + 1] + RS[3 * i + 2] * R[3 * j + 2]);
    S[0] += kEpsMass; S[4] += kEpsMass; S[8] += kEpsMass;
    double Si[9];
    inv3(S, Si);
    double wb = sqrt(Ns * Nm + kEpsMass);
#pragma unroll
    for (int k = 0; k < 9; ++k) Si[k] *= wb;
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] += Si[k];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[9 + i] += Si[3 * i] * tb[0] + Si[3 * i + 1] * tb[1] + Si[3 * i + 2] * tb[2];
    v[12] += wb;
  }
  block_sum<kPtNV>(v, lds);
  if (threadIdx.x == 0)
    for (int k = 0; k < kPtNV; ++k) partials[(size_t)blockIdx.x * kPtNV + k] = v[k];
}

__global__ __launch_bounds__(kBlock) void k_pt_final(const double* __restrict__ partials, int nblocks, double* scalars) {
  __shared__ double lds[kWaves * kPtNV];
  double v[kPtNV];
#pragma unroll
  for (int k = 0; k < kPtNV; ++k) v[k] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock)
#pragma unroll
    for (int k = 0; k < kPtNV; ++k) v[k] += partials[(size_t)b * kPtNV + k];
  block_sum<kPtNV>(v, lds);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 9; ++k) scalars[SC_PT_L + k] = v[k];
    for (int k = 0; k < 3; ++k) scalars[SC_PT_H + k] = v[9 + k];
    scalars[SC_PT_NEFF] = v[12];
  }
}

// ---------------------------------------------------------------- row 11: pushforward (declared)
// Per bin: forgetting + world-frame increments at z_t = (R, t) + derived stats.  With u = R p_bar
// and X = [u]x the pose-covariance pushforward J S J^T (J = [I, -R [p_bar]x]) is
// S_tt - X F - (X F)^T + X G X^T with F = R S_rt, G = R S_rr R^T precomputed on the host.
__device__ __forceinline__ void derive_bin(const double* sd, double nd, double np, const double* sp,
                                           const double* spp, double* derived, size_t Bs, int b) {
  double sn = sqrt(dot3_exact(sd[0], sd[1], sd[2], sd[0], sd[1], sd[2]));
  double dn = sn + kEpsMass;
#pragma unroll
  for (int k = 0; k < 3; ++k) derived[(MD_MU + k) * Bs + b] = sd[k] / dn;
  double invNd = 1.0 / (nd + kEpsMass + kF64Eps);
  derived[MD_KAPPA * Bs + b] = kappa_from_rbar(sn * invNd);
  double invNp = 1.0 / (np + kEpsMass + kF64Eps);
  double c[3] = {sp[0] * invNp, sp[1] * invNp, sp[2] * invNp};
  double raw[9], sig[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) raw[3 * i + j] = spp[3 * i + j] * invNp - c[i] * c[j];
  psd_project3(raw, sig);
#pragma unroll
  for (int k = 0; k < 3; ++k) derived[(MD_C + k) * Bs + b] = c[k];
#pragma unroll
  for (int k = 0; k < 9; ++k) derived[(MD_SIG + k) * Bs + b] = sig[k];
}

__global__ __launch_bounds__(kBlock) void k_pushforward(const double* __restrict__ scan, double* map, double* derived,
                                                        int B, PushArgs pa) {
  const size_t Bs = (size_t)B;
  const double* R = pa.R;
  const double g = pa.gamma;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    const double N = scan[SF_N * Bs + b];
    double pb[3], u[3], q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) pb[k] = scan[(SF_PB + k) * Bs + b];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u[i] = R[3 * i] * pb[0] + R[3 * i + 1] * pb[1] + R[3 * i + 2] * pb[2];
      q[i] = u[i] + pa.t[i];
    }
    // S_dir += R s_dir
    double sd[3];
    {
      double s0 = scan[(SF_SD + 0) * Bs + b], s1 = scan[(SF_SD + 1) * Bs + b], s2 = scan[(SF_SD + 2) * Bs + b];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        sd[i] = g * map[(MF_SD + i) * Bs + b] + (R[3 * i] * s0 + R[3 * i + 1] * s1 + R[3 * i + 2] * s2);
        map[(MF_SD + i) * Bs + b] = sd[i];
      }
    }
    // S_dir_scatter += R S R^T
    {
      double S[9], RS[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) S[k] = scan[(SF_S + k) * Bs + b];
      mat3_mul(R, S, RS);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          double v = RS[3 * i] * R[3 * j] + RS[3 * i + 1] * R[3 * j + 1] + RS[3 * i + 2] * R[3 * j + 2];
          map[(MF_S + 3 * i + j) * Bs + b] = g * map[(MF_S + 3 * i + j) * Bs + b] + v;
        }
    }
    const double nd = g * map[MF_ND * Bs + b] + N;
    const double np = g * map[MF_NP * Bs + b] + N;
    map[MF_ND * Bs + b] = nd;
    map[MF_NP * Bs + b] = np;
    double sp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sp[k] = g * map[(MF_SP + k) * Bs + b] + N * q[k];
      map[(MF_SP + k) * Bs + b] = sp[k];
    }
    // sum_ppT += N [ R (Sigma_p + p p^T) R^T + J S J^T + q q^T - u u^T ]
    double spp[9];
    {
      double M2[9], RM[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) M2[3 * i + j] = scan[(SF_SIG + 3 * i + j) * Bs + b] + pb[i] * pb[j];
      mat3_mul(R, M2, RM);
      double X[9], XF[9], XG[9];
      skew3(u, X);
      mat3_mul(X, pa.F, XF);
      mat3_mul(X, pa.G, XG);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          double rmr = RM[3 * i] * R[3 * j] + RM[3 * i + 1] * R[3 * j + 1] + RM[3 * i + 2] * R[3 * j + 2];
          double xgx = XG[3 * i] * X[3 * j] + XG[3 * i + 1] * X[3 * j + 1] + XG[3 * i + 2] * X[3 * j + 2];
          double jsj = pa.Stt[3 * i + j] - XF[3 * i + j] - XF[3 * j + i] + xgx;
          spp[3 * i + j] = g * map[(MF_SPP + 3 * i + j) * Bs + b] + N * (rmr + jsj + q[i] * q[j] - u[i] * u[j]);
          map[(MF_SPP + 3 * i + j) * Bs + b] = spp[3 * i + j];
        }
    }
    derive_bin(sd, nd, np, sp, spp, derived, Bs, b);
  }
}

// derived stats from map sufficient stats only (used after set_map / reset)
__global__ __launch_bounds__(kBlock) void k_map_derive(const double* __restrict__ map, double* derived, int B) {
  const size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    double sd[3], sp[3], spp[9];
    for (int k = 0; k < 3; ++k) { sd[k] = map[(MF_SD + k) * Bs + b]; sp[k] = map[(MF_SP + k) * Bs + b]; }
    for (int k = 0; k < 9; ++k) spp[k] = map[(MF_SPP + k) * Bs + b];
    derive_bin(sd, map[MF_ND * Bs + b], map[MF_NP * Bs + b], sp, spp, derived, Bs, b);
  }
}

// ---------------------------------------------------------------- launchers
static int grid_for(long n, int cap_blocks) {
  long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > cap_blocks ? cap_blocks : g);
}

hipError_t launch_budget(const double* w, int n_raw, int stride, double* partials, int nblk, double* scalars,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_budget_partial, dim3(nblk), dim3(kBlock), 0, s, w, n_raw, stride, partials);
  hipLaunchKernelGGL(k_budget_final, dim3(1), dim3(kBlock), 0, s, (const double*)partials, nblk, scalars);
  return hipGetLastError();
}

hipError_t launch_points(const PointKernelArgs& a, bool scale, double* partials, int nblk, hipStream_t s) {
  if (scale) {
    switch (a.k) {
      case 8: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_points<true, 8>), dim3(nblk), dim3(kBlock), 0, s, a, partials); break;
      case 16: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_points<true, 16>), dim3(nblk), dim3(kBlock), 0, s, a, partials); break;
      case 32: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_points<true, 32>), dim3(nblk), dim3(kBlock), 0, s, a, partials); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_points<false, 1>), dim3(nblk), dim3(kBlock), 0, s, a, partials);
  }
  // per-point cert partials -> scalars[SC_DESKEW_WIN..]: (sum wb, sum wn^2, sum wout, sum H, max r)
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_partials_final<5, 16u>), dim3(1), dim3(kBlock), 0, s, (const double*)partials,
                     nblk, a.scalars, (int)SC_DESKEW_WIN);
  return hipGetLastError();
}

hipError_t launch_bucketing(uint32_t* counts, uint32_t* starts, uint32_t* tile_sums, const uint32_t* keys,
                            const uint32_t* slots, int n, int n_bins, uint32_t* sorted, uint32_t* big_list,
                            uint32_t* big_n, hipStream_t s) {
  int tiles = (n_bins + kScanTile - 1) / kScanTile;
  hipLaunchKernelGGL(k_scan_tiles, dim3(tiles), dim3(kBlock), 0, s, (const uint32_t*)counts, n_bins, tile_sums);
  hipLaunchKernelGGL(k_scan_apply, dim3(tiles), dim3(kBlock), 0, s, (const uint32_t*)counts, n_bins,
                     (const uint32_t*)tile_sums, starts);
  hipLaunchKernelGGL(k_place, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, keys, slots, (const uint32_t*)starts, n,
                     n_bins, sorted);
  hipLaunchKernelGGL(k_bucket_order, dim3(grid_for(n_bins, 2048)), dim3(kBlock), 0, s, (const uint32_t*)counts,
                     (const uint32_t*)starts, n_bins, sorted, big_list, big_n);
  hipLaunchKernelGGL(k_bucket_big, dim3(64), dim3(kBlock), 0, s, keys, n, (const uint32_t*)starts,
                     (const uint32_t*)big_list, (const uint32_t*)big_n, sorted);
  return hipGetLastError();
}

int bins_scale_blocks(int n_bins) { return (n_bins + kTile - 1) / kTile; }

hipError_t launch_bins_scale(const BinKernelArgs& a, double* partials, hipStream_t s) {
  int nblk = bins_scale_blocks(a.n_bins);
  hipLaunchKernelGGL(k_bins_scale, dim3(nblk), dim3(kBlock), 0, s, a, partials);
  return hipGetLastError();
}

hipError_t launch_dense(const BinKernelArgs& a, double* bin_partials, double* partials, hipStream_t s) {
  int nchunks = (a.cap + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_dense_accum, dim3(nchunks), dim3(kBlock), 0, s, a, bin_partials);
  int nblk = (a.n_bins + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_dense_finalize, dim3(nblk), dim3(kBlock), 0, s, a, (const double*)bin_partials, nchunks, partials);
  return hipGetLastError();
}

hipError_t launch_bin_cert_final(const double* partials, int nblk, double* scalars, hipStream_t s) {
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_partials_final<5, 16u>), dim3(1), dim3(kBlock), 0, s, partials, nblk, scalars,
                     (int)SC_BIN_NSUM);
  return hipGetLastError();
}

hipError_t launch_mf(const double* scan, const double* map, int B, double* partials, int nblk, double* scalars,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_mf_partial, dim3(nblk), dim3(kBlock), 0, s, scan, map, B, partials);
  hipLaunchKernelGGL(k_mf_final, dim3(1), dim3(kBlock), 0, s, (const double*)partials, nblk, scalars);
  return hipGetLastError();
}

hipError_t launch_pt(const double* scan, const double* map, const double* derived, int B, double* partials, int nblk,
                     double* scalars, hipStream_t s) {
  hipLaunchKernelGGL(k_pt_partial, dim3(nblk), dim3(kBlock), 0, s, scan, map, derived, B, (const double*)scalars, partials);
  hipLaunchKernelGGL(k_pt_final, dim3(1), dim3(kBlock), 0, s, (const double*)partials, nblk, scalars);
  return hipGetLastError();
}

hipError_t launch_pushforward(const double* scan, double* map, double* derived, int B, const PushArgs& pa,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_pushforward, dim3(grid_for(B, 4096)), dim3(kBlock), 0, s, scan, map, derived, B, pa);
  return hipGetLastError();
}

hipError_t launch_map_derive(const double* map, double* derived, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_map_derive, dim3(grid_for(B, 4096)), dim3(kBlock), 0, s, map, derived, B);
  return hipGetLastError();
}

}  // namespace gcs
