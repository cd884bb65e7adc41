// HIP kernels for the GC-SLAM bin-path hot path on gfx950 (MI355X).
//
//   k_budget        PointBudgetResample mass sums (+ clears the bucketing state)  point_budget.py:50-109
//   k_points        budget fold + gather + DeskewConstantTwist + ray direction + nearest bin +
//                   K-candidate softmax normaliser (BinSoftAssign, scale mode) or dense
//                   softmax normaliser, and the per-point certificate partials
//                   deskew_constant_twist.py:31-69, pipeline.py:589-593, binning.py:56-76
//   k_scan, k_place, k_bucket_rank   deterministic bucketing of points by nearest bin
//   k_bins_scale    tiled bin-centric gather: ScanBinMomentMatch + Kappa + Matrix-Fisher terms
//                   binning.py:139-209, kappa.py:130-169, matrix_fisher_evidence.py:181-211
//   k_dense_*       the reference's dense N x B form (legacy B=48)
//   k_mf            MatrixFisherRotation bin reduction (dense mode / per-operator entry point)
//   k_pt            PlanarTranslationEvidence bin reduction   matrix_fisher_evidence.py:413-499
//   k_pushforward   PoseCovInflationPushforward + forgetting + derived map stats + map totals
//                   (declared; bin_atlas.py:137-257)
//   k_final         one-block folds of block partials (+ R_mf by polar Newton)
//
// All reductions are fixed-shape (fixed grid, fixed lane/LDS trees, fixed-order final pass),
// so results are bitwise reproducible run to run (docs/GC_SLAM.md:1150).  No float atomics.
#include <hip/hip_runtime.h>


#include "gcs_kernels.h"

#include <hip/hip_ext.h>
#include <string.h>
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

// Block partials are stored as rows of pstride(NV) doubles (16, or 32 for NV > 16).  In the fold
// G = stride / 4 threads share a row, thread t loading columns 4 (t % G) .. +3 (one 32-B load) of
// rows t / G, t / G + 256 / G, ...: the block sweeps 64 (or 32) rows per pass with coalesced,
// independent loads, the lanes of one column group meet in a fixed xor tree, then a fixed
// cross-wave order.
// The result is valid in thread 0.  Bit k of MAXMASK selects max instead of sum for component k.
// lds must hold kWaves * pstride(NV).  Columns >= NV are never read back.
template <int NV>
__host__ __device__ constexpr int pstride() { return NV <= 16 ? 16 : 32; }
int partial_stride(int nv) { return nv <= 16 ? 16 : 32; }

template <int NV, unsigned MAXMASK, int NT = kBlock>
__device__ __forceinline__ void reduce_partials(const double* __restrict__ partials, int nblocks, double (&v)[NV],
                                                double* lds) {
  constexpr int S = pstride<NV>();
  constexpr int G = S / 4;
  constexpr int R = NT / G;
  const int c0 = 4 * (threadIdx.x % G), r0 = threadIdx.x / G;
  bool mx[4];
  double a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mx[k] = c0 + k < NV && ((MAXMASK >> (c0 + k)) & 1u);
    a[k] = mx[k] ? -INFINITY : 0.0;
  }
#pragma unroll 8
  for (int b = r0; b < nblocks; b += R) {
    const double4 x = *(const double4*)(partials + (size_t)b * S + c0);
    a[0] = mx[0] ? fmax(a[0], x.x) : a[0] + x.x;
    a[1] = mx[1] ? fmax(a[1], x.y) : a[1] + x.y;
    a[2] = mx[2] ? fmax(a[2], x.z) : a[2] + x.z;
    a[3] = mx[3] ? fmax(a[3], x.w) : a[3] + x.w;
  }
#pragma unroll
  for (int off = G; off < 64; off <<= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double y = __shfl_xor(a[k], off, 64);
      a[k] = mx[k] ? fmax(a[k], y) : a[k] + y;
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < G)
#pragma unroll
    for (int k = 0; k < 4; ++k) lds[wid * S + c0 + k] = a[k];
  __syncthreads();
  // the cross-wave fold: lane k of wave 0 folds component k over the waves in order (the serial
  // fold by thread 0 was NV x waves dependent LDS reads: the tail of a 1024-thread fold)
  double s = 0.0;
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    const bool mx = (MAXMASK >> k) & 1u;
    s = lds[k];
    for (int w = 1; w < NT / 64; ++w) s = mx ? fmax(s, lds[w * S + k]) : s + lds[w * S + k];
  }
  if (threadIdx.x < 64) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __shfl(s, k, 64);
  }
  __syncthreads();
}

// Block partials are folded by a separate one-block k_final launch queued right behind the
// producer (back-to-back dispatch, no gap).  Measured against "last block finishes" tickets in the
// producer (sc1 stores + ticket + in-kernel fold): the separate fold was 15 us faster on the bin
// kernel, because the in-kernel form holds every block until its ticket returns and runs the
// fold and the 3x3 polar factor as a serial tail of the producer.
template <int NV>
__device__ __forceinline__ void store_partials(const double (&v)[NV], double* base, int idx) {
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) base[(size_t)idx * pstride<NV>() + k] = v[k];
}

// ---------------------------------------------------------------- PointCloud2 parse (before row 1)
// parse_pointcloud2_vlp16 (backend_node.py:377-468) + the base transform (:1677-1680), one thread
// per point over the raw message bytes: x/y/z FLOAT32 with the non-finite sentinel (nan_to_num),
// ring, per-point time (seconds, or ns when any value exceeds 1e6: an integer flag word reduced
// with atomicOr, applied by k_parse_time_scale), range-sigmoid weights on the lidar-frame range,
// points in the base frame (f64, 3 per point).  numpy's operation order, no contraction.
__device__ __forceinline__ double pc2_field(const uint8_t* p, int datatype) {
  switch (datatype) {  // sensor_msgs/PointField codes, little endian
    case 1: { int8_t v; __builtin_memcpy(&v, p, 1); return (double)v; }
    case 2: { uint8_t v; __builtin_memcpy(&v, p, 1); return (double)v; }
    case 3: { int16_t v; __builtin_memcpy(&v, p, 2); return (double)v; }
    case 4: { uint16_t v; __builtin_memcpy(&v, p, 2); return (double)v; }
    case 5: { int32_t v; __builtin_memcpy(&v, p, 4); return (double)v; }
    case 6: { uint32_t v; __builtin_memcpy(&v, p, 4); return (double)v; }
    case 7: { float v; __builtin_memcpy(&v, p, 4); return (double)v; }
    default: { double v; __builtin_memcpy(&v, p, 8); return v; }
  }
}
__device__ __forceinline__ double nan_to_num_sentinel(double v) {
  if (v != v) return 1e6;  // GC_NONFINITE_SENTINEL, constants.py:256-262
  if (v == INFINITY) return 1e6;
  if (v == -INFINITY) return -1e6;
  return v;
}
__global__ __launch_bounds__(kBlock) void k_parse_pc2(ParseArgs a) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const uint8_t* rec = a.data + (size_t)i * (size_t)a.point_step;
  const double x = nan_to_num_sentinel(pc2_field(rec + a.off_x, 7));
  const double y = nan_to_num_sentinel(pc2_field(rec + a.off_y, 7));
  const double z = nan_to_num_sentinel(pc2_field(rec + a.off_z, 7));
  if (a.ring) a.ring[i] = (uint8_t)(int64_t)pc2_field(rec + a.off_ring, a.ring_datatype);
  double t = a.header_stamp;
  if (a.off_t >= 0) {
    t = pc2_field(rec + a.off_t, a.t_datatype);
    if (t > 1e6) atomicOr(a.ns_flag, 1u);
  }
  a.t[i] = t;
  const double dist = sqrt((x * x + y * y) + z * z);
  const double ra = (dist - 0.5) / 0.25, rb = (50.0 - dist) / 0.25;  // constants.py:256-262
  const double w_raw = (1.0 / (1.0 + exp(-ra))) * (1.0 / (1.0 + exp(-rb)));
  a.w[i] = w_raw * (1.0 - kWeightFloor) + kWeightFloor;
  const double* R = a.R;
  double* o = a.points + 3 * (size_t)i;
  o[0] = ((R[0] * x + R[1] * y) + R[2] * z) + a.tb[0];
  o[1] = ((R[3] * x + R[4] * y) + R[5] * z) + a.tb[1];
  o[2] = ((R[6] * x + R[7] * y) + R[8] * z) + a.tb[2];
}
__global__ __launch_bounds__(kBlock) void k_parse_time_scale(double* t, int n, const uint32_t* ns_flag) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n && *ns_flag) t[i] = t[i] * 1e-9;
}

// ---------------------------------------------------------------- row 1: budget mass sums
// Also clears the scale-mode bucketing state of this scan (counts, flags, look-back status),
// replacing three memsets.  mass_scale = total_mass_in / (total_mass_selected + eps_mass)
// (point_budget.py:80-84) is produced by k_final<FIN_BUDGET>.
// zero nb bytes at p with the grid's threads: 16-B stores for the aligned body, byte stores for the
// head and tail (nb and p need no alignment; nb <= 0 or p null: nothing)
__device__ __forceinline__ void clear_bytes16(uint8_t* p, long nb, long gid, long gsz) {
  if (!p || nb <= 0) return;
  long head = (long)((16 - ((uintptr_t)p & 15)) & 15);
  head = head > nb ? nb : head;
  for (long j = gid; j < head; j += gsz) p[j] = 0u;
  const long nq = (nb - head) / 16;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (long j = gid; j < nq; j += gsz) q[j] = make_uint4(0u, 0u, 0u, 0u);
  for (long j = head + 16 * nq + gid; j < nb; j += gsz) p[j] = 0u;
}

__global__ __launch_bounds__(kBlock) void k_budget(BudgetArgs a) {
  __shared__ double lds[kWaves * 2];
  const int gid = blockIdx.x * kBlock + threadIdx.x, gsz = gridDim.x * kBlock;
  // 16-B stores for the aligned body, element stores for the head and tail (1-B stores ran the C3
  // clear at ~0.4 TB/s)
  clear_bytes16(reinterpret_cast<uint8_t*>(a.zero32), 4L * a.n_zero32, gid, gsz);
  clear_bytes16(a.zero8, a.n_zero8, gid, gsz);
  double v[2] = {0.0, 0.0};
  for (int j = gid; j < a.n_raw; j += gsz) {
    double x = a.w[j];
    v[0] += x;
    if (j % a.stride == 0) v[1] += x;
  }
  block_sum<2>(v, lds);
  store_partials<2>(v, a.partials, blockIdx.x);
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

// ray_dir (the point direction from the LiDAR origin): gcs_math.h

// ---------------------------------------------------------------- row 1+3+5: the point kernel
// One thread per budget output slot i in [0, cap).  SCALE = candidate-restricted softmax.
// At C2 the grid is ~1 wave per SIMD, so the kernel is bound by each lane's dependent chain:
// loads are issued in independent batches (whole pool row, whole candidate row) so the chain is
// xyz -> pool ids -> pool dirs -> knn row -> candidate dirs -> slot atomic, and the softmax
// evaluates one exp per candidate and no per-candidate log (entropy identity below).
// LP > 1 (scale mode): LP lanes per point.  Each lane scans every LP-th chunk of the pool row and
// takes KC/LP of the candidates, so the chain's load batches are LP times narrower per lane and
// the register file holds KC/LP candidate terms; the lanes' nearest bins meet in a (dot, lower
// id) max, their softmax terms in fixed xor trees (identical on every lane of the point).  One
// lane per point takes the slot atomic and writes the record.
#ifndef GCS_POINT_WAVES
#define GCS_POINT_WAVES 0  // register target (waves per SIMD) of k_points; 0: compiler default
#endif
#ifndef GCS_PROBE_NOPOOL
#define GCS_PROBE_NOPOOL 0
#endif
#ifndef GCS_PROBE_NOFLAGS
#define GCS_PROBE_NOFLAGS 0  // timing probe (not a parity build): no first-arrival flag stores
#endif
#ifndef GCS_CAND_GROUP
#define GCS_CAND_GROUP 16  // candidate direction loads in flight per group (16: all at once)
#endif
// KC == 0 (!SCALE): deskew only -- the live primitive path's point stage (pipeline.py:399-418,
// 568-587): budget gather, deskew, window weights and the budget / deskew certificate partials, no
// soft assign and no record (the surfel extraction reads p0_out / w_out / t_out).
template <bool SCALE, int KC, int LP>
__global__ __launch_bounds__(kBlock)
#if GCS_POINT_WAVES
__attribute__((amdgpu_waves_per_eu(GCS_POINT_WAVES)))
#endif
void k_points(PointKernelArgs a, double* partials) {
  static_assert(LP == 1 || (SCALE && (LP == 2 || LP == 4) && KC % LP == 0), "lanes per point");
  constexpr int KL = KC / LP, kPB = kBlock / LP;  // candidates per lane, points per block
  constexpr int kCandGroup = KL < GCS_CAND_GROUP ? (KL > 0 ? KL : 1) : GCS_CAND_GROUP;
  const int sub = threadIdx.x % LP;
  __shared__ double lds[kWaves * 5];
  __shared__ double s_mass[2];
  // budget mass sums: every block folds k_budget's partial rows itself (same fixed order in every
  // block), so no separate fold launch sits between the two kernels; block 0 publishes them.  The
  // rows are loaded here and folded after the first point's geometry (which needs no weight), so
  // their latency and the fold's barriers overlap the point's dependent chain.
  static_assert(kBlock * 4 >= 1024, "k_budget launches at most 1024 blocks: four rows per thread");
  double2 brow[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = threadIdx.x + k * kBlock;
    brow[k] = r < a.budget_blocks ? *(const double2*)(a.budget_partials + (size_t)r * pstride<2>())
                                  : make_double2(0.0, 0.0);
  }
  // the deskew twist: by value, or (pre-launched scan front) from the device word k_gate wrote
  // before this kernel started (stream order makes it visible)
  double xi[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) xi[k] = a.xi_dev ? a.xi_dev[k] : a.xi[k];
  const double denom = a.t1 - a.t0 > 1e-12 ? a.t1 - a.t0 : 1e-12;
  const double inv_tau = 1.0 / a.tau;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sum w_budget, sum wn^2, sum w_out, sum H
  double rmax = -INFINITY;
  double mass_scale = 0.0, mass_in = 0.0;
  // self-budget (PointKernelArgs.mass_rows, scale mode): no fold; the block's raw mass sums go to its row
  const bool self = SCALE && a.mass_rows != nullptr;
  double msum[2] = {0.0, 0.0};
  if (self) mass_scale = 1.0;
  // uniform trip count (the budget fold inside the first iteration has barriers)
  const int gstride = gridDim.x * kPB;
  const int niter = (a.cap + gstride - 1) / gstride;
  for (int it = 0; it < niter; ++it) {
    const int i = blockIdx.x * kPB + (int)threadIdx.x / LP + it * gstride;
    const bool live = i < a.cap;
    double p[3] = {0.0, 0.0, 0.0}, t = 0.0, w_raw = 0.0;
    bool valid = live && i < a.n_sel;
    if (valid) {
      size_t src = (size_t)i * (size_t)a.stride;
      if (a.xyz_f64) {  // parsed base-frame points (k_parse_pc2)
        const double* rec = (const double*)(a.xyz + src * (size_t)a.point_step);
        p[0] = rec[0]; p[1] = rec[1]; p[2] = rec[2];
      } else {
        const float* rec = (const float*)(a.xyz + src * (size_t)a.point_step);
        p[0] = (double)rec[0]; p[1] = (double)rec[1]; p[2] = (double)rec[2];
      }
      t = a.timestamps[src];
      w_raw = a.weights[src];
      if (self && sub == 0) {
        double wall = w_raw;
        for (int q = 1; q < a.stride && src + q < (size_t)a.n_raw; ++q) wall += a.weights[src + q];
        msum[0] += wall;
        msum[1] += w_raw;
      }
    }
    double alpha = (t - a.t0) / denom;
    double p0[3];
    deskew_point(alpha, xi, p, p0);
    const double win = smooth_window(t, a.t0, a.t1, kTimeWarpSigmaFrac * denom);
    double d[3];
    ray_dir(p0[0], p0[1], p0[2], a.origin, d);
    double m = -INFINITY, Z = 0.0, H = 0.0, rm = 0.0;
    int nearest = 0;
    if constexpr (!SCALE && KC == 0) {
      // deskew only: no soft assign
    } else if constexpr (SCALE) {
      // exact nearest atlas bin: the first maximum of the exact dot in reference-id order over the
      // pool of the direction's cube cell.  The pool is nearest-first (angle from the cell centre)
      // with a per-entry upper bound of the dot of any in-cell direction with that entry and every
      // later one: the search stops at the first batch whose successor's bound is below the best dot
      // (no later bin can reach or tie it), typically after one batch of 8 instead of the whole row.
      bool zero = (d[0] == 0.0 && d[1] == 0.0 && d[2] == 0.0);
      if (!zero) {
        const size_t prow = (size_t)cube_cell(d[0], d[1], d[2], a.grid) * a.pool_width;
        const int4* pool = (const int4*)(a.pools + prow);
        const float* pbound = a.pool_bound + prow;
        const int nq = a.pool_width >> 2;
        double best = -INFINITY;
        // 4 * CH ids per batch and lane: all loads in flight together
        constexpr int CH = LP >= 4 ? 1 : 2;
        // GCS_PROBE_NOPOOL (timing probe, not a parity build): the first pool id only
        for (int q = sub; q < (GCS_PROBE_NOPOOL ? 1 : nq); q += CH * LP) {
          int4 u0 = pool[q];
          int4 u1 = CH == 2 && q + LP < nq ? pool[q + LP] : make_int4(-1, -1, -1, -1);
          const int qn = q + CH * LP;  // this lane's next batch
          const float bnext = qn < nq ? pbound[4 * qn] : -2.0f;
          int ids[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
          double s[8];
          // branch-free: a guarded load per id compiled to one branch and one wait per id (the
          // batch's loads went out one round trip at a time); padding ids (-1) read bin 0 and
          // are masked to -inf after the loads
#pragma unroll
          for (int u = 0; u < 4 * CH; ++u) {
            const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)(ids[u] >= 0 ? ids[u] : 0));
            const double sv = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
            s[u] = ids[u] >= 0 ? sv : -INFINITY;
          }
#pragma unroll
          for (int u = 0; u < 4 * CH; ++u) {
            if (s[u] > best) {
              best = s[u];
              nearest = ids[u];
            } else if (s[u] == best && ids[u] >= 0 && a.bin_ref[ids[u]] < a.bin_ref[nearest]) {
              nearest = ids[u];  // an exact tie (measure zero): the lower reference id
            }
          }
          // the bound is for unit directions and |d| < 1 (ray_dir divides by nrm + eps): it bounds the
          // scaled dot of a later entry only while best > 0 (always, for any atlas of >= 48 bins)
          if ((CH == 2 ? u1.w : u0.w) < 0 || (best > 0.0 && (double)bnext < best)) break;
        }
#pragma unroll
        for (int off = 1; off < LP; off <<= 1) {  // first maximum in reference-id order
          const double ob = __shfl_xor(best, off, 64);
          const int oi = __shfl_xor(nearest, off, 64);
          if (ob > best || (ob == best && a.bin_ref[oi] < a.bin_ref[nearest])) { best = ob; nearest = oi; }
        }
      }
      int cand[KL];
      if constexpr (KL % 4 == 0) {
        const int4* cand4 = (const int4*)(a.knn + (size_t)nearest * KC + sub * KL);
#pragma unroll
        for (int k = 0; k < KL / 4; ++k) {
          int4 c4 = cand4[k];
          cand[4 * k] = c4.x; cand[4 * k + 1] = c4.y; cand[4 * k + 2] = c4.z; cand[4 * k + 3] = c4.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < KL; ++k) cand[k] = a.knn[(size_t)nearest * KC + sub * KL + k];
      }
      double e[KL];
      // the candidates' directions in groups of GCS_CAND_GROUP loads in flight (x, y, z only: 24 B)
#pragma unroll
      for (int k0 = 0; k0 < KL; k0 += kCandGroup) {
        double3 bd[kCandGroup];
#pragma unroll
        for (int k = 0; k < kCandGroup; ++k) {
          const double* p = a.bin_dirs + 4 * (size_t)cand[k0 + k];
          const double2 xy = *(const double2*)p;
          bd[k] = make_double3(xy.x, xy.y, p[2]);
        }
#pragma unroll
        for (int k = 0; k < kCandGroup; ++k) {
          e[k0 + k] = dot3_exact(d[0], d[1], d[2], bd[k].x, bd[k].y, bd[k].z);
          m = fmax(m, e[k0 + k]);
        }
        if (kCandGroup < KL) __builtin_amdgcn_sched_barrier(0);  // keep the groups apart (registers)
      }
#pragma unroll
      for (int off = 1; off < LP; off <<= 1) m = fmax(m, __shfl_xor(m, off, 64));
      // e_k = exp(x_k), x_k = (sim_k - m)/tau (binning.py:69 softmax, shifted by the max)
      double sxe = 0.0;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        double x = (e[k] - m) * inv_tau;
        e[k] = exp(x);
        Z += e[k];
        sxe += x * e[k];
      }
#pragma unroll
      for (int off = 1; off < LP; off <<= 1) {
        Z += __shfl_xor(Z, off, 64);
        sxe += __shfl_xor(sxe, off, 64);
      }
      const double iz = 1.0 / Z;
      // entropy of r_k = e_k/Z (binning.py:71-75): -sum r log(r + eps)
      //   = log Z - sum r_k x_k - sum r_k log1p(eps/r_k),
      // with r log1p(eps/r) in [0, eps] taken as eps r/(r + eps) (|error| < 0.2 eps per term)
      double corr = 0.0;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        double r = e[k] * iz;
        corr += r * __builtin_amdgcn_rcp(r + kEpsMass);
        rm = fmax(rm, r);
      }
#pragma unroll
      for (int off = 1; off < LP; off <<= 1) {
        corr += __shfl_xor(corr, off, 64);
        rm = fmax(rm, __shfl_xor(rm, off, 64));
      }
      H = log(Z) - sxe * iz - kEpsMass * corr;
      uint32_t key = (uint32_t)a.n_bins;
      if (valid && sub == 0) {
        // bucket slot: arrival order only (re-ranked by point index by k_bucket_rank, or by the bin
        // kernel's staging for the direct buckets)
        const uint32_t sl = atomicAdd(a.counts + nearest, 1u);
        key = (uint32_t)nearest;
        if (a.members) {
          // direct buckets: slots / keys only feed the sorted bucketing (an overflowing scan is
          // redone from k_points with members == nullptr), so they are not written here
          if (sl < (uint32_t)a.capb) a.members[(size_t)nearest * a.capb + sl] = (uint32_t)i;
          else *a.overflow = 1u;  // vector store to host-mapped memory; gcs_scan redoes the scan sorted
          if (!GCS_PROBE_NOFLAGS && sl == 0u) {  // first arrival: mark the candidate bins and their tiles
            // (storing each tile flag once per row measured 20 us slower at C3: the compare chain)
            const int ts = a.tile_shift;
            uint8_t* tf = a.flags + a.n_bins;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
              const int c = LP == 1 ? cand[k % KL] : a.knn[(size_t)nearest * KC + k];
              a.flags[c] = 1;
              tf[c >> ts] = 1;
            }
          }
        } else {
          a.slots[i] = sl;
        }
      }
      if (live && sub == 0 && !a.members) a.keys[i] = key;
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
    if (it == 0 && !self) {  // block-uniform: the budget fold
      double v[2] = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[0] += brow[k].x;
        v[1] += brow[k].y;
      }
      block_sum<2>(v, lds);
      if (threadIdx.x == 0) {
        s_mass[0] = v[0];
        s_mass[1] = v[0] / (v[1] + kEpsMass);  // mass_scale, point_budget.py:80-84
        if (blockIdx.x == 0) {
          a.scalars[SC_MASS_IN] = v[0];
          a.scalars[SC_MASS_SEL] = v[1];
          a.scalars[SC_MASS_SCALE] = s_mass[1];
        }
      }
      __syncthreads();
      mass_scale = s_mass[1];
      mass_in = s_mass[0];
    }
    if (!live || sub != 0) continue;
    const double wb = w_raw * mass_scale;
    const double wout = wb * win;
    if (a.t_out) a.t_out[i] = t;
    if constexpr (SCALE) {  // the 32-B record (gcs_layout.h PointRec32)
      reinterpret_cast<double4*>(a.recs)[i] = make_double4(p0[0], p0[1], p0[2], wout * Z);
    } else if constexpr (KC != 0) {
      PointRec pr;
      pr.x = p0[0]; pr.y = p0[1]; pr.z = p0[2];
      pr.dx = d[0]; pr.dy = d[1]; pr.dz = d[2];
      pr.m = m; pr.wz = wout * Z;
      a.recs[i] = pr;
    }
    if (a.iz_out) a.iz_out[i] = Z;
    if (a.p0_out) { a.p0_out[3 * (size_t)i] = p0[0]; a.p0_out[3 * (size_t)i + 1] = p0[1]; a.p0_out[3 * (size_t)i + 2] = p0[2]; }
    if (a.w_out) a.w_out[i] = wout;
    if (a.w_budget_out) a.w_budget_out[i] = wb;
    if (a.nearest_out) a.nearest_out[i] = nearest;
    double wn = self ? wb : wb / (mass_in + kEpsMass);  // (self-budget: raw sums, k_lean's convention)
    acc[0] += wb;
    acc[1] += wn * wn;
    acc[2] += wout;
    acc[3] += H;
    rmax = fmax(rmax, rm);
  }
  if (self) {
    block_sum<2>(msum, lds);
    if (threadIdx.x == 0) a.mass_rows[blockIdx.x] = make_double2(msum[0], msum[1]);
  }
  block_sum<4>(acc, lds);
  rmax = block_max(rmax, lds);
  double v[5] = {acc[0], acc[1], acc[2], acc[3], rmax};
  // (sum wb, sum wn^2, sum w_out, sum H, max r) -> scalars[SC_DESKEW_WIN..] by k_final<FIN_POINTS>
  store_partials<5>(v, partials, blockIdx.x);
}

// ---------------------------------------------------------------- row 1+3+5, scale mode: the lean point kernel
// The same per-point arithmetic as k_points<true, KC, 1> (bitwise the same records, buckets, flags
// and partial rows), laid out for occupancy and for the XCDs' L2s:
//  * registers: the budget rows are folded into two doubles as soon as they land, the nearest-bin
//    batch loads x, y, z only (24 B per id), the candidate directions arrive in groups of CG and the
//    candidate ids are not kept past their loads (the rare first-arrival flag marking re-reads the
//    kNN row), so the kernel fits 128 VGPRs: four waves per SIMD, the whole C3 grid (1,024 blocks)
//    resident in one round instead of four rounds at one wave per SIMD;
//  * XCD-aware block order: blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
//    "Workgroup dispatch"), so block b computes logical block (b % 8) * (grid / 8) + b / 8: each XCD
//    takes one contiguous eighth of the scan (an azimuth sector), and the atlas rows that sector
//    touches (cube-cell pools, bin directions, kNN rows) are fetched into one L2 instead of all
//    eight.  Partial rows are stored at the logical block index: the fold order is unchanged.
#ifndef GCS_PROBE_NOEXP
#define GCS_PROBE_NOEXP 0
#endif
#ifndef GCS_PROBE_NOMASS
#define GCS_PROBE_NOMASS 0  // timing probe (not a parity build): the bin kernel's blocks skip the mass-row loads
#endif
#ifndef GCS_PROBE_NOFIN
#define GCS_PROBE_NOFIN 0  // timing probe (not a parity build): phase D skips finalize_bin / the MF term
#endif
#ifndef GCS_LEAN_CG
#define GCS_LEAN_CG 8  // candidate direction loads in flight per group
#endif
#ifndef GCS_LEAN_XCD
#define GCS_LEAN_XCD 1  // XCD-aware block order (0: identity, for A/B)
#endif
#ifndef GCS_LEAN_EG
#define GCS_LEAN_EG 4  // candidate exps interleaved per group (registers)
#endif
// WIDE: grids of at most one wave per SIMD (cap <= 256 CUs x 4 SIMDs x 64 lanes, C2): occupancy is
// one wave per SIMD whatever the registers, so the 128-register target is dropped and the candidate
// directions go out in one group (one dependent memory round trip fewer on the point's chain).
template <int KC, bool WIDE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WIDE ? 1 : 4)))
void k_points_lean(PointKernelArgs a, double* partials) {
  // one point per thread (the grid covers cap: points_blocks); no grid-stride loop, so nothing
  // loop-invariant is hoisted into registers across the point's chain
  constexpr int CG = (WIDE || KC < GCS_LEAN_CG) ? KC : GCS_LEAN_CG;
  static_assert(KC % CG == 0, "candidate groups");
  __shared__ double lds[kWaves * 5];
  __shared__ double s_mass[2];
  const int nb = (int)gridDim.x;
  const int lb = (!GCS_LEAN_XCD || (nb & 7)) ? (int)blockIdx.x
                                             : (int)(blockIdx.x & 7u) * (nb >> 3) + (int)(blockIdx.x >> 3);
  static_assert(kBlock * 4 >= 1024, "k_budget launches at most 1024 blocks: four rows per thread");
  double2 brow[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = threadIdx.x + k * kBlock;
    brow[k] = r < a.budget_blocks ? *(const double2*)(a.budget_partials + (size_t)r * pstride<2>())
                                  : make_double2(0.0, 0.0);
  }
  const int i = lb * kBlock + (int)threadIdx.x;
  const bool live = i < a.cap;
  const bool valid = live && i < a.n_sel;
  double p[3] = {0.0, 0.0, 0.0}, t = 0.0, w_raw = 0.0;
  if (valid) {
    const size_t src = (size_t)i * (size_t)a.stride;
    if (a.xyz_f64) {
      const double* rec = (const double*)(a.xyz + src * (size_t)a.point_step);
      p[0] = rec[0]; p[1] = rec[1]; p[2] = rec[2];
    } else {
      const float* rec = (const float*)(a.xyz + src * (size_t)a.point_step);
      p[0] = (double)rec[0]; p[1] = (double)rec[1]; p[2] = (double)rec[2];
    }
    t = a.timestamps[src];
    w_raw = a.weights[src];
  }
  // the budget rows landed before the point's loads: two doubles from here on.  Self-budget (no
  // k_budget, PointKernelArgs.mass_rows): this point's own raw mass instead -- every raw weight of its
  // stride window (point_budget.py:80-84's mass_in) and its selected one (mass_sel)
  double bsum[2] = {0.0, 0.0};
  if (a.mass_rows) {
    if (valid) {
      const size_t src = (size_t)i * (size_t)a.stride;
      bsum[0] = w_raw;
      for (int q = 1; q < a.stride && src + q < (size_t)a.n_raw; ++q) bsum[0] += a.weights[src + q];
      bsum[1] = w_raw;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bsum[0] += brow[k].x;
      bsum[1] += brow[k].y;
    }
  }
  double p0[3], d[3], win;
  {
    double xi[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) xi[k] = a.xi_dev ? a.xi_dev[k] : a.xi[k];
    const double denom = a.t1 - a.t0 > 1e-12 ? a.t1 - a.t0 : 1e-12;
    const double alpha = (t - a.t0) / denom;
    deskew_point(alpha, xi, p, p0);
    win = smooth_window(t, a.t0, a.t1, kTimeWarpSigmaFrac * denom);
    ray_dir(p0[0], p0[1], p0[2], a.origin, d);
  }
  int nearest = 0;
  // exact nearest atlas bin (k_points: first maximum in reference-id order over the cube cell's
  // nearest-first pool, stopped once no later entry can reach the best dot)
  if (!(d[0] == 0.0 && d[1] == 0.0 && d[2] == 0.0)) {
    const size_t prow = (size_t)cube_cell(d[0], d[1], d[2], a.grid) * a.pool_width;
    const int4* pool = (const int4*)(a.pools + prow);
    const float* pbound = a.pool_bound + prow;
    const int nq = a.pool_width >> 2;
    double best = -INFINITY;
    for (int q = 0; q < nq; q += 2) {
      const int4 u0 = pool[q];
      const int4 u1 = q + 1 < nq ? pool[q + 1] : make_int4(-1, -1, -1, -1);
      const float bnext = q + 2 < nq ? pbound[4 * (q + 2)] : -2.0f;
      const int ids[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      double s[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double* bp = a.bin_dirs + 4 * (size_t)(ids[u] >= 0 ? ids[u] : 0);
        const double2 xy = *(const double2*)bp;
        const double sv = dot3_exact(d[0], d[1], d[2], xy.x, xy.y, bp[2]);
        s[u] = ids[u] >= 0 ? sv : -INFINITY;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (s[u] > best) {
          best = s[u];
          nearest = ids[u];
        } else if (s[u] == best && ids[u] >= 0 && a.bin_ref[ids[u]] < a.bin_ref[nearest]) {
          nearest = ids[u];
        }
      }
      if (u1.w < 0 || (best > 0.0 && (double)bnext < best)) break;  // (k_points: the bound needs best > 0)
    }
  }
  double e[KC];
  double m = -INFINITY;
  {
    const int* krow = a.knn + (size_t)nearest * KC;
#pragma unroll
    for (int k0 = 0; k0 < KC; k0 += CG) {
      int cid[CG];
#pragma unroll
      for (int k = 0; k < CG; k += 4) {
        const int4 c4 = *(const int4*)(krow + k0 + k);
        cid[k] = c4.x; cid[k + 1] = c4.y; cid[k + 2] = c4.z; cid[k + 3] = c4.w;
      }
      // a later group's direction loads wait for the previous group's dots (the compiler would
      // otherwise issue all KC loads at once: 6 KC registers in flight)
      if (k0 > 0)
#pragma unroll
        for (int k = 0; k < CG; ++k) __asm__ volatile("" : "+v"(cid[k]) : "v"(m));
      double3 bd[CG];
#pragma unroll
      for (int k = 0; k < CG; ++k) {
        const double* bp = a.bin_dirs + 4 * (size_t)cid[k];
        const double2 xy = *(const double2*)bp;
        bd[k] = make_double3(xy.x, xy.y, bp[2]);
      }
#pragma unroll
      for (int k = 0; k < CG; ++k) {
        e[k0 + k] = dot3_exact(d[0], d[1], d[2], bd[k].x, bd[k].y, bd[k].z);
        m = fmax(m, e[k0 + k]);
      }
      if (CG < KC) __builtin_amdgcn_sched_barrier(0);
    }
  }
  const double inv_tau = 1.0 / a.tau;
  double Z = 0.0, sxe = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const double x = (e[k] - m) * inv_tau;
    e[k] = exp(x);
    Z += e[k];
    sxe += x * e[k];
    if ((k & (GCS_LEAN_EG - 1)) == GCS_LEAN_EG - 1) __builtin_amdgcn_sched_barrier(0);  // bound the exps in flight
  }
  const double iz = 1.0 / Z;
  double corr = 0.0, rm = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const double r = e[k] * iz;
    corr += r * __builtin_amdgcn_rcp(r + kEpsMass);
    rm = fmax(rm, r);
  }
  const double H = log(Z) - sxe * iz - kEpsMass * corr;
  if (valid) {
    const uint32_t sl = atomicAdd(a.counts + nearest, 1u);
    if (a.members) {
      if (sl < (uint32_t)a.capb) a.members[(size_t)nearest * a.capb + sl] = (uint32_t)i;
      else *a.overflow = 1u;
      if (sl == 0u) {  // first arrival: mark the candidate bins and their tiles active
        const int ts = a.tile_shift;
        uint8_t* tf = a.flags + a.n_bins;
        const int* krow = a.knn + (size_t)nearest * KC;
        for (int k = 0; k < KC; k += 4) {
          const int4 c4 = *(const int4*)(krow + k);
          a.flags[c4.x] = 1; tf[c4.x >> ts] = 1;
          a.flags[c4.y] = 1; tf[c4.y >> ts] = 1;
          a.flags[c4.z] = 1; tf[c4.z >> ts] = 1;
          a.flags[c4.w] = 1; tf[c4.w >> ts] = 1;
        }
      }
    } else {
      a.slots[i] = sl;
    }
  }
  if (live && !a.members) a.keys[i] = valid ? (uint32_t)nearest : (uint32_t)a.n_bins;
  // the budget fold (block-uniform); self-budget: the block's mass row (the bin kernel folds the rows)
  block_sum<2>(bsum, lds);
  if (threadIdx.x == 0) {
    if (a.mass_rows) {
      a.mass_rows[lb] = make_double2(bsum[0], bsum[1]);
      s_mass[0] = 0.0;
      s_mass[1] = 1.0;
    } else {
      s_mass[0] = bsum[0];
      s_mass[1] = bsum[0] / (bsum[1] + kEpsMass);  // mass_scale, point_budget.py:80-84
      if (lb == 0) {
        a.scalars[SC_MASS_IN] = bsum[0];
        a.scalars[SC_MASS_SEL] = bsum[1];
        a.scalars[SC_MASS_SCALE] = s_mass[1];
      }
    }
  }
  __syncthreads();
  const double mass_scale = s_mass[1], mass_in = s_mass[0];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sum w_budget, sum wn^2, sum w_out, sum H
  double rmax = -INFINITY;
  if (live) {
    const double wb = w_raw * mass_scale;
    const double wout = wb * win;
    // the 32-B record: d and m are recomputed by the bin kernel's staging (gcs_layout.h PointRec32)
    reinterpret_cast<double4*>(a.recs)[i] = make_double4(p0[0], p0[1], p0[2], wout * iz);
    if (a.t_out) a.t_out[i] = t;
    if (a.iz_out) a.iz_out[i] = iz;
    if (a.p0_out) { a.p0_out[3 * (size_t)i] = p0[0]; a.p0_out[3 * (size_t)i + 1] = p0[1]; a.p0_out[3 * (size_t)i + 2] = p0[2]; }
    if (a.w_out) a.w_out[i] = wout;
    if (a.w_budget_out) a.w_budget_out[i] = wb;
    if (a.nearest_out) a.nearest_out[i] = nearest;
    // (self-budget: raw sums -- wb is w and the second column sum w^2; k_bins_scale's block 0 scales them)
    const double wn = a.mass_rows ? wb : wb / (mass_in + kEpsMass);
    acc[0] = 0.0 + wb;
    acc[1] = 0.0 + wn * wn;
    acc[2] = 0.0 + wout;
    acc[3] = 0.0 + H;
    rmax = fmax(rmax, rm);
  }
  block_sum<4>(acc, lds);
  rmax = block_max(rmax, lds);
  double v[5] = {acc[0], acc[1], acc[2], acc[3], rmax};
  store_partials<5>(v, partials, lb);
}

// ---------------------------------------------------------------- deterministic bucketing by nearest bin
// k_points took an arrival slot per point (atomic per-bucket counts).  k_scan: start[] =
// exclusive scan of the counts in one pass (decoupled look-back over 4096-bucket tiles, one
// wave reading 64 predecessors per step).  k_place scatters point indices by slot.
// k_bucket_rank ranks every bucket's members by point index (one lane per bucket up to
// kLaneRank members, the lane's wave for larger ones) into perm[], so perm lists each bucket's
// points contiguously in point-index order and the bin kernel visits them in a
// scheduling-independent order; it also marks the K candidate bins of every non-empty bucket
// active.
constexpr int kScanThreads = 256;
constexpr int kScanTile = 16 * kScanThreads;  // 16 counts per thread (4 x 16-B loads)
constexpr int kLaneRank = 16;
constexpr int kRankMax = 8192;
constexpr uint32_t kLbAgg = 1u << 30, kLbPre = 2u << 30, kLbVal = (1u << 30) - 1u;

__global__ __launch_bounds__(kScanThreads) void k_scan(const uint32_t* __restrict__ counts, int n, uint32_t* status,
                                                       uint32_t* ticket, uint32_t* start, uint32_t* err,
                                                       uint32_t spin_limit, int inject_fail) {
  constexpr int kSW = kScanThreads / 64;
  __shared__ uint32_t wsum[kSW];
  __shared__ uint32_t s_tile, s_excl;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) s_tile = atomicAdd(ticket, 1u);  // tiles are numbered in start order (forward progress)
  __syncthreads();
  const uint32_t tile = s_tile;
  const int base = (int)tile * kScanTile + 16 * t;
  uint32_t v[16];
  if (base + 16 <= n) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 u = *(const uint4*)(counts + base + 4 * q);
      v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (base + j < n) ? counts[base + j] : 0u;
  }
  uint32_t tot = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) tot += v[j];
  uint32_t x = tot;
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    uint32_t agg = 0;
    for (int w = 0; w < kSW; ++w) agg += wsum[w];
    uint32_t excl = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(status, kLbPre | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(status + tile, kLbAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // look back in windows of 64 predecessors: lane l reads tile (w0 - l)
      // On spin exhaustion the tile reports failure and continues with excl = 0: every start then
      // stays below the scan's point count, so k_place / k_bucket_rank / k_bins_scale index in
      // bounds (with wrong bucket ranges) and the host fails the scan from err[0].
      uint32_t spins = 0;
      bool failed = inject_fail && tile == 1;
      int w0 = failed ? -1 : (int)tile - 1;
      while (w0 >= 0) {
        const int j = w0 - lane;
        uint32_t s = j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbPre;
        // the window is usable up to (and including) its nearest published prefix
        const unsigned long long pre = __ballot((s & ~kLbVal) == kLbPre);
        const int stop = pre ? (__ffsll((long long)pre) - 1) : 63;
        const unsigned long long unpub = __ballot(s == 0u && lane <= stop);
        if (unpub) {  // bounded so a broken invariant cannot hang the GPU; the host fails the scan
          if (++spins > spin_limit) { excl = 0u; failed = true; break; }
          continue;
        }
        uint32_t val = (lane <= stop && j >= 0) ? (s & kLbVal) : 0u;
        for (int off = 32; off >= 1; off >>= 1) val += __shfl_xor(val, off, 64);
        excl += val;
        if (pre) break;
        w0 -= 64;
      }
      if (lane == 0) __hip_atomic_store(status + tile, kLbPre | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (failed && lane == 0) err[0] = 1u;  // vector store to host-mapped memory, checked by gcs_scan
    }
    if (lane == 0) {
      s_excl = excl;
      if (tile == gridDim.x - 1) atomicExch(ticket, 0u);  // every tile has drawn its number by now
    }
  }
  __syncthreads();
  uint32_t pre = s_excl + x - tot;
  for (int w = 0; w < wid; ++w) pre += wsum[w];
  uint32_t o[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    o[j] = pre;
    pre += v[j];
  }
  if (base + 16 <= n) {
#pragma unroll
    for (int q = 0; q < 4; ++q) *(uint4*)(start + base + 4 * q) = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (base + j < n) start[base + j] = o[j];
  }
}

__global__ __launch_bounds__(kBlock) void k_place(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ slots,
                                                  const uint32_t* __restrict__ start, int n, int n_bins,
                                                  uint32_t* slot_idx) {
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    uint32_t key = keys[i];
    if (key < (uint32_t)n_bins) slot_idx[start[key] + slots[i]] = (uint32_t)i;
  }
}

// One lane per bucket (grid covers all buckets exactly once).  Buckets of up to kLaneRank members
// are ranked in the lane's registers; larger ones are ranked afterwards by the whole wave (64
// members per step by shuffles), and above kRankMax by an in-order compaction over all keys (one
// wave, O(N): a degenerate case).  perm[start + rank] = point index.
__global__ __launch_bounds__(kBlock) void k_bucket_rank(BucketArgs b, int n) {
  const int a = blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t c = a < b.n_bins ? b.counts[a] : 0u;
  const uint32_t st = c ? b.starts[a] : 0u;
  if (c) {  // candidate bins active, and their k_bins_scale tiles (flags[n_bins + tile])
    const int* kr = b.knn + (size_t)a * b.k;
    uint8_t* tf = b.flags + b.n_bins;
    for (int q = 0; q < b.k; q += 4) {
      int4 c4 = *(const int4*)(kr + q);
      b.flags[c4.x] = 1; b.flags[c4.y] = 1; b.flags[c4.z] = 1; b.flags[c4.w] = 1;
      const int ts = b.tile_shift;
      tf[c4.x >> ts] = 1; tf[c4.y >> ts] = 1; tf[c4.z >> ts] = 1; tf[c4.w >> ts] = 1;
    }
  }
  if (c && c <= (uint32_t)kLaneRank) {
    const uint32_t* sl = b.slot_idx + st;
    uint32_t idx[kLaneRank];
#pragma unroll
    for (int j = 0; j < kLaneRank; ++j) idx[j] = (uint32_t)j < c ? sl[j] : 0xffffffffu;
#pragma unroll
    for (int j = 0; j < kLaneRank; ++j) {
      if ((uint32_t)j < c) {
        uint32_t r = 0;
#pragma unroll
        for (int q = 0; q < kLaneRank; ++q) r += idx[q] < idx[j] ? 1u : 0u;
        b.perm[st + r] = idx[j];
      }
    }
  }
  unsigned long long big = __ballot(c > (uint32_t)kLaneRank);
  while (big) {  // wave-cooperative ranking of this wave's large buckets, one at a time
    const int src = __ffsll((long long)big) - 1;
    big &= big - 1ull;
    const uint32_t cb = __shfl(c, src, 64), sb = __shfl(st, src, 64);
    const uint32_t ab = (uint32_t)__shfl(a, src, 64);
    if (cb <= (uint32_t)kRankMax) {
      for (uint32_t j0 = 0; j0 < cb; j0 += 64) {
        const uint32_t v = (j0 + lane < cb) ? b.slot_idx[sb + j0 + lane] : 0xffffffffu;
        uint32_t rank = 0;
        for (uint32_t k0 = 0; k0 < cb; k0 += 64) {
          const uint32_t u = (k0 + lane < cb) ? b.slot_idx[sb + k0 + lane] : 0xffffffffu;
          for (int jj = 0; jj < 64; ++jj) rank += (__shfl(u, jj, 64) < v) ? 1u : 0u;
        }
        if (j0 + lane < cb) b.perm[sb + rank] = v;
      }
    } else {
      if (lane == 0) b.err[1] = 1u;  // degenerate bucket: reported in the scan certificate
      uint32_t pos = sb;
      for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const bool hit = i < n && b.keys[i] == ab;
        const unsigned long long m = __ballot(hit);
        if (hit) b.perm[pos + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
        pos += (uint32_t)__popcll(m);
      }
    }
  }
}

// ---------------------------------------------------------------- bin finalize (shared)
// Raw sums layout (19): N, sd[3], S[xx,xy,xz,yy,yz,zz], sp[3], spp[xx,xy,xz,yy,yz,zz]
__device__ __forceinline__ void finalize_bin(const double* r, double* __restrict__ scan, int B, int b,
                                             double* cert /*5*/) {
  double N = r[0];
  double den = N + kEpsMass + kF64Eps;          // inv_mass_core, primitives.py:195-212
  double invN = rcp_fast(den);
  double epsr = kEpsMass * invN;
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
#if GCS_PROBE_NOFIN == 3  // timing probe: no PSD / kappa (the stores stay)
  double delta = 0.0;
  for (int k = 0; k < 9; ++k) sig[k] = sc[k];
  double kap = r[1];
#else
  double delta = psd_project3(sc, sig);
  double sn = sqrt(dot3_exact(r[1], r[2], r[3], r[1], r[2], r[3]));
  double kap = kappa_from_rbar(sn * invN);
#endif
  size_t Bs = (size_t)B;
#if GCS_PROBE_NOFIN == 2  // timing probe: the arithmetic without the 26 row stores
  if (delta == 12345.0) scan[b] = kap + sig[4];
  if (r[0] == 12345.0)
#endif
  {
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
  }
  cert[0] += N;
  cert[1] += N * N;
  cert[2] += N * rcp_fast(N + kEpsMass);
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
  cert[0] = v[0]; cert[1] = v[1]; cert[2] = v[2]; cert[3] = v[3]; cert[4] = mx;
}

// ---------------------------------------------------------------- row 7 helpers (Matrix-Fisher)
// Per bin (matrix_fisher_evidence.py:181-211): w_b = sqrt(N_s N_m + eps), u = S/(|S|+eps),
// conf = Rbar_s Rbar_m, H += w_b conf u_map u_scan^T; out[9] += w_b conf; out[10] += N_s.
struct MapDir {
  double Nm, mx, my, mz;  // map N_dir, S_dir of the bin
};
__device__ __forceinline__ MapDir load_map_dir(const double* __restrict__ map, int B, int b) {
  const size_t Bs = (size_t)B;
  return MapDir{map[MF_ND * Bs + b], map[MF_SD * Bs + b], map[(MF_SD + 1) * Bs + b], map[(MF_SD + 2) * Bs + b]};
}
__device__ __forceinline__ void mf_bin_term(double Ns, double sx, double sy, double sz, const MapDir& md,
                                            double* out /*11*/) {
  const double Nm = md.Nm, mx = md.mx, my = md.my, mz = md.mz;
  double wb = sqrt(Ns * Nm + kEpsMass);
  double sn = sqrt(dot3_exact(sx, sy, sz, sx, sy, sz));
  double mn = sqrt(dot3_exact(mx, my, mz, mx, my, mz));
  // four reciprocals for the eight divisions of the restatement (matrix_fisher_evidence.py:181-211)
  const double isn = rcp_fast(sn + kEpsMass), imn = rcp_fast(mn + kEpsMass);
  double us[3] = {sx * isn, sy * isn, sz * isn};
  double um[3] = {mx * imn, my * imn, mz * imn};
  double conf = (sn * rcp_fast(Ns + kEpsMass)) * (mn * rcp_fast(Nm + kEpsMass));
  double wf = wb * conf;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) out[3 * i + j] += wf * um[i] * us[j];
  out[9] += wf;
  out[10] += Ns;
}

// H (9), sum w conf, sum N_s -> scalars; the det-fixed R_mf = U diag(1,1,det(UV^T)) V^T
// (:215-222) on one thread (polar Newton, Jacobi SVD fallback: gcs_math.h mf_rotation).  The host
// recomputes the singular values / V it needs for L_rot from H.
__device__ void mf_finish(const double* v, double* scalars) {
  for (int k = 0; k < 9; ++k) scalars[SC_MF_H + k] = v[k];
  scalars[SC_MF_NEFF] = v[9];
  scalars[SC_MF_SCANN] = v[10];
  double R[9];
#if GCS_PROBE_NOPOLAR  // timing probe (not a parity build): R = I
  for (int k = 0; k < 9; ++k) R[k] = k % 4 == 0 ? 1.0 : 0.0;
#else
  mf_rotation(v, R);
#endif
  for (int k = 0; k < 9; ++k) scalars[SC_MF_R + k] = R[k];
}

// fused bin-kernel partial: [sum N, sum N^2, sum N/(N+eps), sum psd delta, max eps ratio | MF 11]
constexpr int kBinNV = 16;

// ---------------------------------------------------------------- row 5+6 scale mode: bin-centric
// One 256-thread workgroup per tile of TB consecutive device bins (a compact Hilbert patch of the
// sphere, gcs_atlas.h): TB = 64 with four lanes per bin.  TB = 32 with eight lanes per bin
// (GCSLAM_BIN_TILE=32) was measured at C2 and dropped: 1,019 active tiles no longer start together
// (a quarter start after 15 us), the gather phase did not shorten (5.7 vs 5.9 us with half the
// records per lane), and a tile over its 256-record stage took the unstaged path (69 us): kernel
// 69.7 vs 28.3 us.
//  0: a tile none of whose bins is a candidate of a non-empty bucket (tile flag, set by
//     k_bucket_rank) has exact-zero sums: wave 0 writes the zero-bin rows and the tile's partial
//     row in closed form; A-D are skipped.  With the VLP-16-like scans (rings within +-15 deg)
//     most tiles of the sphere are such.  A per-tile dirty byte (persistent across scans) records
//     whether the tile's rows and partial row differ from those zero-bin values: a tile inactive
//     in this scan and the last one exits without writing (its output is already in place).
//  A: the tile's bin directions, reverse-kNN ranges and local source indices go to LDS; the
//     tile's unique source buckets (host table, ~2.3 per bin) get sizes, starts and staged
//     offsets (block scan); each bin's work (records to visit) is summed.
//  B: the sources' records, which each bin of the tile reads ~K/2.3 times, are staged once into
//     LDS (64 B: p, d, m, w/Z); a tile with more than STAGE records reads them from HBM/L2.
//  C: LANES lanes per bin accumulate the bin's records in fixed order (the bin's sources in
//     ascending bucket id, each source's points in ascending index, as one flattened list; lane l
//     takes the l-th share; a fixed xor tree) -- LDS traffic only.  LANES = 4 for both scan
//     densities.  (LANES = 8, 512-thread workgroups, was measured at C2: the active tile's life
//     fell 23 -> 20 us, but at 122 VGPRs only two such workgroups fit a CU, the 540 active tiles
//     no longer started together and the kernel went 32 -> 40 us.)  (Work-proportional lane groups
//     were measured slower: the group bookkeeping and the deeper shuffle trees cost more than the
//     balance bought back)
//  D: wave 0, one lane per bin: PSD, kappa, the bin's Matrix-Fisher term, coalesced 64-bin output
//     rows, the tile's partial row by a wave reduction.
// STAGE: kStageBig when the scan is dense in the map (cap >= 0.4 B, C2: 41 KiB of LDS, three
// workgroups per CU), kStageSmall otherwise (C3: 25 KiB; four per CU, register-limited).
// per-tile table capacities, proportional to the tile: for 64-bin tiles 320 sources (the atlas tables
// for B = 1k .. 1M have at most 199) and 1280 reverse-kNN entries (~K x 64; at most 1070)
__host__ __device__ constexpr int max_src(int tb) { return 5 * tb; }
__host__ __device__ constexpr int max_rl(int tb) { return 20 * tb; }
#ifndef GCS_STAGE_BIG
#define GCS_STAGE_BIG 512  // 480 (four workgroups per CU in LDS instead of three) measured slower at C2: 27.2 -> 30.5 us
#endif
constexpr int kStageBig = GCS_STAGE_BIG, kStageSmall = 256;
// record stages of the wider tiles (LDS per workgroup: tables + stage x 64 B)
#ifndef GCS_STAGE_128_BIG
#define GCS_STAGE_128_BIG 768
#endif
#ifndef GCS_STAGE_128_SMALL
#define GCS_STAGE_128_SMALL 320
#endif
#ifndef GCS_STAGE_256_BIG
#define GCS_STAGE_256_BIG 1024
#endif
#ifndef GCS_STAGE_256_SMALL
#define GCS_STAGE_256_SMALL 640
#endif
#ifndef GCS_DALL64
#define GCS_DALL64 false  // 64-bin tiles: phase D on wave 0 (every wave measured slower in round 1)
#endif
#ifndef GCS_DALL128
#define GCS_DALL128 false  // 128-bin tiles: phase D on waves 0-1, one lane per bin (true: on every wave)
#endif
constexpr int kStage128Big = GCS_STAGE_128_BIG, kStage128Small = GCS_STAGE_128_SMALL;
constexpr int kStage256Big = GCS_STAGE_256_BIG, kStage256Small = GCS_STAGE_256_SMALL;
// staged record: x y z dx dy dz m w/Z as four double2 chunks (+ GCS_REC_PAD doubles of stride
// padding); GCS_REC_SWZ stores chunk c of record r at slot c ^ ((r >> 2) & 3) (LDS bank spread)
#ifndef GCS_REC_PAD
#define GCS_REC_PAD 0
#endif
#ifndef GCS_REC_SWZ
#define GCS_REC_SWZ 1  // A/B at C2: 33.0 -> 31.0 us; C3 unchanged (LDS conflicts are ~1/3 of LDS cycles)
#endif
constexpr int kRecD = 8 + GCS_REC_PAD;
__device__ __forceinline__ uint32_t rec_swz(uint32_t r) { return GCS_REC_SWZ ? ((r >> 2) & 3u) : 0u; }
int bins_max_tile_sources(int tile_bins) { return max_src(tile_bins); }
int bins_max_tile_entries(int tile_bins) { return max_rl(tile_bins); }

// ray_dir (gcs_math.h) with its three divisions issued one after another: the same operations, so the
// same bits, for the rare unstaged gather, whose loop otherwise set the kernel's register peak
__device__ __forceinline__ void ray_dir_serial(double px, double py, double pz, const double* o, double* d) {
#pragma clang fp contract(off)
  const double rx = px - o[0], ry = py - o[1], rz = pz - o[2];
  const double den = sqrt(dot3_exact(rx, ry, rz, rx, ry, rz)) + kEpsMass;
  d[0] = rx / den;
  __builtin_amdgcn_sched_barrier(0);
  d[1] = ry / den;
  __builtin_amdgcn_sched_barrier(0);
  d[2] = rz / den;
}

__device__ __forceinline__ void bin_contrib(double* acc, const double3& bd, double inv_tau, double px, double py,
                                            double pz, double dx, double dy, double dz, double m, double wz) {
  double d[3] = {dx, dy, dz};
  double p[3] = {px, py, pz};
  double sim = dot3_exact(dx, dy, dz, bd.x, bd.y, bd.z);
  // w r = w exp((s - m)/tau) / Z   (binning.py:69 softmax, :159-160 weighting)
#if GCS_PROBE_NOEXP  // timing probe (not a parity build): the exp's share of the gather
  add_contrib(acc, wz * fmax(1.0 + (sim - m) * inv_tau, 1e-3), d, p);
#else
  add_contrib(acc, wz * exp((sim - m) * inv_tau), d, p);
#endif
}

#ifdef GCS_PHASE_PROF
__device__ unsigned long long g_prof[32768 * 16];
extern "C" int gcs_debug_prof(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), (size_t)n * sizeof(unsigned long long));
}
extern "C" int gcs_debug_psd_count(unsigned long long* out /*4*/, int reset) {
  int e = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_psd_count), 4 * sizeof(unsigned long long));
  if (reset) {
    unsigned long long z[4] = {0, 0, 0, 0};
    e |= (int)hipMemcpyToSymbol(HIP_SYMBOL(g_psd_count), z, sizeof(z));
  }
  return e;
}
#define PROF(k) \
  if (threadIdx.x == 0) g_prof[blockIdx.x * 16 + (k)] = wall_clock64();
#define PROFV(k, v) \
  if (threadIdx.x == 0) g_prof[blockIdx.x * 16 + (k)] = (unsigned long long)(v);
#else
#define PROF(k)
#define PROFV(k, v)
#endif

// Wave 0's reduction of the per-bin cert / Matrix-Fisher terms into the tile's partial row:
// [sum N, sum N^2, sum N/(N+eps), sum psd delta, max eps ratio | MF 11] (fixed xor tree).
__device__ __forceinline__ void wave_reduce_bin_terms(double (&v)[kBinNV]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int k = 0; k < kBinNV; ++k) {
      const double y = __shfl_xor(v[k], off, 64);
      v[k] = k == 4 ? fmax(v[k], y) : v[k] + y;
    }
}

#ifndef GCS_RANK_LANES
#define GCS_RANK_LANES 4  // phase A's per-bin work sum + source compaction: 4 lanes per bin (1: wave 0 alone)
#endif
#ifndef GCS_UNSTAGED_IDX
#define GCS_UNSTAGED_IDX 1  // direct buckets, tile over its record stage: stage point indices (phase B)
#endif
#ifndef GCS_GATHER_PIPE
// phase C: 1 loads the next staged record while accumulating the current one; 2 takes two
// records per trip (two independent exp chains in flight)
#define GCS_GATHER_PIPE 2
#endif
#ifndef GCS_STAGE_SERIAL
#define GCS_STAGE_SERIAL 1  // phase B expands its staged 32-B records one after another (register peak)
#endif
#ifndef GCS_MAPV_EARLY
#define GCS_MAPV_EARLY 1  // phase D's map direction stats are loaded before phase A
#endif
#ifndef GCS_BINS_WAVES
#define GCS_BINS_WAVES 0  // waves per SIMD the register allocation targets (0: compiler default)
#endif
#ifndef GCS_BINS_WAVES_SMALL
// the small-stage instantiation (C3: 25 KiB of LDS, six workgroups per CU by LDS) is register-bound:
// 5 waves per SIMD needs <= 96 VGPRs (the register allocator spills ~28 dwords to reach it)
#define GCS_BINS_WAVES_SMALL 0
#endif
#ifndef GCS_GATHER_BAL
// phase C's lanes (tiles finalized by the first waves, !DALL): bin tiles of at least GCS_GATHER_BAL bins
// give each bin of a wave a lane group sized by its records (balanced), smaller ones the fixed LANES
// lanes per bin of rounds 1-4.  Same box, alternated (profiles/r05/bal/): C3 (128-bin tiles) bins
// 84.6-85.3 -> 82.3-82.7 us; C2 (64-bin tiles) 26.9 -> 28.5-28.9 us, so 128 (0: never).
#define GCS_GATHER_BAL 128
#endif
// Balanced phase-C lanes.  Wave wid gathers the bins [wid BW, wid BW + BW) (BW = 64 / LANES, the fixed
// partition of rounds 1-4), but the 64 lanes are dealt by work: with W records and nz non-empty bins
// in the wave and c = ceil(W / (64 - nz)), bin b gets cnt_b = ceil(w_b / c) contiguous lanes (sum <= 64:
// ceil(w_b / c) < w_b / c + 1), so no lane visits more than c records (the fixed split let the
// heaviest bin's lanes visit w_max / LANES: C2 55 / 4 against a balanced 10, C3 50 / 2 against 12).
// Lane j of a group takes records [w_b j / cnt_b, w_b (j + 1) / cnt_b) of the bin's list; the group's
// sums meet in a fixed segmented tree (seg_reduce), so the result is deterministic.  All integer,
// wave-uniform control; lanes past the last group idle (lb valid, empty range).
template <int LANES>
__device__ __forceinline__ void balanced_lanes(const uint32_t* s_work, int wid, int lane, int& lb, uint32_t& i0,
                                               uint32_t& i1, int& j, int& cnt_b, int& maxl) {
  constexpr int BW = 64 / LANES;
  const uint32_t wk = lane < BW ? s_work[wid * BW + lane] : 0u;
  uint32_t W = wk, nz = wk ? 1u : 0u;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    W += (uint32_t)__shfl_xor((int)W, off, 64);
    nz += (uint32_t)__shfl_xor((int)nz, off, 64);
  }
  const uint32_t avail = 64u - nz;
  const uint32_t c = avail ? (W + avail - 1u) / avail : 0u;
  const uint32_t cnt = wk ? (avail ? (wk + c - 1u) / c : 1u) : 0u;
  uint32_t incl = cnt, mx = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
    if (lane >= off) incl += y;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  maxl = (int)mx;
  const uint32_t used = (uint32_t)__shfl((int)incl, BW - 1, 64);
  // the lane's bin: the smallest b with incl_b > lane (incl is non-decreasing over b)
  int b = 0;
#pragma unroll
  for (int bit = BW >> 1; bit >= 1; bit >>= 1) {
    const uint32_t v = (uint32_t)__shfl((int)incl, b + bit - 1, 64);
    if (v <= (uint32_t)lane) b += bit;
  }
  const uint32_t inc_b = (uint32_t)__shfl((int)incl, b, 64);
  const uint32_t cn_b = (uint32_t)__shfl((int)cnt, b, 64);
  const uint32_t wk_b = (uint32_t)__shfl((int)wk, b, 64);
  lb = wid * BW + b;
  if ((uint32_t)lane >= used) {  // idle lane
    j = 0;
    cnt_b = 0;
    i0 = i1 = 0u;
    return;
  }
  j = lane - (int)(inc_b - cn_b);
  cnt_b = (int)cn_b;
  i0 = wk_b * (uint32_t)j / cn_b;
  i1 = wk_b * (uint32_t)(j + 1) / cn_b;
}
// the lane groups' sums in a fixed tree: ((s0 + s1) + (s2 + s3)) + ..., the result in the group's lane 0
template <int NF>
__device__ __forceinline__ void seg_reduce(double (&acc)[NF], int j, int cnt_b, int maxl) {
  for (int off = 1; off < maxl; off <<= 1) {
    const bool take = (j & (2 * off - 1)) == 0 && j + off < cnt_b;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const double y = __shfl_down(acc[f], off, 64);
      if (take) acc[f] += y;
    }
  }
}

// Self-budget scans (BinKernelArgs.mass_rows): the budget's mass sums from k_points' per-block rows.
// Thread t sums rows t, t + NT, ... in order, a fixed xor tree sums the wave, and mass_totals adds the
// waves in order -- every block of the launch gets the same bits (point_budget.py:80-84).
template <int NT>
__device__ __forceinline__ double2 mass_rows_wave(const double2* __restrict__ rows, int n) {
  double sx = 0.0, sy = 0.0;
  for (int r0 = 0; r0 < n; r0 += 4 * NT) {
    double2 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = r0 + (int)threadIdx.x + k * NT;
      x[k] = r < n ? rows[r] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sx += x[k].x;
      sy += x[k].y;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    sx += __shfl_xor(sx, off, 64);
    sy += __shfl_xor(sy, off, 64);
  }
  return make_double2(sx, sy);
}
// mass_rows_wave with its first chunk (rows t + k NT, k < 4) already loaded into x0: the same sums in the
// same order, so every block's mass_scale is bit for bit block 0's
template <int NT>
__device__ __forceinline__ double2 mass_rows_wave_pre(const double2* __restrict__ rows, int n, const double2 (&x0)[4]) {
  double sx = 0.0, sy = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sx += x0[k].x;
    sy += x0[k].y;
  }
  for (int r0 = 4 * NT; r0 < n; r0 += 4 * NT) {
    double2 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = r0 + (int)threadIdx.x + k * NT;
      x[k] = r < n ? rows[r] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sx += x[k].x;
      sy += x[k].y;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    sx += __shfl_xor(sx, off, 64);
    sy += __shfl_xor(sy, off, 64);
  }
  return make_double2(sx, sy);
}

template <int NW>
__device__ __forceinline__ double mass_scale_of(const double2* s_mw, double* m_in = nullptr, double* m_sel = nullptr) {
  double mi = s_mw[0].x, ms = s_mw[0].y;
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    mi += s_mw[w].x;
    ms += s_mw[w].y;
  }
  if (m_in) *m_in = mi;
  if (m_sel) *m_sel = ms;
  return mi / (ms + kEpsMass);  // mass_scale (point_budget.py:80-84)
}

// DALL: phase D on every wave -- the first lane of each bin's lane group finalizes the bin from its
// registers right after the lanes' xor tree (no LDS hand-off, no idle waves); required for tiles
// wider than one wave (TB > 64).  !DALL: wave 0 alone, one lane per bin (the 64-bin tile's form).
// SPLIT (sparse maps, 128-bin tiles): phases 0 and A-C only -- each active bin's 19 raw sums go to a.raw
// and k_bins_finalize runs phase D one thread per bin at full occupancy (the two-wave serial phase D held
// the tile's workgroup, its LDS and its registers; the gather's register peak is lower without it).
template <int STAGE, int TB, int LANES, bool DALL, bool SPLIT = false>
__global__ __launch_bounds__(TB * LANES)
#if GCS_BINS_WAVES
__attribute__((amdgpu_waves_per_eu(GCS_BINS_WAVES)))
#elif GCS_BINS_WAVES_SMALL
__attribute__((amdgpu_waves_per_eu(STAGE == kStageSmall ? GCS_BINS_WAVES_SMALL : 1)))
#endif
void k_bins_scale(BinKernelArgs a, double* partials) {
  constexpr int NT = TB * LANES, NW = NT / 64;
  constexpr int kMaxSrc = max_src(TB), kMaxRl = max_rl(TB);
  static_assert(LANES == 1 || LANES == 2 || LANES == 4 || LANES == 8, "phase C splits each bin over 1-8 lanes");
  static_assert(DALL || TB <= 64 || (TB % 64 == 0 && TB <= NT), "phase D on the first TB / 64 waves: one lane per bin");
  static_assert(DALL || STAGE * kRecD >= 19 * TB, "phase D reuses the record stage for the bin sums");
  __shared__ uint32_t s_cnt[kMaxSrc], s_off[kMaxSrc], s_st[kMaxSrc];
  __shared__ double s_rec[STAGE * kRecD];
#if GCS_RANK_LANES == 4
  // the raw reverse-kNN list is dead once phase A has compacted it, before phase B stages the
  // records: it lives in the record stage (2.5 KiB less LDS per workgroup)
  static_assert(kMaxRl * sizeof(uint16_t) <= STAGE * kRecD * sizeof(double), "raw list fits the stage");
  uint16_t* const s_rl = reinterpret_cast<uint16_t*>(s_rec);
  __shared__ uint16_t s_rlc[kMaxRl];  // each bin's non-empty sources, compacted (phase C's list)
  __shared__ uint8_t s_act[TB];
  uint16_t* const rlist = s_rlc;
#else
  static_assert(!DALL, "the wave-0 work sum assumes TB <= 64");
  __shared__ uint16_t s_rl[kMaxRl];
  uint16_t* const rlist = s_rl;
#endif
  __shared__ double4 s_bd[TB];
  __shared__ int s_q[TB + 1];
  __shared__ uint32_t s_work[TB];
  __shared__ uint32_t s_wsum[NW];
  __shared__ double lds[NW * 16];
  // the LiDAR origin for the staging's ray directions, from LDS: as kernel-argument SGPRs live through
  // the phases it pushed the kernel past its scalar registers (spilled to a VGPR lane: 3 waves / SIMD)
  __shared__ double s_org[3];
  __shared__ double2 s_mw[NW];  // self-budget: the waves' mass-row sums
  __shared__ double s_msc;      // self-budget: mass_scale (thread 0, after phase A's first barrier)
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // dispatch order: the previous scan's active tiles first, heaviest first (k_tile_order), so the
  // multi-round C3 grid starts its long tiles early and ends on clean ones; identity if null
  const int tile = a.tile_order ? a.tile_order[blockIdx.x] : (int)blockIdx.x;
  const int b0 = tile * TB;
  const int nb = min(TB, a.n_bins - b0);
  PROF(0);
  for (int j = blockIdx.x * NT + t; j < a.n_zero_after; j += gridDim.x * NT) a.zero_after[j] = 0u;
  if (blockIdx.x == 0 && (a.pts_partials || a.mass_rows)) {  // k_points' cert partials (off the critical path here)
    double pv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    if (a.pts_partials) reduce_partials<5, 16u, NT>(a.pts_partials, a.pts_blocks, pv, lds);
    if (a.mass_rows) {  // self-budget: the budget scalars, and the raw cert sums scaled by mass_scale
      const double2 ws = mass_rows_wave<NT>(a.mass_rows, a.mass_nrows);
      if (lane == 0) s_mw[wid] = ws;
      __syncthreads();
      if (t == 0) {
        double m_in, m_sel;
        const double msc = mass_scale_of<NW>(s_mw, &m_in, &m_sel);
        a.scalars[SC_MASS_IN] = m_in;
        a.scalars[SC_MASS_SEL] = m_sel;
        a.scalars[SC_MASS_SCALE] = msc;
        const double q = msc / (m_in + kEpsMass);  // w_budget / (mass_in + eps) = q w
        pv[0] *= msc;      // sum w_budget
        pv[1] = pv[1] * q * q;  // sum (w_budget / (mass_in + eps))^2
        pv[2] *= msc;      // sum w_out
      }
      __syncthreads();  // (phase A rewrites s_mw with the same values)
    }
    if (t == 0 && a.pts_partials)
      for (int f = 0; f < 5; ++f) a.scalars[SC_DESKEW_WIN + f] = pv[f];
  }
  // the tile flags and phase A's first-level table loads are issued together
  const bool tile_active = a.flags[a.n_bins + tile] != 0;  // block-uniform
  const bool tile_dirty = a.tile_dirty[tile] != 0;
  const int q_t = t < nb ? a.rknn_off[b0 + t] : 0;
  const int q0 = a.rknn_off[b0], q1t = a.rknn_off[b0 + nb];
  const int s0 = a.tile_src_off[tile];
  const int ns = a.tile_src_off[tile + 1] - s0;
  if (!tile_active && !tile_dirty) {
    PROF(6);
    PROFV(7, 2);
    return;
  }
  // every wave reads the tile's dirty word itself (with phase A's loads): an inactive tile's is cleared
  // only after the barrier below, which every wave of such a tile reaches -- a clear before another
  // wave's read sent that wave out through the clean-tile return above, leaving its 64 bins' rows
  // unwritten (stale rows of the previous scan, or the allocation's zeros: the run-to-run differences
  // of tools/determinism_check.py at C3, and the one C3 parity failure of round 6)
  if (t == 0 && tile_active && !tile_dirty) a.tile_dirty[tile] = 1;
  if (!tile_active) {
    __syncthreads();
    if (t == 0) a.tile_dirty[tile] = 0;
    // every bin of the tile has exact-zero sums: the zero-bin finalize writes its rows (N = 0,
    // Sigma = eps I, ...); partial row = nb x the zero bin's terms, no MF term
    if (DALL || t < TB) {
      double z[19], c5[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
#pragma unroll
      for (int f = 0; f < 19; ++f) z[f] = 0.0;
      if (t < nb) finalize_bin(z, a.scan, a.n_bins, b0 + t, c5);
      if (t == 0) {  // every zero bin has the same terms: the partial row is nb x thread 0's
        double v[kBinNV];
#pragma unroll
        for (int f = 0; f < kBinNV; ++f) v[f] = 0.0;
        v[3] = (double)nb * c5[3];
        v[4] = c5[4];
        store_partials<kBinNV>(v, partials, tile);  // folded by k_final<FIN_BINS>
      }
    }
    PROF(6);
    PROFV(7, 0);
    return;
  }
  // phase D's bin (wave 0: thread t < nb owns bin b0 + t; DALL: lane 0 of the bin's lane group owns
  // bin b0 + t / LANES): flag and map direction stats up front
  const int own_b = DALL ? t / LANES : t;
  const bool own = DALL ? (t % LANES == 0 && own_b < nb) : t < nb;
  const bool act_t = t < nb && a.flags[b0 + t];  // bin b0 + t (the phase-A rank's table)
  const bool own_act = DALL ? own && a.flags[b0 + own_b] : act_t;
  MapDir mapv{0.0, 0.0, 0.0, 0.0};
  if (GCS_MAPV_EARLY && !SPLIT && own_act) mapv = load_map_dir(a.map, a.n_bins, b0 + own_b);
  // phase A
  if (t < nb) s_bd[t] = *(const double4*)(a.bin_dirs + 4 * (size_t)(b0 + t));
  if (t < 3) s_org[t] = a.origin[t];
  if (t < nb) s_q[t] = q_t;
  if (t == 0) s_q[nb] = q1t;
#if GCS_RANK_LANES == 4
  if (t < TB) s_act[t] = act_t ? 1 : 0;
#endif
  {
    // fixed trip counts: every thread issues all of its table loads before the first LDS write,
    // so the reverse-kNN entries (up to kMaxRl / NT per thread) cost one round trip, not one each,
    // and the sources two (tile_src, then their counts / starts).  Self-budget: the mass rows' first
    // chunk is loaded first and summed after the LDS writes (its round trip hidden behind the tables')
    constexpr int RL = (kMaxRl + NT - 1) / NT, SR = (kMaxSrc + NT - 1) / NT;
    double2 mw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = t + k * NT;
      const bool ok = a.mass_rows && r < a.mass_nrows;
      mw[k] = ok ? (GCS_PROBE_NOMASS ? make_double2(1.0, 1.0) : a.mass_rows[r]) : make_double2(0.0, 0.0);
    }
    uint16_t rl[RL];
#pragma unroll
    for (int k = 0; k < RL; ++k) {
      const int q = q0 + t + k * NT;
      rl[k] = q < q1t ? a.rknn_local[q] : (uint16_t)0;
    }
    int src[SR];
#pragma unroll
    for (int k = 0; k < SR; ++k) src[k] = t + k * NT < ns ? a.tile_src[s0 + t + k * NT] : 0;
    uint32_t cn[SR], st[SR];
#pragma unroll
    for (int k = 0; k < SR; ++k) {
      cn[k] = t + k * NT < ns ? a.counts[src[k]] : 0u;
      if (a.members) cn[k] = min(cn[k], (uint32_t)a.capb);  // an overflowing scan is redone (rows in bounds)
      // sorted bucketing: the bucket's start in perm; direct buckets: its member row
      st[k] = t + k * NT < ns ? (a.members ? (uint32_t)src[k] * (uint32_t)a.capb : a.starts[src[k]]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < RL; ++k)
      if (q0 + t + k * NT < q1t) s_rl[t + k * NT] = rl[k];
#pragma unroll
    for (int k = 0; k < SR; ++k)
      if (t + k * NT < ns) {
        s_cnt[t + k * NT] = cn[k];
        s_st[t + k * NT] = st[k];
      }
    if (a.mass_rows) {
      const double2 ws = mass_rows_wave_pre<NT>(a.mass_rows, a.mass_nrows, mw);
      if (lane == 0) s_mw[wid] = ws;
    }
  }
  __syncthreads();
  PROF(1);
  if (a.mass_rows && t == 0) s_msc = mass_scale_of<NW>(s_mw);  // (read after the next barrier)
#if GCS_RANK_LANES == 4
  {
    // Records each bin visits (0: inactive / out of range), on the bin's four phase-C lanes: lane l
    // takes the l-th quarter of the bin's reverse-kNN entries; the non-empty sources are written,
    // in order, to the compacted list s_rlc (offsets by a prefix over the four lanes), so phase C's
    // cursor never walks an empty bucket (each visit was two dependent LDS reads).
    const int rb = t / LANES, rq = t % LANES;
    int qa = 0, lo = 0, hi = 0;
    if (s_act[rb]) {
      qa = s_q[rb] - q0;
      const int n = s_q[rb + 1] - q0 - qa;
      lo = qa + n * rq / LANES;
      hi = qa + n * (rq + 1) / LANES;
    }
    uint32_t w = 0;
    int nz = 0;
    for (int q = lo; q < hi; q += 4) {
      uint16_t j[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) j[u] = q + u < hi ? s_rl[q + u] : (uint16_t)0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t c = q + u < hi ? s_cnt[j[u]] : 0u;
        w += c;
        nz += c ? 1 : 0;
      }
    }
    int x = nz;
#pragma unroll
    for (int off = 1; off < LANES; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (rq >= off) x += y;
    }
    int e = qa + (x - nz);
    for (int q = lo; q < hi; q += 4) {
      uint16_t j[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) j[u] = q + u < hi ? s_rl[q + u] : (uint16_t)0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q + u < hi && s_cnt[j[u]]) s_rlc[e++] = j[u];
    }
#pragma unroll
    for (int off = 1; off < LANES; off <<= 1) w += (uint32_t)__shfl_xor((int)w, off, 64);
    if (rq == 0) s_work[rb] = w;
  }
#else
  if (t < TB) {  // wave 0, lane = bin: records each bin visits (0: inactive / out of range)
    // The bin's reverse-kNN sources are compacted in place to the non-empty ones (same order):
    // most sources of a bin are empty buckets, and phase C's cursor then never walks them (each
    // visit was two dependent LDS reads).  Entries are read four at a time ahead of the writes
    // (a write never passes a read: e <= q).
    uint32_t w = 0;
    int e = s_q[t] - q0;
    if (own_act) {
      const int qa = s_q[t] - q0, qb = s_q[t + 1] - q0;
      for (int q = qa; q < qb; q += 4) {
        uint16_t j[4];
        uint32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) j[u] = q + u < qb ? s_rl[q + u] : (uint16_t)0;
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = q + u < qb ? s_cnt[j[u]] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (c[u]) {
            s_rl[e++] = j[u];
            w += c[u];
          }
      }
    }
    s_work[t] = w;
  }
#endif
  const int chunk = (ns + NT - 1) / NT;
  const int j0 = min(ns, t * chunk), j1 = min(ns, j0 + chunk);
  uint32_t mine = 0;
  for (int j = j0; j < j1; ++j) mine += s_cnt[j];
  uint32_t x = mine;
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  uint32_t run = x - mine;
  for (int w = 0; w < wid; ++w) run += s_wsum[w];
  for (int j = j0; j < j1; ++j) {
    s_off[j] = run;
    run += s_cnt[j];
  }
  uint32_t total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) total += s_wsum[w];
  const bool staged = total <= (uint32_t)STAGE;
  if (t == 0 && a.tile_work) a.tile_work[tile] = total;  // k_tile_order's weight for the next scan
  PROFV(8, total);
#ifdef GCS_PHASE_PROF
  if (t == 0) {
    uint32_t mx = 0, sm = 0;
    for (int i = 0; i < TB; ++i) { mx = max(mx, s_work[i]); sm += s_work[i]; }
    g_prof[blockIdx.x * 16 + 9] = mx;
    g_prof[blockIdx.x * 16 + 10] = sm;
  }
#endif
  __syncthreads();
  PROF(2);
  // phase B: stage the tile's records (record r belongs to the last source with s_off <= r)
  if (staged) {
    // at most RPT records per thread: every perm load is issued before any record load, so a
    // tile with more records than threads still pays two dependent round trips, not 2 x RPT
    constexpr int RPT = (STAGE + NT - 1) / NT;
    uint32_t pi[RPT], dst[RPT], sid[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint32_t r = t + k * NT;
      pi[k] = 0u;
      dst[k] = r;
      sid[k] = 0u;
      if (r < total) {
        int lo = 0, hi = ns - 1;
        while (lo < hi) {
          int mid = (lo + hi + 1) >> 1;
          if (s_off[mid] <= r) lo = mid; else hi = mid - 1;
        }
        sid[k] = (uint32_t)a.tile_src[s0 + lo];  // (L2: phase A read the list; no LDS for it)
        const uint32_t pos = s_st[lo] + (r - s_off[lo]);
        if (a.members) {
          // direct buckets hold arrival order: the record's slot is its source's offset + the rank
          // of its point index among the source's members (the sorted bucketing's order, bit for bit)
          const uint32_t c = s_cnt[lo];
          const uint4* row = (const uint4*)(a.members + s_st[lo]);
          const uint32_t me = a.members[pos];
          uint32_t rank = 0;
          for (uint32_t q = 0; q < c; q += 4) {
            const uint4 m4 = row[q >> 2];
            rank += (m4.x < me) + (q + 1 < c && m4.y < me) + (q + 2 < c && m4.z < me) + (q + 3 < c && m4.w < me);
          }
          pi[k] = me;
          dst[k] = s_off[lo] + rank;
        } else {
          pi[k] = a.perm[pos];
        }
      }
    }
    // the 32-B records and their sources' directions in one round trip; each staged record is then
    // expanded to the 64-B LDS form: d = ray_dir(p), m = d . dir(source) (gcs_layout.h PointRec32)
    const double4* recs4 = reinterpret_cast<const double4*>(a.recs);
    double4 pr[RPT];
    double3 sd[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k)
      if (t + k * NT < total) {
        pr[k] = recs4[pi[k]];
        const double* sp = a.bin_dirs + 4 * (size_t)sid[k];
        const double2 xy = *(const double2*)sp;
        sd[k] = make_double3(xy.x, xy.y, sp[2]);
      }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint32_t r = dst[k];
      if (t + k * NT < total) {
        double dd[3];
        ray_dir(pr[k].x, pr[k].y, pr[k].z, s_org, dd);
        const double m = dot3_exact(dd[0], dd[1], dd[2], sd[k].x, sd[k].y, sd[k].z);
        double2* d = (double2*)(s_rec + (size_t)r * kRecD);
        const uint32_t sw = rec_swz(r);
        d[0 ^ sw] = make_double2(pr[k].x, pr[k].y);
        d[1 ^ sw] = make_double2(pr[k].z, dd[0]);
        d[2 ^ sw] = make_double2(dd[1], dd[2]);
        d[3 ^ sw] = make_double2(m, pr[k].w);
      }
      if (GCS_STAGE_SERIAL) __builtin_amdgcn_sched_barrier(0);  // one record's expansion at a time (registers)
    }
  }
#if GCS_UNSTAGED_IDX
  // a tile over its record stage with direct buckets: stage the records' point indices instead (4 B
  // each, in the stage's memory), ranked by point index within each source as above, so phase C
  // gathers records from L2 without re-ranking members per record
  const bool idx_staged = !staged && a.members && total <= (uint32_t)(STAGE * kRecD * 2);
  if (idx_staged) {
    uint32_t* s_idx = reinterpret_cast<uint32_t*>(s_rec);
    for (uint32_t r = t; r < total; r += NT) {
      int lo = 0, hi = ns - 1;
      while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= r) lo = mid; else hi = mid - 1;
      }
      const uint32_t c = s_cnt[lo];
      const uint4* row = (const uint4*)(a.members + s_st[lo]);
      const uint32_t me = a.members[s_st[lo] + (r - s_off[lo])];
      uint32_t rank = 0;
      for (uint32_t q = 0; q < c; q += 4) {
        const uint4 m4 = row[q >> 2];
        rank += (m4.x < me) + (q + 1 < c && m4.y < me) + (q + 2 < c && m4.z < me) + (q + 3 < c && m4.w < me);
      }
      s_idx[s_off[lo] + rank] = me;
    }
  }
#else
  constexpr bool idx_staged = false;
#endif
  __syncthreads();
  PROF(3);
  // phase C: four lanes per bin; the bin's records (sources in order, points in order) are one
  // flattened list and lane l takes the l-th quarter, so every lane's trip count is its own share
  // (no per-source max over the wave's lanes).
  constexpr bool BAL = GCS_GATHER_BAL && TB >= GCS_GATHER_BAL && !DALL;
  int lb, l, seg_j = 0, seg_n = 0, seg_max = 1;
  uint32_t i0, i1;
  if constexpr (BAL) {
    l = 0;
    balanced_lanes<LANES>(s_work, wid, lane, lb, i0, i1, seg_j, seg_n, seg_max);
  } else {
    lb = t / LANES;
    l = t % LANES;
    const uint32_t work = s_work[lb];
    i0 = work * (uint32_t)l / (uint32_t)LANES;
    i1 = work * (uint32_t)(l + 1) / (uint32_t)LANES;
  }
  double acc[19];
#pragma unroll
  for (int f = 0; f < 19; ++f) acc[f] = 0.0;
  if (i1 > i0) {
    const double3 bd = make_double3(s_bd[lb].x, s_bd[lb].y, s_bd[lb].z);  // (not the pad: registers)
    const double inv_tau = 1.0 / a.tau;
    // cursor: source q (local j), record k within it
    int q = s_q[lb];
    uint32_t skip = i0;
    int j = rlist[q - q0];
    uint32_t c = s_cnt[j];
    while (skip >= c) {
      skip -= c;
      ++q;
      j = rlist[q - q0];
      c = s_cnt[j];
    }
    uint32_t kk = skip;
    if (staged && !GCS_GATHER_PIPE) {
      uint32_t r = s_off[j] + kk, left = c - kk;
      for (uint32_t i = i0; i < i1; ++i) {
        const double2* rp = (const double2*)(s_rec + (size_t)r * kRecD);
        const uint32_t sw = rec_swz(r);
        const double2 c0 = rp[0 ^ sw], c1 = rp[1 ^ sw], c2 = rp[2 ^ sw], c3 = rp[3 ^ sw];
        bin_contrib(acc, bd, inv_tau, c0.x, c0.y, c1.x, c1.y, c2.x, c2.y, c3.x, c3.y);
        if (--left == 0 && i + 1 < i1) {  // next source (compacted: non-empty)
          ++q;
          j = rlist[q - q0];
          left = s_cnt[j];
          r = s_off[j];
        } else {
          ++r;
        }
      }
    } else if (staged && GCS_GATHER_PIPE == 2) {
      // two records per trip: both records' dot / exp chains are independent, so they issue
      // interleaved (the exp chain, not the loads, is the gather's latency); the sums still take
      // record i before record i + 1, so the accumulation order is the one-record loop's
      uint32_t r = s_off[j] + kk, left = c - kk;
      uint32_t i = i0;
      for (; i + 2 <= i1; i += 2) {
        const uint32_t ra = r;
        if (--left == 0) {  // next source (compacted: non-empty); record i + 1 exists
          ++q;
          j = rlist[q - q0];
          left = s_cnt[j];
          r = s_off[j];
        } else {
          ++r;
        }
        const uint32_t rb = r;
        if (i + 2 < i1) {
          if (--left == 0) {
            ++q;
            j = rlist[q - q0];
            left = s_cnt[j];
            r = s_off[j];
          } else {
            ++r;
          }
        }
        const double2* pa = (const double2*)(s_rec + (size_t)ra * kRecD);
        const double2* pb = (const double2*)(s_rec + (size_t)rb * kRecD);
        const uint32_t sa = rec_swz(ra), sb = rec_swz(rb);
        const double2 a0 = pa[0 ^ sa], a1 = pa[1 ^ sa], a2 = pa[2 ^ sa], a3 = pa[3 ^ sa];
        const double2 b0 = pb[0 ^ sb], b1 = pb[1 ^ sb], b2 = pb[2 ^ sb], b3 = pb[3 ^ sb];
        const double ea = exp((dot3_exact(a1.y, a2.x, a2.y, bd.x, bd.y, bd.z) - a3.x) * inv_tau);
        const double eb = exp((dot3_exact(b1.y, b2.x, b2.y, bd.x, bd.y, bd.z) - b3.x) * inv_tau);
        {
          const double d[3] = {a1.y, a2.x, a2.y}, p[3] = {a0.x, a0.y, a1.x};
          add_contrib(acc, a3.y * ea, d, p);
        }
        {
          const double d[3] = {b1.y, b2.x, b2.y}, p[3] = {b0.x, b0.y, b1.x};
          add_contrib(acc, b3.y * eb, d, p);
        }
      }
      if (i < i1) {
        const double2* rp = (const double2*)(s_rec + (size_t)r * kRecD);
        const uint32_t sw = rec_swz(r);
        const double2 c0 = rp[0 ^ sw], c1 = rp[1 ^ sw], c2 = rp[2 ^ sw], c3 = rp[3 ^ sw];
        bin_contrib(acc, bd, inv_tau, c0.x, c0.y, c1.x, c1.y, c2.x, c2.y, c3.x, c3.y);
      }
    } else if (staged) {
      // a source's records are one contiguous LDS run: the record index advances by one and is
      // re-based only at source boundaries, and the next record is loaded (double2 x 4) while the
      // current one is accumulated
      uint32_t r = s_off[j] + kk, left = c - kk;
      const double2* rp = (const double2*)(s_rec + (size_t)r * kRecD);
      uint32_t sw = rec_swz(r);
      double2 x0 = rp[0 ^ sw], x1 = rp[1 ^ sw], x2 = rp[2 ^ sw], x3 = rp[3 ^ sw];
      for (uint32_t i = i0; i < i1; ++i) {
        const double2 c0 = x0, c1 = x1, c2 = x2, c3 = x3;
        if (i + 1 < i1) {
          if (--left == 0) {  // next source (compacted: non-empty)
            ++q;
            j = rlist[q - q0];
            left = s_cnt[j];
            r = s_off[j];
          } else {
            ++r;
          }
          const double2* np = (const double2*)(s_rec + (size_t)r * kRecD);
          sw = rec_swz(r);
          x0 = np[0 ^ sw]; x1 = np[1 ^ sw]; x2 = np[2 ^ sw]; x3 = np[3 ^ sw];
        }
        bin_contrib(acc, bd, inv_tau, c0.x, c0.y, c1.x, c1.y, c2.x, c2.y, c3.x, c3.y);
      }
    } else {
      for (uint32_t i = i0; i < i1; ++i) {
        uint32_t pidx;
        if (idx_staged) {
          pidx = reinterpret_cast<const uint32_t*>(s_rec)[s_off[j] + kk];
        } else if (a.members) {  // the kk-th smallest member (a tile over even the index stage: rarer)
          const uint32_t* row = a.members + s_st[j];
          pidx = row[0];
          for (uint32_t q = 0; q < c; ++q) {
            const uint32_t m = row[q];
            uint32_t rk = 0;
            for (uint32_t q2 = 0; q2 < c; ++q2) rk += row[q2] < m ? 1u : 0u;
            if (rk == kk) pidx = m;
          }
        } else {
          pidx = a.perm[s_st[j] + kk];
        }
        const double4 pr = reinterpret_cast<const double4*>(a.recs)[pidx];
        const double* sp = a.bin_dirs + 4 * (size_t)a.tile_src[s0 + j];
        double dd[3];
        ray_dir_serial(pr.x, pr.y, pr.z, s_org, dd);
        const double m = dot3_exact(dd[0], dd[1], dd[2], sp[0], sp[1], sp[2]);
        bin_contrib(acc, bd, inv_tau, pr.x, pr.y, pr.z, dd[0], dd[1], dd[2], m, pr.w);
        if (++kk == c && i + 1 < i1) {  // next source (compacted: non-empty)
          kk = 0;
          ++q;
          j = rlist[q - q0];
          c = s_cnt[j];
        }
      }
    }
  }
  if (a.mass_rows) {  // self-budget: the lane's sums times mass_scale (the records carry w / Z without it)
    const double msc = s_msc;
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] *= msc;
  }
  if constexpr (BAL) {
    seg_reduce<19>(acc, seg_j, seg_n, seg_max);
  } else {
#pragma unroll
    for (int f = 0; f < 19; ++f)  // the lanes' shares in a fixed xor tree: ((s0 + s1) + (s2 + s3)) + ...
#pragma unroll
      for (int off = 1; off < LANES; off <<= 1) acc[f] += __shfl_xor(acc[f], off, 64);
  }
  PROF(4);
  if constexpr (SPLIT) {
    // the bin's raw sums for k_bins_finalize: the lane group's first lane (a bin without records has no
    // group and is not active: the finalize takes exact zeros for it, as phase D does)
    static_assert(BAL && !DALL, "the split gather is the balanced 128-bin form");
    if (seg_n > 0 && seg_j == 0) {
      const size_t Bs = (size_t)a.n_bins, b = (size_t)(b0 + lb);
#pragma unroll
      for (int f = 0; f < 19; ++f) a.raw[f * Bs + b] = acc[f];
    }
    PROF(6);
    PROFV(7, 1);
    return;
  }
  if constexpr (DALL) {
    // phase D on every wave: the group's first lane finalizes its bin from the summed registers
    double v[kBinNV];
#pragma unroll
    for (int f = 0; f < kBinNV; ++f) v[f] = 0.0;
    v[4] = -INFINITY;
    if (own) {
      finalize_bin(acc, a.scan, a.n_bins, b0 + own_b, v);
      if (!GCS_MAPV_EARLY && own_act) mapv = load_map_dir(a.map, a.n_bins, b0 + own_b);
      if (own_act) mf_bin_term(acc[0], acc[1], acc[2], acc[3], mapv, v + 5);
    }
    PROF(5);
    // the tile's partial row: a fixed xor tree per wave, then the waves in order
    wave_reduce_bin_terms(v);
    if (lane == 0)
#pragma unroll
      for (int f = 0; f < kBinNV; ++f) lds[wid * 16 + f] = v[f];
    __syncthreads();
    if (t < kBinNV) {
      double x = lds[t];
      for (int w = 1; w < NW; ++w) x = t == 4 ? fmax(x, lds[w * 16 + t]) : x + lds[w * 16 + t];
      partials[(size_t)tile * pstride<kBinNV>() + t] = x;  // folded by k_final<FIN_BINS>
    }
    PROF(6);
    PROFV(7, 1);
    return;
  }
#ifdef GCS_PHASE_PROF
  if (lane == 0 && wid > 0 && wid < 4) g_prof[blockIdx.x * 16 + 10 + wid] = wall_clock64();  // waves 1-3 gather end
#endif
  __syncthreads();  // the record stage is free: it now carries the bin sums [19][TB]
  if (BAL ? (seg_n > 0 && seg_j == 0) : l == 0)  // (balanced: a bin without records has no lane group)
#pragma unroll
    for (int f = 0; f < 19; ++f) s_rec[f * TB + lb] = acc[f];
  __syncthreads();
  // Phase D on the first TB / 64 waves, one lane per bin (full waves: a 128-bin tile's finalize is
  // issued by 2 waves of 64 bins, not by 4 waves with one lane in LANES owning a bin)
  if (TB <= 64 && wid != 0) return;
  if (TB > 64 && t >= TB) {  // the other waves take the partial-row barrier only
    __syncthreads();
    return;
  }
  PROF(14);
  // phase D: finalize + this bin's Matrix-Fisher term (row 7, matrix_fisher_evidence.py:181-211).
  // A bin with no scan mass contributes exact zeros to H, so only active bins read the map.
  double v[kBinNV];
#pragma unroll
  for (int f = 0; f < kBinNV; ++f) v[f] = 0.0;
  v[4] = -INFINITY;
  if (own && GCS_PROBE_NOFIN != 1) {
    const bool has = !BAL || s_work[t] != 0u;  // a bin without records: exact-zero sums
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = has ? s_rec[f * TB + t] : 0.0;
    finalize_bin(acc, a.scan, a.n_bins, b0 + t, v);
    PROF(15);
    if (!GCS_MAPV_EARLY && own_act) mapv = load_map_dir(a.map, a.n_bins, b0 + t);
    if (own_act) mf_bin_term(acc[0], acc[1], acc[2], acc[3], mapv, v + 5);
  }
  PROF(5);
  wave_reduce_bin_terms(v);
  if constexpr (TB <= 64) {
    store_partials<kBinNV>(v, partials, tile);  // folded by k_final<FIN_BINS>
  } else {  // the finalizing waves in order
    if (lane == 0)
#pragma unroll
      for (int f = 0; f < kBinNV; ++f) lds[wid * 16 + f] = v[f];
    __syncthreads();
    if (t < kBinNV) {
      double x = lds[t];
      for (int w = 1; w < TB / 64; ++w) x = t == 4 ? fmax(x, lds[w * 16 + t]) : x + lds[w * 16 + t];
      partials[(size_t)tile * pstride<kBinNV>() + t] = x;  // folded by k_final<FIN_BINS>
    }
  }
  PROF(6);
  PROFV(7, 1);
}

// Phase D of the split bin path, one thread per bin of a tile (TB threads, one tile per workgroup): the
// active tiles' bins (tile flag) from k_bins_scale<..., SPLIT>'s raw sums -- finalize (PSD, kappa, the 26
// ScanBinStats rows), the Matrix-Fisher term of active bins, and the tile's partial row in the order of
// the fused kernel's phase D (a fixed xor tree per 64-bin wave, the waves in order): the same bits.
// Inactive tiles were finished by the gather kernel (zero-bin rows, closed-form partial row).
template <int TB>
__global__ __launch_bounds__(TB) void k_bins_finalize(BinKernelArgs a, double* partials) {
  static_assert(TB % 64 == 0, "whole waves");
  __shared__ double lds[(TB / 64) * 16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int tile = (int)blockIdx.x;
  if (!a.flags[a.n_bins + tile]) return;  // block-uniform
  const int b0 = tile * TB, nb = min(TB, a.n_bins - b0);
  const bool own = t < nb;
  const bool act = own && a.flags[b0 + t];
  const size_t Bs = (size_t)a.n_bins;
  double acc[19];
  MapDir mapv{0.0, 0.0, 0.0, 0.0};
  if (act) {
    mapv = load_map_dir(a.map, a.n_bins, b0 + t);
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = a.raw[f * Bs + b0 + t];
  } else {
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = 0.0;
  }
  double v[kBinNV];
#pragma unroll
  for (int f = 0; f < kBinNV; ++f) v[f] = 0.0;
  v[4] = -INFINITY;
  if (own) {
    finalize_bin(acc, a.scan, a.n_bins, b0 + t, v);
    if (act) mf_bin_term(acc[0], acc[1], acc[2], acc[3], mapv, v + 5);
  }
  wave_reduce_bin_terms(v);
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < kBinNV; ++f) lds[wid * 16 + f] = v[f];
  __syncthreads();
  if (t < kBinNV) {
    double x = lds[t];
    for (int w = 1; w < TB / 64; ++w) x = t == 4 ? fmax(x, lds[w * 16 + t]) : x + lds[w * 16 + t];
    partials[(size_t)tile * pstride<kBinNV>() + t] = x;  // folded by k_final<FIN_BINS>
  }
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
      double p[3] = {pts[j].x, pts[j].y, pts[j].z};
      add_contrib(acc, pts[j].wz * exp((s - pts[j].m) * inv_tau), d, p);  // w r = (w / Z) exp(x)
    }
    size_t nb = gridDim.x;
#pragma unroll
    for (int f = 0; f < 19; ++f) bin_partials[((size_t)f * nb + blockIdx.x) * a.n_bins + b] = acc[f];
  }
}

__global__ __launch_bounds__(kBlock) void k_dense_finalize(BinKernelArgs a, const double* __restrict__ bin_partials,
                                                           int nchunks, double* partials) {
  __shared__ double lds[kWaves * 5];
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
  double v5[5] = {cert[0], cert[1], cert[2], cert[3], cert[4]};
  store_partials<5>(v5, partials, blockIdx.x);  // folded by k_final<FIN_DENSE>
}

// ---------------------------------------------------------------- row 7: Matrix-Fisher reduction
// Standalone form (dense mode and the per-operator entry point): H terms over every bin plus the
// map totals sum S_dir_scatter / sum N_dir (planar z precision, :572-587).  In the scale-mode
// scan the H terms are fused into k_bins_scale and the map totals come from the pushforward.
constexpr int kMfNV = 21;
__global__ __launch_bounds__(kBlock) void k_mf(const double* __restrict__ scan, const double* __restrict__ map, int B,
                                               double* partials) {
  __shared__ double lds[kWaves * kMfNV];
  double v[kMfNV];
#pragma unroll
  for (int k = 0; k < kMfNV; ++k) v[k] = 0.0;
  const size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    mf_bin_term(scan[SF_N * Bs + b], scan[SF_SD * Bs + b], scan[(SF_SD + 1) * Bs + b], scan[(SF_SD + 2) * Bs + b],
                load_map_dir(map, B, b), v);
#pragma unroll
    for (int k = 0; k < 9; ++k) v[11 + k] += map[(MF_S + k) * Bs + b];
    v[20] += map[MF_ND * Bs + b];
  }
  block_sum<kMfNV>(v, lds);
  store_partials<kMfNV>(v, partials, blockIdx.x);  // folded by k_final<FIN_MF>
}

// ---------------------------------------------------------------- row 8: planar translation
// Per bin (matrix_fisher_evidence.py:442-475): t_b = c_map - R p_scan,
// S_b = Sigma_map + R Sigma_scan R^T, W_b = w_b inv(S_b + eps I); L += W_b, h += W_b t_b.
// A bin that is empty in the scan (not a candidate: act = 0) and has never received map mass
// (touched = 0) holds the finalize constants of a zero bin in both (N = 0, p_bar = c = 0,
// Sigma = eps I, gcs_math.h psd_project3): its term is computed from those constants without
// reading the bin (bitwise the same term).  act == nullptr (dense mode): every bin is read.
constexpr int kPtNV = 13;
enum FinalKind : int { FIN_BUDGET, FIN_POINTS, FIN_BINS, FIN_DENSE, FIN_MF, FIN_PT, FIN_TOTALS };

template <int NV, int KIND>
__device__ __forceinline__ void final_epilogue(const double (&v)[NV], double* scalars) {
  if (KIND == FIN_BUDGET) {
    scalars[SC_MASS_IN] = v[0];
    scalars[SC_MASS_SEL] = v[1];
    scalars[SC_MASS_SCALE] = v[0] / (v[1] + kEpsMass);  // point_budget.py:80-84
  } else if (KIND == FIN_POINTS) {
    for (int k = 0; k < 5; ++k) scalars[SC_DESKEW_WIN + k] = v[k];
  } else if (KIND == FIN_BINS) {
    for (int k = 0; k < 5; ++k) scalars[SC_BIN_NSUM + k] = v[k];
    mf_finish(v + 5, scalars);
  } else if (KIND == FIN_DENSE) {
    for (int k = 0; k < 5; ++k) scalars[SC_BIN_NSUM + k] = v[k];
  } else if (KIND == FIN_MF) {
    for (int k = 0; k < 9; ++k) scalars[SC_MF_MAPSCAT + k] = v[11 + k];
    scalars[SC_MF_MAPND] = v[20];
    mf_finish(v, scalars);
  } else if (KIND == FIN_PT) {
    for (int k = 0; k < 9; ++k) scalars[SC_PT_L + k] = v[k];
    for (int k = 0; k < 3; ++k) scalars[SC_PT_H + k] = v[9 + k];
    scalars[SC_PT_NEFF] = v[12];
  } else if (KIND == FIN_TOTALS) {
    for (int k = 0; k < 9; ++k) scalars[SC_MF_MAPSCAT + k] = v[k];
    scalars[SC_MF_MAPND] = v[9];
  }
}

// clr32 / clr8 (may be null): the next scan's bucket counts and active-flag buffer, zeroed here (their
// last readers -- the bin kernel, the previous scan's pushforward -- are behind on the device), so
// the next k_budget skips the clears (PtClear in gcs_kernels.h)
__global__ __launch_bounds__(kBlock) void k_pt(const double* __restrict__ scan, const double* __restrict__ map,
                                               const double* __restrict__ derived, int B, double* scalars,
                                               double* partials, const uint8_t* __restrict__ act,
                                               const uint8_t* __restrict__ touched, PtClear clr) {
  __shared__ double lds[kWaves * pstride<kPtNV>()];
  {
    const long gid = (long)blockIdx.x * kBlock + threadIdx.x, gsz = (long)gridDim.x * kBlock;
    clear_bytes16(reinterpret_cast<uint8_t*>(clr.c32), 4L * clr.n32, gid, gsz);
    clear_bytes16(clr.c8, clr.n8, gid, gsz);
  }
  double R[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = scalars[SC_MF_R + k];
  double v[kPtNV];
#pragma unroll
  for (int k = 0; k < kPtNV; ++k) v[k] = 0.0;
  size_t Bs = (size_t)B;
  // the grid-stride bins of this thread in chunks of kPtU: every flag byte of a chunk is loaded before
  // the first bin's rows (one dependent round trip per chunk, not one per bin; C3: four bins per
  // thread).  The bins and their sums keep the one-bin loop's order.
  constexpr int kPtU = 4;
  const int gstride = gridDim.x * kBlock;
  for (int b0 = blockIdx.x * kBlock + threadIdx.x; b0 < B; b0 += kPtU * gstride) {
    bool scu[kPtU], tcu[kPtU];
#pragma unroll
    for (int u = 0; u < kPtU; ++u) {
      const int bu = b0 + u * gstride;
      scu[u] = bu < B && (!act || act[bu]);
      tcu[u] = bu < B && act && touched[bu];  // (dense mode: act null, every bin read)
    }
#pragma unroll
    for (int u = 0; u < kPtU; ++u) {
    const int b = b0 + u * gstride;
    if (b >= B) break;
    double Ns = 0.0, Nm = 0.0;
    double pb[3] = {0.0, 0.0, 0.0}, c[3] = {0.0, 0.0, 0.0};
    double Sp[9] = {kEpsPsd, 0.0, 0.0, 0.0, kEpsPsd, 0.0, 0.0, 0.0, kEpsPsd};
    double Sc[9] = {kEpsPsd, 0.0, 0.0, 0.0, kEpsPsd, 0.0, 0.0, 0.0, kEpsPsd};
    // scan rows of a bin without scan mass hold the zero-bin values the defaults above restate,
    // map / derived rows of a bin the map never reached hold them too: only the rest is read
    const bool sc = scu[u];
    if (sc) {
      Ns = scan[SF_N * Bs + b];
#pragma unroll
      for (int k = 0; k < 3; ++k) pb[k] = scan[(SF_PB + k) * Bs + b];
#pragma unroll
      for (int k = 0; k < 9; ++k) Sp[k] = scan[(SF_SIG + k) * Bs + b];
    }
    if (sc || tcu[u]) {
      Nm = map[MF_NP * Bs + b];
#pragma unroll
      for (int k = 0; k < 3; ++k) c[k] = derived[(MD_C + k) * Bs + b];
#pragma unroll
      for (int k = 0; k < 9; ++k) Sc[k] = derived[(MD_SIG + k) * Bs + b];
    }
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
  }
  block_sum<kPtNV>(v, lds);
  store_partials<kPtNV>(v, partials, blockIdx.x);  // folded by k_final<FIN_PT>
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

// Map totals for the next scan's planar z precision (sum S_dir_scatter, sum N_dir over bins),
// reduced in fixed order by the last block.
constexpr int kTotNV = 10;
__device__ __forceinline__ void map_totals_partial(double (&tot)[kTotNV], double* lds, double* partials) {
  block_sum<kTotNV>(tot, lds);
  store_partials<kTotNV>(tot, partials, blockIdx.x);  // folded by k_final<FIN_TOTALS>
}

// A bin with no scan mass (act = 0: exact-zero scan sums) and a map that never received mass
// (touched = 0: all-zero stats) stays exactly zero under forgetting + push, and its derived stats
// keep the zero-bin constants: it is skipped (adds exact zeros to the totals).  act == nullptr
// (dense mode): every bin is updated.
#ifndef GCS_PUSH_WAVES
#define GCS_PUSH_WAVES 0  // register target (waves per SIMD) of k_pushforward; 0: compiler default
#endif
__global__ __launch_bounds__(kBlock)
#if GCS_PUSH_WAVES
__attribute__((amdgpu_waves_per_eu(GCS_PUSH_WAVES)))
#endif
void k_pushforward(const double* __restrict__ scan, double* __restrict__ map,
                                                        double* __restrict__ derived, int B, PushArgs pa,
                                                        double* __restrict__ partials,
                                                        const uint8_t* __restrict__ act, uint8_t* __restrict__ touched) {
  __shared__ double lds[kWaves * kTotNV];
  double tot[kTotNV];
#pragma unroll
  for (int k = 0; k < kTotNV; ++k) tot[k] = 0.0;
  const size_t Bs = (size_t)B;
  const double* R = pa.R;
  const double g = pa.gamma;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    // sc: the bin has scan mass.  Without it the scan rows hold the zero-bin values (N = 0, zero
    // sums, p_bar = 0, Sigma_p = eps I) and every scan term below is an exact zero (each is
    // multiplied by N or is R 0 R^T), so the update is the forgetting alone: those rows are not
    // read (masked loads of zeros; the arithmetic is unchanged bit for bit).
    bool sc = true;
    if (act) {
      sc = act[b] != 0;
      if (sc) {
        if (!touched[b]) touched[b] = 1;
      } else if (!touched[b]) {
        continue;
      }
    }
    // every load of the bin is issued before any store: the map rows are read and written in
    // place, so loads placed after a store could not be hoisted above it and each field would cost
    // its own memory round trip
    double ms[26];  // map row: S_dir 3 | S_dir_scatter 9 | N_dir | N_pos | sum p 3 | sum ppT 9
#pragma unroll
    for (int k = 0; k < 3; ++k) ms[k] = map[(MF_SD + k) * Bs + b];
#pragma unroll
    for (int k = 0; k < 9; ++k) ms[3 + k] = map[(MF_S + k) * Bs + b];
    ms[12] = map[MF_ND * Bs + b];
    ms[13] = map[MF_NP * Bs + b];
#pragma unroll
    for (int k = 0; k < 3; ++k) ms[14 + k] = map[(MF_SP + k) * Bs + b];
#pragma unroll
    for (int k = 0; k < 9; ++k) ms[17 + k] = map[(MF_SPP + k) * Bs + b];
    double N = 0.0, pb[3] = {0.0, 0.0, 0.0}, s_d[3] = {0.0, 0.0, 0.0}, S[9], Sg[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      S[k] = 0.0;
      Sg[k] = (k % 4 == 0) ? kEpsPsd : 0.0;
    }
    if (sc) {
      N = scan[SF_N * Bs + b];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        pb[k] = scan[(SF_PB + k) * Bs + b];
        s_d[k] = scan[(SF_SD + k) * Bs + b];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        S[k] = scan[(SF_S + k) * Bs + b];
        Sg[k] = scan[(SF_SIG + k) * Bs + b];
      }
    }
    double u[3], q[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u[i] = R[3 * i] * pb[0] + R[3 * i + 1] * pb[1] + R[3 * i + 2] * pb[2];
      q[i] = u[i] + pa.t[i];
    }
    // S_dir += R s_dir
    double sd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      sd[i] = g * ms[i] + (R[3 * i] * s_d[0] + R[3 * i + 1] * s_d[1] + R[3 * i + 2] * s_d[2]);
      map[(MF_SD + i) * Bs + b] = sd[i];
    }
    // S_dir_scatter += R S R^T
    {
      double RS[9];
      mat3_mul(R, S, RS);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          double v = RS[3 * i] * R[3 * j] + RS[3 * i + 1] * R[3 * j + 1] + RS[3 * i + 2] * R[3 * j + 2];
          double sn = g * ms[3 + 3 * i + j] + v;
          map[(MF_S + 3 * i + j) * Bs + b] = sn;
          tot[3 * i + j] += sn;
        }
    }
    const double nd = g * ms[12] + N;
    const double np = g * ms[13] + N;
    map[MF_ND * Bs + b] = nd;
    map[MF_NP * Bs + b] = np;
    tot[9] += nd;
    double sp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sp[k] = g * ms[14 + k] + N * q[k];
      map[(MF_SP + k) * Bs + b] = sp[k];
    }
    // sum_ppT += N [ R (Sigma_p + p p^T) R^T + J S J^T + q q^T - u u^T ]
    double spp[9];
    {
      double M2[9], RM[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) M2[3 * i + j] = Sg[3 * i + j] + pb[i] * pb[j];
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
          spp[3 * i + j] = g * ms[17 + 3 * i + j] + N * (rmr + jsj + q[i] * q[j] - u[i] * u[j]);
          map[(MF_SPP + 3 * i + j) * Bs + b] = spp[3 * i + j];
        }
    }
    derive_bin(sd, nd, np, sp, spp, derived, Bs, b);
  }
  map_totals_partial(tot, lds, partials);
}

// derived stats + map totals from map sufficient stats only (used after set_map / reset)
__global__ __launch_bounds__(kBlock) void k_map_derive(const double* __restrict__ map, double* derived, int B,
                                                       double* partials, uint8_t* touched) {
  __shared__ double lds[kWaves * kTotNV];
  double tot[kTotNV];
#pragma unroll
  for (int k = 0; k < kTotNV; ++k) tot[k] = 0.0;
  const size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    bool nz = false;
    for (int f = 0; f < MF_COUNT; ++f) nz = nz || map[f * Bs + b] != 0.0;
    if (touched) touched[b] = nz ? 1 : 0;  // any map mass: k_pt / k_pushforward must read the bin
    double sd[3], sp[3], spp[9];
    for (int k = 0; k < 3; ++k) { sd[k] = map[(MF_SD + k) * Bs + b]; sp[k] = map[(MF_SP + k) * Bs + b]; }
    for (int k = 0; k < 9; ++k) { spp[k] = map[(MF_SPP + k) * Bs + b]; tot[k] += map[(MF_S + k) * Bs + b]; }
    tot[9] += map[MF_ND * Bs + b];
    derive_bin(sd, map[MF_ND * Bs + b], map[MF_NP * Bs + b], sp, spp, derived, Bs, b);
  }
  map_totals_partial(tot, lds, partials);
}

// ---------------------------------------------------------------- one-block folds of block partials
// mir.mirror (may be null): after the epilogue the whole scalar block, the device error words, the
// scan's sequence number and a checksum go to the pinned host mirror (gcs_layout.h Mirror), so the
// host reads the scan's results without a separate D2H copy and never consumes a torn mirror.
template <int NV, unsigned MAXMASK, int KIND, int NT = kBlock>
__global__ __launch_bounds__(NT) void k_final(const double* __restrict__ partials, int nblocks, double* scalars,
                                              MirrorArgs mir) {
  static_assert(NT >= MIR_SEQ, "one mirror word per thread");
  __shared__ double lds[(NT / 64) * pstride<NV>()];
  double v[NV];
  reduce_partials<NV, MAXMASK, NT>(partials, nblocks, v, lds);
  if (threadIdx.x == 0) final_epilogue<NV, KIND>(v, scalars);
  if (mir.mirror) {
    __syncthreads();  // thread 0's epilogue stores before every thread's loads (one workgroup)
    const int i = threadIdx.x, lane = i & 63, wid = i >> 6;
    uint64_t* mw = reinterpret_cast<uint64_t*>(mir.mirror);
    uint64_t w = 0;
    if (i < SC_COUNT) {
      w = (uint64_t)__double_as_longlong(scalars[i]);
    } else if (i < MIR_SEQ) {  // the error words, read and re-armed for the next scan
      const int e = 2 * (i - MIR_ERR);
      w = (uint64_t)mir.err[e] | ((uint64_t)mir.err[e + 1] << 32);
      mir.err[e] = 0u;
      mir.err[e + 1] = 0u;
    }
    // the checksum: an integer sum, so any reduction order gives the same value
    unsigned long long h = i < MIR_SEQ ? mirror_word_hash(w, (uint32_t)i) : 0ull;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) h += __shfl_xor(h, off, 64);
    unsigned long long* lh = reinterpret_cast<unsigned long long*>(lds);
    if (lane == 0) lh[wid] = h;
    __syncthreads();
    uint64_t sum = 0;
    if (i == 0) {
      for (int k = 0; k < NT / 64; ++k) sum += lh[k];
      sum += mirror_word_hash(mir.seq, MIR_SEQ);
    }
    if (mir.torn) {  // test knob: the sequence word and checksum first, the data torn microseconds later
      if (i == 0) {
        mw[MIR_SUM] = sum;
        mw[MIR_SEQ] = mir.seq;
      }
      __threadfence_system();
      __syncthreads();
      const uint64_t t0 = wall_clock64();
      while (wall_clock64() - t0 < 100ull * (uint64_t)mir.torn) __builtin_amdgcn_s_sleep(8);
      if (i < MIR_SEQ) mw[i] = w;
      return;
    }
    if (i < MIR_SEQ) mw[i] = w;
    // the block's data stores complete before the checksum and the sequence word are stored (the
    // host still checks the sum, so a transport that reorders them costs a re-read, not a torn result)
    __threadfence_system();
    __syncthreads();
    if (i == 0) {
      mw[MIR_SUM] = sum;
      mw[MIR_SEQ] = mir.seq;
    }
  }
}

// First level of a two-level fold: block j folds partial rows [64 j, 64 j + 64) into row j of out.
// One block reads ~10 B/clk from HBM, so a single-block fold of the 8192 rows (1 MiB) of the
// bin kernel at C3 took 30 us; with a first level on 128 CUs the one-block tail folds 128 rows.
constexpr int kFoldRows = 64;
constexpr int kFoldDirect = 2048;  // up to this many rows a single block folds directly (C2 bins: 1563)
#ifndef GCS_FINAL_WIDE
// threads of a direct fold over more than kFinalWideRows rows (kBlock: off).  Same-box rocprof at C2
// (1,563 rows, profiles/r02/foldab/): 1024 threads 9.9 us, 256 threads 7.8 us -> off
#define GCS_FINAL_WIDE 256
#endif
constexpr int kFinalWide = GCS_FINAL_WIDE, kFinalWideRows = 512;
template <int NV, unsigned MAXMASK>
__global__ __launch_bounds__(kBlock) void k_fold(const double* __restrict__ partials, int nblocks, double* out) {
  __shared__ double lds[kWaves * pstride<NV>()];
  const int r0 = blockIdx.x * kFoldRows;
  double v[NV];
  reduce_partials<NV, MAXMASK>(partials + (size_t)r0 * pstride<NV>(), min(kFoldRows, nblocks - r0), v, lds);
  store_partials<NV>(v, out, blockIdx.x);
}

// Fold nblk partial rows into the scalars (one or two levels).  The level-1 rows are written
// behind the nblk rows of `partials` (partials_need() reserves them).
// e0 / e1 (may be null): the first kernel's start / the last kernel's end.
template <int NV, unsigned MAXMASK, int KIND>
void launch_fold(const double* partials, int nblk, hipStream_t s, hipEvent_t e1, double* scalars, const MirrorArgs& mirror,
                 hipEvent_t e0 = nullptr) {
  if (nblk > kFoldDirect) {
    double* lvl = (double*)partials + (size_t)nblk * pstride<NV>();
    const int g = (nblk + kFoldRows - 1) / kFoldRows;
    hipExtLaunchKernelGGL(k_fold<NV, MAXMASK>, dim3(g), dim3(kBlock), 0, s, e0, nullptr, 0, partials, nblk, lvl);
    hipExtLaunchKernelGGL(k_final<NV, MAXMASK, KIND>, dim3(1), dim3(kBlock), 0, s, nullptr, e1, 0,
                          (const double*)lvl, g, scalars, mirror);
  } else if (kFinalWide != kBlock && nblk > kFinalWideRows) {  // C2 bins: 1563 rows in one or two round trips
    hipExtLaunchKernelGGL((k_final<NV, MAXMASK, KIND, kFinalWide>), dim3(1), dim3(kFinalWide), 0, s, e0, e1, 0,
                          partials, nblk, scalars, mirror);
  } else {
    hipExtLaunchKernelGGL(k_final<NV, MAXMASK, KIND>, dim3(1), dim3(kBlock), 0, s, e0, e1, 0, partials, nblk,
                          scalars, mirror);
  }
}
size_t partials_need(long nblocks, int nv) {
  return (size_t)(nblocks + (nblocks + kFoldRows - 1) / kFoldRows + 1) * partial_stride(nv);
}
#define GCS_FINAL_M(NV, MASK, KIND, nblk, s, e1, partials, scalars, mirror) \
  launch_fold<NV, MASK, KIND>((const double*)(partials), (int)(nblk), s, e1, scalars, mirror)
#define GCS_FINAL(NV, MASK, KIND, nblk, s, e1, partials, scalars) \
  GCS_FINAL_M(NV, MASK, KIND, nblk, s, e1, partials, scalars, MirrorArgs{})

// ---------------------------------------------------------------- bin-tile dispatch order
// One 1024-thread block after the scan's pushforward (off the critical path): the tiles active in this
// scan (tile_dirty after k_bins_scale) in four classes of staged records against the active mean
// (>= 1.5x, >= 1x, >= 0.5x, below), then every other tile, tile order inside a class.  The next
// scan's k_bins_scale dispatches blocks in that order (the sensor's coverage moves little from scan
// to scan): its long tiles start in the first round and the clean tiles fill the last one.  Only
// the dispatch order changes -- each tile's rows and partial row are the same whichever block
// computes them.
constexpr int kOrderNT = 1024, kOrderClasses = 5, kOrderLds = 8192;
__global__ __launch_bounds__(kOrderNT) void k_tile_order(const uint8_t* active, const uint32_t* work, int n,
                                                         int* order) {
  __shared__ uint32_t s_sum[2][kOrderNT / 64];
  __shared__ int s_cnt[kOrderClasses][kOrderNT / 64];
  // up to kOrderLds tiles: the flags and work staged in LDS by coalesced loads (the per-thread chunks
  // below then read LDS, not memory: 19 -> a few us at C3's 8,192 tiles)
  __shared__ uint32_t s_w[kOrderLds];
  __shared__ uint8_t s_a[kOrderLds];
  const bool lds = n <= kOrderLds;
  if (lds) {
    for (int j = threadIdx.x; j < n; j += kOrderNT) {
      s_a[j] = active[j];
      s_w[j] = work[j];
    }
    __syncthreads();
    active = s_a;
    work = s_w;
  }
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int chunk = (n + kOrderNT - 1) / kOrderNT;
  const int j0 = min(n, t * chunk), j1 = min(n, j0 + chunk);
  uint32_t ws = 0, na = 0;
  for (int j = j0; j < j1; ++j)
    if (active[j]) { ws += work[j]; ++na; }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    ws += (uint32_t)__shfl_xor((int)ws, off, 64);
    na += (uint32_t)__shfl_xor((int)na, off, 64);
  }
  if (lane == 0) { s_sum[0][wid] = ws; s_sum[1][wid] = na; }
  __syncthreads();
  unsigned long long W = 0, A = 0;
  for (int w = 0; w < kOrderNT / 64; ++w) { W += s_sum[0][w]; A += s_sum[1][w]; }
  auto cls = [&](int j) -> int {
    if (!active[j]) return 4;
    const unsigned long long wa = (unsigned long long)work[j] * A;  // work / mean = wa / W
    return 2 * wa >= 3 * W ? 0 : (wa >= W ? 1 : (2 * wa >= W ? 2 : 3));
  };
  int cnt[kOrderClasses] = {0, 0, 0, 0, 0};
  for (int j = j0; j < j1; ++j) ++cnt[cls(j)];
  int pos[kOrderClasses];
#pragma unroll
  for (int c = 0; c < kOrderClasses; ++c) {
    int x = cnt[c];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_cnt[c][wid] = x;
    pos[c] = x - cnt[c];
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int c = 0; c < kOrderClasses; ++c) {
    int pre = 0, tot = 0;
    for (int w = 0; w < kOrderNT / 64; ++w) {
      const int v = s_cnt[c][w];
      pre += w < wid ? v : 0;
      tot += v;
    }
    pos[c] += base + pre;
    base += tot;
  }
  for (int j = j0; j < j1; ++j) {
    const int c = cls(j);
    order[pos[c]++] = j;
  }
}

// The same classes, dealt to the 8 XCDs (blocks are dealt round-robin over them: block b runs on the
// XCD of b % 8; MI355X_MICROARCH.md "Workgroup dispatch", for speed only).  The active tiles, in tile
// (Hilbert) order, are cut into 8 contiguous groups of equal count, the inactive tiles likewise so
// that every group holds n / 8 tiles; group g's tiles go to blocks g, g + 8, g + 16, ... in the class
// order above (heaviest first, then tile order; its inactive tiles last).  Each XCD then stages the
// records of one compact patch of the scan's coverage -- a bucket feeds ~2.3 neighbouring tiles,
// which now share that XCD's L2 -- instead of every XCD touching the whole band.  n % 8 == 0.
__global__ __launch_bounds__(kOrderNT) void k_tile_order_xcd(const uint8_t* active, const uint32_t* work, int n,
                                                             int* order) {
  constexpr int NC = kOrderClasses - 1;  // active classes
  __shared__ uint32_t s_sum[2][kOrderNT / 64];
  __shared__ int s_cnt[kOrderClasses][kOrderNT / 64];
  __shared__ int s_gstart[8][NC];  // per-class prefix at each group's first active tile
  __shared__ int s_gcnt[8][NC];    // per-group class counts
  __shared__ uint32_t s_w[kOrderLds];
  __shared__ uint8_t s_a[kOrderLds];
  const bool lds = n <= kOrderLds;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t < 8 * NC) {
    (&s_gcnt[0][0])[t] = 0;
    (&s_gstart[0][0])[t] = 0;
  }
  if (lds) {
    for (int j = t; j < n; j += kOrderNT) {
      s_a[j] = active[j];
      s_w[j] = work[j];
    }
    active = s_a;
    work = s_w;
  }
  __syncthreads();
  const int chunk = (n + kOrderNT - 1) / kOrderNT;
  const int j0 = min(n, t * chunk), j1 = min(n, j0 + chunk);
  uint32_t ws = 0, na = 0;
  for (int j = j0; j < j1; ++j)
    if (active[j]) { ws += work[j]; ++na; }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    ws += (uint32_t)__shfl_xor((int)ws, off, 64);
    na += (uint32_t)__shfl_xor((int)na, off, 64);
  }
  if (lane == 0) { s_sum[0][wid] = ws; s_sum[1][wid] = na; }
  __syncthreads();
  unsigned long long W = 0, A = 0;
  for (int w = 0; w < kOrderNT / 64; ++w) { W += s_sum[0][w]; A += s_sum[1][w]; }
  auto cls = [&](int j) -> int {
    if (!active[j]) return NC;
    const unsigned long long wa = (unsigned long long)work[j] * A;  // work / mean = wa / W
    return 2 * wa >= 3 * W ? 0 : (wa >= W ? 1 : (2 * wa >= W ? 2 : 3));
  };
  // per-class exclusive prefixes at the chunk start (class NC: the inactive tiles' rank)
  int cnt[kOrderClasses] = {0, 0, 0, 0, 0};
  for (int j = j0; j < j1; ++j) ++cnt[cls(j)];
  int pre[kOrderClasses];
#pragma unroll
  for (int c = 0; c < kOrderClasses; ++c) {
    int x = cnt[c];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_cnt[c][wid] = x;
    pre[c] = x - cnt[c];
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kOrderClasses; ++c)
    for (int w = 0; w < wid; ++w) pre[c] += s_cnt[c][w];
  const int nq = n >> 3;                     // tiles per group
  const int Ai = (int)A;
  auto gbound = [&](int g) { return (int)(((long long)g * Ai + 7) / 8); };  // first active rank of group g
  // pass 2: each group's class counts, and the class prefixes at its first active tile
  {
    int P[kOrderClasses];
#pragma unroll
    for (int c = 0; c < kOrderClasses; ++c) P[c] = pre[c];
    for (int j = j0; j < j1; ++j) {
      const int c = cls(j);
      if (c < NC) {
        const int r = P[0] + P[1] + P[2] + P[3];  // active rank
        const int g = (int)((8LL * r) / Ai);
        if (r == gbound(g))
#pragma unroll
          for (int cc = 0; cc < NC; ++cc) s_gstart[g][cc] = P[cc];
        atomicAdd(&s_gcnt[g][c], 1);
      }
      ++P[c];
    }
  }
  __syncthreads();
  // pass 3: positions
  {
    int P[kOrderClasses];
#pragma unroll
    for (int c = 0; c < kOrderClasses; ++c) P[c] = pre[c];
    for (int j = j0; j < j1; ++j) {
      const int c = cls(j);
      int g, pos;
      if (c < NC) {
        const int r = P[0] + P[1] + P[2] + P[3];
        g = (int)((8LL * r) / Ai);
        pos = P[c] - s_gstart[g][c];
        for (int cc = 0; cc < c; ++cc) pos += s_gcnt[g][cc];
      } else {
        // inactive rank q: group g holds ranks [g nq - gbound(g), (g + 1) nq - gbound(g + 1))
        const int q = P[NC];
        g = 0;
        while (g < 7 && q >= (g + 1) * nq - gbound(g + 1)) ++g;
        pos = (gbound(g + 1) - gbound(g)) + (q - (g * nq - gbound(g)));
      }
      order[8 * pos + g] = j;
      ++P[c];
    }
  }
}

hipError_t launch_tile_order_variant(const uint8_t* active, const uint32_t* work, int n, int* order, bool xcd,
                                     hipStream_t s) {
  if (xcd && (n & 7) == 0)
    hipLaunchKernelGGL(k_tile_order_xcd, dim3(1), dim3(kOrderNT), 0, s, active, work, n, order);
  else
    hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(kOrderNT), 0, s, active, work, n, order);
  return hipGetLastError();
}
hipError_t launch_tile_order(const uint8_t* active, const uint32_t* work, int n, int* order, hipStream_t s) {
  // GCSLAM_TILE_XCD=0: the round-3 order (classes only), for A/B
  static const bool xcd = [] {
    const char* e = getenv("GCSLAM_TILE_XCD");
    return !(e && atoi(e) == 0);
  }();
  return launch_tile_order_variant(active, work, n, order, xcd, s);
}

// ---------------------------------------------------------------- launchers
static int grid_for(long n, int cap_blocks) {
  long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > cap_blocks ? cap_blocks : g);
}
// The pushforward's grid is capped at 1,024 blocks (a grid-stride loop of four bins per thread at C3):
// the 4,096-block grid took every CU's registers (256 VGPRs, two waves per SIMD) for its whole
// length, so the next scan's budget and point kernels, which overlap it, waited for its blocks to
// drain.  Same box, alternated (profiles/r04/pushb/): C3 0.2201 vs 0.2392-0.2396 ms per step, the
// pushforward itself 56.8 vs 65.5-66.1 us; 256 / 512 blocks 0.2249-0.2275 ms.  GCSLAM_PUSH_BLOCKS for A/B.
int push_blocks(int n_bins) {
  static const int cap = [] {
    const char* e = getenv("GCSLAM_PUSH_BLOCKS");
    return e ? std::max(1, std::min(4096, atoi(e))) : 1024;
  }();
  return grid_for(n_bins, cap);
}

hipError_t launch_parse(const ParseArgs& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  const int nblk = (a.n + kBlock - 1) / kBlock;
  hipError_t e = hipMemsetAsync(a.ns_flag, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_parse_pc2, dim3(nblk), dim3(kBlock), 0, s, a);
  if (a.off_t >= 0)
    hipLaunchKernelGGL(k_parse_time_scale, dim3(nblk), dim3(kBlock), 0, s, a.t, a.n, (const uint32_t*)a.ns_flag);
  return hipGetLastError();
}

hipError_t launch_budget(const BudgetArgs& a, int nblk, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_budget, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a);  // folded inside k_points
  return hipGetLastError();
}

// ---------------------------------------------------------------- launch gate of the scan front
// One wave, queued between k_budget and k_points by the pre-launched scan front: lane 0 polls the
// host gate word (coherent host memory; relaxed system-scope loads are uncached reads, where an
// acquire would add a cache invalidate per poll) until it holds seq, then copies the deskew twist to
// device memory for k_points, which the stream starts right behind it.  One poller, one wave: the
// point kernel itself (~360 registers per lane: one wave per SIMD) is not resident while the host
// prologue runs, so the previous scan's pushforward keeps the SIMDs (a resident, polling k_points
// starved it: C2 device wait 77 -> 120 us).  Not opened within kGateTimeoutTicks: zero twist and
// *err = 1 (gcs_scan fails).
__global__ __launch_bounds__(64) void k_gate(const uint64_t* gate, uint64_t seq, double* xi_out, uint32_t* err) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  bool open = false;
  for (;;) {
    if (__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq) { open = true; break; }
    if (wall_clock64() - t0 > kGateTimeoutTicks) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __asm__ volatile("" ::: "memory");
  for (int k = 0; k < 6; ++k)
    xi_out[k] = open ? __longlong_as_double((long long)__hip_atomic_load(gate + 1 + k, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_SYSTEM))
                     : 0.0;
  if (!open) *err = 1u;
}

// ---------------------------------------------------------------- hypothesis payload staging
// The per-scan all-reduce (gcs_combine_allreduce) on the context's combine stream: ncclAllReduce reads
// the host-packed payload from pinned memory, k_payload_out copies the sum back to a second pinned host
// buffer followed by the call's sequence number and a checksum (the scan mirror's protocol,
// gcs_layout.h), and the host polls that instead of a copy call and a stream synchronize.
__global__ __launch_bounds__(kBlock) void k_payload_out(const double* __restrict__ src, double* host, int n,
                                                        uint64_t* dseq) {
  __shared__ unsigned long long lh[kWaves];
  unsigned long long h = 0;
  uint64_t* hw = reinterpret_cast<uint64_t*>(host);
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const uint64_t w = (uint64_t)__double_as_longlong(src[i]);
    hw[i] = w;
    h += mirror_word_hash(w, (uint32_t)i);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) h += __shfl_xor(h, off, 64);
  if ((threadIdx.x & 63) == 0) lh[threadIdx.x >> 6] = h;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {  // the launch's sequence number: a device counter (the chain is queued ahead)
    const uint64_t seq = *dseq + 1u;
    *dseq = seq;
    uint64_t sum = mirror_word_hash(seq, (uint32_t)n);
    for (int k = 0; k < kWaves; ++k) sum += lh[k];
    hw[n + 1] = sum;
    hw[n] = seq;
  }
}
hipError_t launch_payload_out(const double* src, double* host, int n, uint64_t* dseq, hipStream_t s) {
  hipLaunchKernelGGL(k_payload_out, dim3(1), dim3(kBlock), 0, s, src, host, n, dseq);
  return hipGetLastError();
}

// GCS_DEBUG_COMBINE_DELAY's stand-in for a late peer: one wave sleeps on the 100 MHz wall clock
__global__ __launch_bounds__(64) void k_delay(uint32_t us) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < 100ull * (uint64_t)us) __builtin_amdgcn_s_sleep(64);
}

hipError_t launch_delay(int us, hipStream_t s) {
  hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, (uint32_t)us);
  return hipGetLastError();
}

hipError_t launch_gate(const uint64_t* gate, uint64_t seq, double* xi_out, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, gate, seq, xi_out, err);
  return hipGetLastError();
}

#ifndef GCS_POINT_LANES
#define GCS_POINT_LANES 1  // lanes per point (scale mode); 2 and 4 measured slower, DESIGN.md section 5
#endif
constexpr int kPointLanes = GCS_POINT_LANES;
constexpr int kPointsMaxBlocks = 4096;
int points_max_blocks() { return kPointsMaxBlocks; }
int points_blocks(long cap, bool scale) {
  const long lanes = scale ? kPointLanes : 1;
  const long need = (cap * lanes + kBlock - 1) / kBlock;
  return (int)std::max(1L, std::min((long)(scale ? kPointsMaxBlocks : 1024), need));
}

hipError_t launch_points(const PointKernelArgs& a, bool scale, double* partials, int nblk, bool fold, hipStream_t s,
                         hipEvent_t e0, hipEvent_t e1, bool legacy, const MirrorArgs& mir) {
  // without the fold (it rides in k_bins_scale's block 0) the stage ends with k_points itself
  hipEvent_t ek = fold ? nullptr : e1;
  // legacy: the round-3 point kernel (one wave per SIMD; GCSLAM_POINTS=legacy / GCS_DEBUG_POINT_KERNEL), for A/B
  if (scale && !legacy && kPointLanes == 1 && (long)nblk * kBlock >= (long)a.cap) {  // one point per thread
    // at most one wave per SIMD: the wide form (all 16 candidate directions in one load group, one
    // wave per SIMD) measured slower than the 4-wave form on the same grid -- C2 points 19.8-19.9 vs
    // 18.9 us (profiles/r04/rcp/) -- so it is opt-in (GCSLAM_POINTS_WIDE=1), kept for A/B
    static const bool wide_ok = [] {
      const char* e = getenv("GCSLAM_POINTS_WIDE");
      return e && atoi(e) != 0;
    }();
    const bool wide = wide_ok && (long)nblk * kBlock <= 1024L * 64;
    switch (a.k) {
      case 8:
        if (wide) hipExtLaunchKernelGGL((k_points_lean<8, true>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        else hipExtLaunchKernelGGL((k_points_lean<8, false>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        break;
      case 16:
        if (wide) hipExtLaunchKernelGGL((k_points_lean<16, true>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        else hipExtLaunchKernelGGL((k_points_lean<16, false>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        break;
      case 32:
        if (wide) hipExtLaunchKernelGGL((k_points_lean<32, true>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        else hipExtLaunchKernelGGL((k_points_lean<32, false>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
        break;
      default: return hipErrorInvalidValue;
    }
  } else if (scale) {
    switch (a.k) {
      case 8: hipExtLaunchKernelGGL((k_points<true, 8, kPointLanes>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials); break;
      case 16: hipExtLaunchKernelGGL((k_points<true, 16, kPointLanes>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials); break;
      case 32: hipExtLaunchKernelGGL((k_points<true, 32, kPointLanes>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials); break;
      default: return hipErrorInvalidValue;
    }
  } else if (a.n_bins == 0) {  // deskew only (gcs_scan_begin)
    hipExtLaunchKernelGGL((k_points<false, 0, 1>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
  } else {
    hipExtLaunchKernelGGL((k_points<false, 1, 1>), dim3(nblk), dim3(kBlock), 0, s, e0, ek, 0, a, partials);
  }
  if (fold) GCS_FINAL_M(5, 16u, FIN_POINTS, nblk, s, e1, partials, a.scalars, mir);
  return hipGetLastError();
}

int scan_tiles(int n_bins) { return (n_bins + kScanTile - 1) / kScanTile; }

hipError_t launch_bucketing(const BucketArgs& b, int n, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_scan, dim3(scan_tiles(b.n_bins)), dim3(kScanThreads), 0, s, e0, nullptr, 0,
                        (const uint32_t*)b.counts, b.n_bins, b.scan_status, b.scan_ticket, b.starts, b.err,
                        b.spin_limit, b.inject_scan_fail);
  hipLaunchKernelGGL(k_place, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, (const uint32_t*)b.keys,
                     (const uint32_t*)b.slots, (const uint32_t*)b.starts, n, b.n_bins, b.slot_idx);
  hipExtLaunchKernelGGL(k_bucket_rank, dim3((b.n_bins + kBlock - 1) / kBlock), dim3(kBlock), 0, s, nullptr, e1, 0, b,
                        n);
  return hipGetLastError();
}

int bins_tile_for(long cap, int n_bins) {
  if (const char* e = getenv("GCSLAM_BIN_TILE")) {
    const int v = atoi(e);
    if (v == 32 || v == 64 || v == 128 || v == 256) return v;
  }
  // Sparse maps (under 0.4 points per bin, C3: 262,144 points over 1,048,576 bins) run 128-bin tiles:
  // half the tiles, each amortising its table phase over twice the bins (C3 bins 88 vs 106 us, sweep
  // profiles/r03).  Denser maps (C2: 65,536 points over 100,000 bins) keep 64-bin tiles, whose stage
  // fits the heavier per-bin record load (25.5 vs 30.5 us).
  return (long)cap * 5 < (long)n_bins * 2 ? 128 : 64;
}
int bins_scale_blocks(int n_bins, int tile_bins) { return (n_bins + tile_bins - 1) / tile_bins; }
int bins_partial_nv() { return kBinNV; }

hipError_t launch_bins_scale(const BinKernelArgs& a, double* partials, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                             hipEvent_t f0, hipEvent_t f1) {
  const int nblk = bins_scale_blocks(a.n_bins, a.tile_bins);
  const bool big = (long)a.cap * 5 >= (long)a.n_bins * 2;  // C2-like: dense in the map
  if (a.tile_bins == 32)  // half the records of a 64-bin tile: the small stage holds them
    hipExtLaunchKernelGGL((k_bins_scale<kStageSmall, 32, 8, false>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  else if (a.tile_bins == 128 && big)
    hipExtLaunchKernelGGL((k_bins_scale<kStage128Big, 128, 2, GCS_DALL128>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  else if (a.tile_bins == 128 && a.raw) {  // split: the gather, then phase D one thread per bin (e0 .. e1: both)
    hipExtLaunchKernelGGL((k_bins_scale<kStage128Small, 128, 2, false, true>), dim3(nblk), dim3(256), 0, s, e0, nullptr, 0, a,
                          partials);
    hipExtLaunchKernelGGL(k_bins_finalize<128>, dim3(nblk), dim3(128), 0, s, nullptr, e1, 0, a, partials);
  } else if (a.tile_bins == 128)
    hipExtLaunchKernelGGL((k_bins_scale<kStage128Small, 128, 2, GCS_DALL128>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  else if (a.tile_bins == 256 && big)
    hipExtLaunchKernelGGL((k_bins_scale<kStage256Big, 256, 1, true>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  else if (a.tile_bins == 256)
    hipExtLaunchKernelGGL((k_bins_scale<kStage256Small, 256, 1, true>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  // (eight lanes per bin on the 64-bin tile, 512 threads: 35.2 vs 25.4 us at C2, same box)
  else if (big)
    hipExtLaunchKernelGGL((k_bins_scale<kStageBig, 64, 4, GCS_DALL64>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  else
    hipExtLaunchKernelGGL((k_bins_scale<kStageSmall, 64, 4, GCS_DALL64>), dim3(nblk), dim3(256), 0, s, e0, e1, 0, a, partials);
  launch_fold<kBinNV, 16u, FIN_BINS>(partials, nblk, s, f1, a.scalars, MirrorArgs{}, f0);
  return hipGetLastError();
}

hipError_t launch_dense(const BinKernelArgs& a, double* bin_partials, double* partials, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1) {
  int nchunks = (a.cap + kBlock - 1) / kBlock;
  hipExtLaunchKernelGGL(k_dense_accum, dim3(nchunks), dim3(kBlock), 0, s, e0, nullptr, 0, a, bin_partials);
  int nblk = (a.n_bins + kBlock - 1) / kBlock;
  hipExtLaunchKernelGGL(k_dense_finalize, dim3(nblk), dim3(kBlock), 0, s, nullptr, nullptr, 0, a,
                        (const double*)bin_partials, nchunks, partials);
  GCS_FINAL(5, 16u, FIN_DENSE, nblk, s, e1, partials, a.scalars);
  return hipGetLastError();
}

hipError_t launch_mf(const double* scan, const double* map, int B, double* partials, int nblk, double* scalars,
                     hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_mf, dim3(nblk), dim3(kBlock), 0, s, e0, nullptr, 0, scan, map, B, partials);
  GCS_FINAL(kMfNV, 0u, FIN_MF, nblk, s, e1, partials, scalars);
  return hipGetLastError();
}

hipError_t launch_pt(const double* scan, const double* map, const double* derived, int B, double* partials, int nblk,
                     double* scalars, const MirrorArgs& mirror, const uint8_t* act, const uint8_t* touched,
                     hipStream_t s, hipEvent_t e0, hipEvent_t e1, PtClear clr) {
  // (measured slower and removed: a last-block fold in k_pt, ticket + agent-scope release per block:
  // 16.4 vs 12.3 us at C2, 46 vs 25 us at C3; the same with sc1 stores / loads and no fence: C2
  // 105.4-105.9 vs 103.5-104.1 us per step, profiles/r03/ptfold/)
  hipExtLaunchKernelGGL(k_pt, dim3(nblk), dim3(kBlock), 0, s, e0, nullptr, 0, scan, map, derived, B, scalars, partials,
                        act, touched, clr);
  GCS_FINAL_M(kPtNV, 0u, FIN_PT, nblk, s, e1, partials, scalars, mirror);
  return hipGetLastError();
}

hipError_t launch_pushforward(const double* scan, double* map, double* derived, int B, const PushArgs& pa,
                              double* partials, double* scalars, const uint8_t* act, uint8_t* touched, hipStream_t s,
                              hipEvent_t e0, hipEvent_t e1) {
  const int nblk = push_blocks(B);
  hipExtLaunchKernelGGL(k_pushforward, dim3(nblk), dim3(kBlock), 0, s, e0, nullptr, 0, scan, map, derived, B, pa,
                        partials, act, touched);
  GCS_FINAL(kTotNV, 0u, FIN_TOTALS, nblk, s, e1, partials, scalars);
  return hipGetLastError();
}

hipError_t launch_map_derive(const double* map, double* derived, int B, double* partials, double* scalars,
                             uint8_t* touched, hipStream_t s) {
  const int nblk = push_blocks(B);
  hipLaunchKernelGGL(k_map_derive, dim3(nblk), dim3(kBlock), 0, s, map, derived, B, partials, touched);
  GCS_FINAL(kTotNV, 0u, FIN_TOTALS, nblk, s, nullptr, partials, scalars);
  return hipGetLastError();
}

}  // namespace gcs
