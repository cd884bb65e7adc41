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

#include <hip/hip_ext.h>
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

// Final pass over per-block partials inside one block: thread t folds partials t, t+256, ... in
// order, then a fixed tree; the result is valid in thread 0.  Bit k of MAXMASK selects max
// instead of sum for component k.  lds must hold kWaves*NV doubles.
template <int NV, unsigned MAXMASK>
__device__ __forceinline__ void reduce_partials(const double* __restrict__ partials, int nblocks, double (&v)[NV],
                                                double* lds) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = ((MAXMASK >> k) & 1u) ? -INFINITY : 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      // device-coherent load (sc1): partials of other blocks were stored device-coherently
      double x = __hip_atomic_load(partials + (size_t)b * NV + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
      v[k] = s;
    }
  }
  __syncthreads();
}

// "Last block finishes", two levels: thread 0 of every block stores the block partial
// device-coherently (sc1 stores, no L2 write-back), waits for the stores to complete and draws a
// ticket of its group of 64 blocks; the last block of a group folds the group's partials (fixed
// order, sc1 loads) into a group partial and draws the kernel-wide ticket; the last group runs
// the final fold.  No single block ever reads more than 64 partials, and a full
// __threadfence() (buffer_wbl2: write-back of the XCD's whole L2, per block) is never needed.
// Tickets re-arm themselves.  Layout: partials[nblocks*NV] then group partials[ngroups*NV];
// tickets[0] kernel-wide, tickets[1 + g] per group.
constexpr int kFinGroup = 64;  // kTicketStride (gcs_kernels.h) >= 1 + ngroups

template <int NV>
__device__ __forceinline__ void store_partials(const double (&v)[NV], double* base, int idx) {
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k)
      __hip_atomic_store(base + (size_t)idx * NV + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool ticket_last(uint32_t* ticket, uint32_t expected) {
  __shared__ uint32_t s_last;
  if (threadIdx.x == 0) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // this thread's partial stores have completed
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint32_t prev = atomicAdd(ticket, 1u);
    uint32_t last = (prev == expected - 1u) ? 1u : 0u;
    if (last) atomicExch(ticket, 0u);
    s_last = last;
  }
  __syncthreads();
  return s_last != 0u;
}

// v: block partial (valid in thread 0).  Returns true in the one block that finishes, with the
// kernel-wide fold in v (thread 0).
template <int NV, unsigned MAXMASK>
__device__ bool finish_blocks(double (&v)[NV], double* partials, uint32_t* tickets, double* lds) {
  const int nb = gridDim.x;
  const int ng = (nb + kFinGroup - 1) / kFinGroup;
  store_partials<NV>(v, partials, blockIdx.x);
  const int g = blockIdx.x / kFinGroup;
  const int gsz = min(kFinGroup, nb - g * kFinGroup);
  if (!ticket_last(tickets + 1 + g, (uint32_t)gsz)) return false;
  reduce_partials<NV, MAXMASK>(partials + (size_t)g * kFinGroup * NV, gsz, v, lds);
  double* gp = partials + (size_t)nb * NV;
  store_partials<NV>(v, gp, g);
  if (!ticket_last(tickets, (uint32_t)ng)) return false;
  reduce_partials<NV, MAXMASK>(gp, ng, v, lds);
  return true;
}

// ---------------------------------------------------------------- row 1: budget mass sums
// Also clears the scale-mode bucketing state of this scan (counts, flags, look-back status),
// replacing three memsets.  mass_scale = total_mass_in / (total_mass_selected + eps_mass)
// (point_budget.py:80-84) is produced by the last block.
__global__ __launch_bounds__(kBlock) void k_budget(BudgetArgs a) {
  __shared__ double lds[kWaves * 2];
  const int gid = blockIdx.x * kBlock + threadIdx.x, gsz = gridDim.x * kBlock;
  for (int j = gid; j < a.n_zero32; j += gsz) a.zero32[j] = 0u;
  for (int j = gid; j < a.n_zero8; j += gsz) a.zero8[j] = 0u;
  double v[2] = {0.0, 0.0};
  for (int j = gid; j < a.n_raw; j += gsz) {
    double x = a.w[j];
    v[0] += x;
    if (j % a.stride == 0) v[1] += x;
  }
  block_sum<2>(v, lds);
  if (!finish_blocks<2, 0u>(v, a.partials, a.ticket, lds)) return;
  if (threadIdx.x == 0) {
    a.scalars[SC_MASS_IN] = v[0];
    a.scalars[SC_MASS_SEL] = v[1];
    a.scalars[SC_MASS_SCALE] = v[0] / (v[1] + kEpsMass);
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
// At C2 the grid is ~1 wave per SIMD, so the kernel is bound by each lane's dependent chain:
// loads are issued in independent batches (whole pool row, whole candidate row) so the chain is
// xyz -> pool ids -> pool dirs -> knn row -> candidate dirs -> slot atomic, and the softmax
// evaluates one exp per candidate and no per-candidate log (entropy identity below).
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
        const int nq = a.pool_width >> 2;
        double best = -INFINITY;
        for (int q = 0; q < nq; q += 2) {  // 8 ids per batch: all loads in flight together
          int4 u0 = pool[q];
          int4 u1 = q + 1 < nq ? pool[q + 1] : make_int4(-1, -1, -1, -1);
          int ids[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
          double s[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            s[u] = -INFINITY;
            if (ids[u] >= 0) {
              const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)ids[u]);
              s[u] = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (s[u] > best) { best = s[u]; nearest = ids[u]; }
          if (u1.w < 0) break;
        }
      }
      const int4* cand4 = (const int4*)(a.knn + (size_t)nearest * KC);
      int cand[KC];
#pragma unroll
      for (int k = 0; k < KC / 4; ++k) {
        int4 c4 = cand4[k];
        cand[4 * k] = c4.x; cand[4 * k + 1] = c4.y; cand[4 * k + 2] = c4.z; cand[4 * k + 3] = c4.w;
      }
      double e[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)cand[k]);
        e[k] = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
        m = fmax(m, e[k]);
      }
      // e_k = exp(x_k), x_k = (sim_k - m)/tau (binning.py:69 softmax, shifted by the max)
      double sxe = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        double x = (e[k] - m) * inv_tau;
        e[k] = exp(x);
        Z += e[k];
        sxe += x * e[k];
      }
      const double iz = 1.0 / Z;
      // entropy of r_k = e_k/Z (binning.py:71-75): -sum r log(r + eps)
      //   = log Z - sum r_k x_k - sum r_k log1p(eps/r_k),
      // with r log1p(eps/r) in [0, eps] taken as eps r/(r + eps) (|error| < 0.2 eps per term)
      double corr = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        double r = e[k] * iz;
        corr += r * __builtin_amdgcn_rcp(r + kEpsMass);
        rm = fmax(rm, r);
      }
      H = log(Z) - sxe * iz - kEpsMass * corr;
      uint32_t key = (uint32_t)a.n_bins;
      if (valid) {
        // bucket slot: arrival order only (re-ranked by point index in k_bucket_build)
        a.slots[i] = atomicAdd(a.counts + nearest, 1u);
        key = (uint32_t)nearest;
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
  double v[5] = {acc[0], acc[1], acc[2], acc[3], rmax};
  // (sum wb, sum wn^2, sum w_out, sum H, max r) -> scalars[SC_DESKEW_WIN..]
  if (!finish_blocks<5, 16u>(v, partials, a.ticket, lds)) return;
  if (threadIdx.x == 0)
    for (int k = 0; k < 5; ++k) a.scalars[SC_DESKEW_WIN + k] = v[k];
}

// ---------------------------------------------------------------- deterministic bucketing by nearest bin
// k_points took an arrival slot per point (atomic per-bucket counts).  k_scan: start[] =
// exclusive scan of the counts in one pass (decoupled look-back over 4096-bucket tiles, one
// wave reading 64 predecessors per step).  k_place scatters point indices by slot.
// k_bucket_rank gives every member its rank by point index inside its bucket (one lane per
// bucket up to kLaneRank members, else one wave per bucket in k_bucket_mid; above kRankMax an
// in-order compaction over all keys) and writes the member's destination start+rank; it also
// marks the K candidate bins of every non-empty bucket active.  k_gather then moves every point
// record to its destination, so each bucket's records are contiguous in point-index order and
// the bin gather streams them in a scheduling-independent order.
constexpr int kScanTile = 4096;
constexpr int kLaneRank = 16;
constexpr int kRankMax = 8192;
constexpr uint32_t kLbAgg = 1u << 30, kLbPre = 2u << 30, kLbVal = (1u << 30) - 1u;

__global__ __launch_bounds__(kBlock) void k_scan(const uint32_t* __restrict__ counts, int n, uint32_t* status,
                                                 uint32_t* ticket, uint32_t* start) {
  __shared__ uint32_t wsum[kWaves];
  __shared__ uint32_t s_tile, s_excl;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) s_tile = atomicAdd(ticket, 1u);  // tiles are numbered in start order (forward progress)
  __syncthreads();
  const uint32_t tile = s_tile;
  const int base = (int)tile * kScanTile + 16 * t;
  uint32_t v[16];
  uint32_t tot = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    v[j] = (base + j < n) ? counts[base + j] : 0u;
    tot += v[j];
  }
  uint32_t x = tot;
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    const uint32_t agg = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    uint32_t excl = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(status, kLbPre | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(status + tile, kLbAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // look back in windows of 64 predecessors: lane l reads tile (w0 - l)
      uint32_t spins = 0;
      int w0 = (int)tile - 1;
      while (w0 >= 0) {
        const int j = w0 - lane;
        uint32_t s = j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbPre;
        // the window is usable up to (and including) its nearest published prefix
        const unsigned long long pre = __ballot((s & ~kLbVal) == kLbPre);
        const int stop = pre ? (__ffsll((long long)pre) - 1) : 63;
        const unsigned long long unpub = __ballot(s == 0u && lane <= stop);
        if (unpub) {  // bounded so a broken invariant cannot hang the GPU
          if (++spins > (1u << 22)) { excl = 0xffffffffu; break; }
          continue;
        }
        uint32_t val = (lane <= stop && j >= 0) ? (s & kLbVal) : 0u;
        for (int off = 32; off >= 1; off >>= 1) val += __shfl_xor(val, off, 64);
        excl += val;
        if (pre) break;
        w0 -= 64;
      }
      if (lane == 0) __hip_atomic_store(status + tile, kLbPre | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      if (tile == gridDim.x - 1) atomicExch(ticket, 0u);  // every tile has drawn its number by now
    }
  }
  __syncthreads();
  uint32_t pre = s_excl + x - tot;
  for (int w = 0; w < wid; ++w) pre += wsum[w];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (base + j < n) start[base + j] = pre;
    pre += v[j];
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

// one lane per bucket (grid covers all buckets exactly once)
__global__ __launch_bounds__(kBlock) void k_bucket_rank(BucketArgs b) {
  const int a = blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t c = a < b.n_bins ? b.counts[a] : 0u;
  const bool mid = c > (uint32_t)kLaneRank;
  const unsigned long long mm = __ballot(mid);
  if (mm) {  // wave-aggregated append to the mid list
    const int leader = __ffsll((long long)mm) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(b.mid_n, (uint32_t)__popcll(mm));
    base = __shfl(base, leader, 64);
    if (mid) b.mid_list[base + (uint32_t)__popcll(mm & ((1ull << lane) - 1ull))] = (uint32_t)a;
  }
  if (c == 0u) return;
  const int* kr = b.knn + (size_t)a * b.k;
  for (int q = 0; q < b.k; q += 4) {
    int4 c4 = *(const int4*)(kr + q);
    b.flags[c4.x] = 1; b.flags[c4.y] = 1; b.flags[c4.z] = 1; b.flags[c4.w] = 1;
  }
  if (mid) return;
  const uint32_t st = b.starts[a];
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
      b.dest[idx[j]] = st + r;
    }
  }
}

// one wave per bucket with more than kLaneRank members
__global__ __launch_bounds__(kBlock) void k_bucket_mid(BucketArgs b, int n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nb = *b.mid_n;
  const uint32_t nw = gridDim.x * kWaves;
  for (uint32_t w = blockIdx.x * kWaves + (threadIdx.x >> 6); w < nb; w += nw) {
    const uint32_t a = b.mid_list[w];
    const uint32_t c = b.counts[a], st = b.starts[a];
    if (c <= (uint32_t)kRankMax) {
      for (uint32_t j0 = 0; j0 < c; j0 += 64) {
        uint32_t v = (j0 + lane < c) ? b.slot_idx[st + j0 + lane] : 0xffffffffu;
        uint32_t rank = 0;
        for (uint32_t k0 = 0; k0 < c; k0 += 64) {
          uint32_t u = (k0 + lane < c) ? b.slot_idx[st + k0 + lane] : 0xffffffffu;
          for (int jj = 0; jj < 64; ++jj) rank += (__shfl(u, jj, 64) < v) ? 1u : 0u;
        }
        if (j0 + lane < c) b.dest[v] = st + rank;
      }
    } else {  // in-order compaction over all keys
      uint32_t pos = st;
      for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const bool hit = i < n && b.keys[i] == a;
        const unsigned long long m = __ballot(hit);
        if (hit) b.dest[i] = pos + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        pos += (uint32_t)__popcll(m);
      }
    }
  }
}

// every valid point record to its bucket-ordered destination
__global__ __launch_bounds__(kBlock) void k_gather(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ dest,
                                                   int n, int n_bins, const PointRec* __restrict__ recs,
                                                   PointRec* __restrict__ recs_s) {
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    if (keys[i] < (uint32_t)n_bins) recs_s[dest[i]] = recs[i];
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
  cert[0] = v[0]; cert[1] = v[1]; cert[2] = v[2]; cert[3] = v[3]; cert[4] = mx;
}

// ---------------------------------------------------------------- row 7 helpers (Matrix-Fisher)
// Per bin (matrix_fisher_evidence.py:181-211): w_b = sqrt(N_s N_m + eps), u = S/(|S|+eps),
// conf = Rbar_s Rbar_m, H += w_b conf u_map u_scan^T; out[9] += w_b conf; out[10] += N_s.
__device__ __forceinline__ void mf_bin_term(double Ns, double sx, double sy, double sz, const double* __restrict__ map,
                                            int B, int b, double* out /*11*/) {
  const size_t Bs = (size_t)B;
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
    for (int j = 0; j < 3; ++j) out[3 * i + j] += wf * um[i] * us[j];
  out[9] += wf;
  out[10] += Ns;
}

// H (9), sum w conf, sum N_s -> scalars; 3x3 SVD and the det-fixed R_mf (:215-222) on one thread
__device__ void mf_finish(const double* v, double* scalars) {
  for (int k = 0; k < 9; ++k) scalars[SC_MF_H + k] = v[k];
  scalars[SC_MF_NEFF] = v[9];
  scalars[SC_MF_SCANN] = v[10];
  double U[9], s[3], V[9];
  svd3(v, U, s, V);
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

// fused bin-kernel partial: [sum N, sum N^2, sum N/(N+eps), sum psd delta, max eps ratio | MF 11]
constexpr int kBinNV = 16;

// ---------------------------------------------------------------- row 5+6 scale mode: bin-centric
// One 256-thread workgroup per tile of 64 consecutive bins.  Phase 1 compacts the tile's active
// bins (ballot).  Phase 2: a 4-lane group per active bin (all 64 bins of a tile in flight);
// lane l owns the bin's reverse-kNN buckets l, l+4, ... and streams each bucket's contiguous
// records (ascending point index); the 4 lane sums meet in a fixed xor tree.  Phase 3: the
// first wave finalizes the 64 bins (PSD, kappa) and streams the 26 field-major outputs.
constexpr int kTile = 64;
constexpr int kGroup = 4;
__global__ __launch_bounds__(kBlock) void k_bins_scale(BinKernelArgs a, double* partials) {
  __shared__ double sums[19 * kTile];
  __shared__ int active[kTile];
  __shared__ int n_active;
  __shared__ double lds[kWaves * kBinNV];
  const int t = threadIdx.x;
  const int b0 = blockIdx.x * kTile;
  for (int j = blockIdx.x * kBlock + t; j < a.n_zero_after; j += gridDim.x * kBlock) a.zero_after[j] = 0u;
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
    const int lb = active[j];
    const int bb = b0 + lb;
    const double4 bd = *(const double4*)(a.bin_dirs + 4 * (size_t)bb);
    double acc[19];
#pragma unroll
    for (int f = 0; f < 19; ++f) acc[f] = 0.0;
    const int q1 = a.rknn_off[bb + 1];
    // lane l owns reverse-kNN buckets l, l+4, ...; each bucket streams its contiguous records
    for (int q = a.rknn_off[bb] + l; q < q1; q += kGroup) {
      const uint32_t src = (uint32_t)a.rknn[q];
      const uint32_t c = a.counts[src];
      const PointRec* rp = a.recs_s + a.starts[src];
      for (uint32_t i = 0; i < c; ++i) {
        const PointRec pr = rp[i];
        double d[3] = {pr.dx, pr.dy, pr.dz};
        double p[3] = {pr.x, pr.y, pr.z};
        double sim = dot3_exact(d[0], d[1], d[2], bd.x, bd.y, bd.z);
        double r = exp((sim - pr.m) * inv_tau) * pr.iz;
        add_contrib(acc, pr.w * r, d, p);
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
  // phase 3: finalize + this bin's Matrix-Fisher term (row 7, matrix_fisher_evidence.py:181-211).
  // A bin with no scan mass contributes exact zeros to H, so only active bins read the map.
  double v[kBinNV];
#pragma unroll
  for (int f = 0; f < kBinNV; ++f) v[f] = 0.0;
  v[4] = -INFINITY;
  if (t < kTile && b0 + t < a.n_bins) {
    double r[19];
#pragma unroll
    for (int f = 0; f < 19; ++f) r[f] = sums[f * kTile + t];
    finalize_bin(r, a.scan, a.n_bins, b0 + t, v);
    if (a.flags[b0 + t]) mf_bin_term(r[0], r[1], r[2], r[3], a.map, a.n_bins, b0 + t, v + 5);
  }
  // block reduce: 4 sums, 1 max, 11 sums
  double s4[4] = {v[0], v[1], v[2], v[3]};
  block_sum<4>(s4, lds);
  double mx = block_max(v[4], lds);
  double m11[11];
#pragma unroll
  for (int f = 0; f < 11; ++f) m11[f] = v[5 + f];
  block_sum<11>(m11, lds);
  v[0] = s4[0]; v[1] = s4[1]; v[2] = s4[2]; v[3] = s4[3]; v[4] = mx;
#pragma unroll
  for (int f = 0; f < 11; ++f) v[5 + f] = m11[f];
  if (!finish_blocks<kBinNV, 16u>(v, partials, a.ticket, lds)) return;
  if (t == 0) {
    for (int f = 0; f < 5; ++f) a.scalars[SC_BIN_NSUM + f] = v[f];
    mf_finish(v + 5, a.scalars);
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
  if (!finish_blocks<5, 16u>(v5, partials, a.ticket, lds)) return;
  for (int f = 0; f < 5; ++f) cert[f] = v5[f];
  if (threadIdx.x == 0)
    for (int f = 0; f < 5; ++f) a.scalars[SC_BIN_NSUM + f] = cert[f];
}

// ---------------------------------------------------------------- row 7: Matrix-Fisher reduction
// Standalone form (dense mode and the per-operator entry point): H terms over every bin plus the
// map totals sum S_dir_scatter / sum N_dir (planar z precision, :572-587).  In the scale-mode
// scan the H terms are fused into k_bins_scale and the map totals come from the pushforward.
constexpr int kMfNV = 21;
__global__ __launch_bounds__(kBlock) void k_mf(const double* __restrict__ scan, const double* __restrict__ map, int B,
                                               double* partials, double* scalars, uint32_t* ticket) {
  __shared__ double lds[kWaves * kMfNV];
  double v[kMfNV];
#pragma unroll
  for (int k = 0; k < kMfNV; ++k) v[k] = 0.0;
  const size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    mf_bin_term(scan[SF_N * Bs + b], scan[SF_SD * Bs + b], scan[(SF_SD + 1) * Bs + b], scan[(SF_SD + 2) * Bs + b], map,
                B, b, v);
#pragma unroll
    for (int k = 0; k < 9; ++k) v[11 + k] += map[(MF_S + k) * Bs + b];
    v[20] += map[MF_ND * Bs + b];
  }
  block_sum<kMfNV>(v, lds);
  if (!finish_blocks<kMfNV, 0u>(v, partials, ticket, lds)) return;
  if (threadIdx.x == 0) {
    for (int k = 0; k < 9; ++k) scalars[SC_MF_MAPSCAT + k] = v[11 + k];
    scalars[SC_MF_MAPND] = v[20];
    mf_finish(v, scalars);
  }
}

// ---------------------------------------------------------------- row 8: planar translation
// Per bin (matrix_fisher_evidence.py:442-475): t_b = c_map - R p_scan,
// S_b = Sigma_map + R Sigma_scan R^T, W_b = w_b inv(S_b + eps I); L += W_b, h += W_b t_b.
constexpr int kPtNV = 13;
__global__ __launch_bounds__(kBlock) void k_pt(const double* __restrict__ scan, const double* __restrict__ map,
                                               const double* __restrict__ derived, int B, double* scalars,
                                               double* partials, uint32_t* ticket) {
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
  if (!finish_blocks<kPtNV, 0u>(v, partials, ticket, lds)) return;
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

// Map totals for the next scan's planar z precision (sum S_dir_scatter, sum N_dir over bins),
// reduced in fixed order by the last block.
constexpr int kTotNV = 10;
__device__ __forceinline__ void map_totals_finish(double (&tot)[kTotNV], double* lds, double* partials,
                                                  double* scalars, uint32_t* ticket) {
  block_sum<kTotNV>(tot, lds);
  if (!finish_blocks<kTotNV, 0u>(tot, partials, ticket, lds)) return;
  if (threadIdx.x == 0) {
    for (int k = 0; k < 9; ++k) scalars[SC_MF_MAPSCAT + k] = tot[k];
    scalars[SC_MF_MAPND] = tot[9];
  }
}

__global__ __launch_bounds__(kBlock) void k_pushforward(const double* __restrict__ scan, double* map, double* derived,
                                                        int B, PushArgs pa, double* partials, double* scalars,
                                                        uint32_t* ticket) {
  __shared__ double lds[kWaves * kTotNV];
  double tot[kTotNV];
#pragma unroll
  for (int k = 0; k < kTotNV; ++k) tot[k] = 0.0;
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
          double sn = g * map[(MF_S + 3 * i + j) * Bs + b] + v;
          map[(MF_S + 3 * i + j) * Bs + b] = sn;
          tot[3 * i + j] += sn;
        }
    }
    const double nd = g * map[MF_ND * Bs + b] + N;
    const double np = g * map[MF_NP * Bs + b] + N;
    map[MF_ND * Bs + b] = nd;
    map[MF_NP * Bs + b] = np;
    tot[9] += nd;
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
  map_totals_finish(tot, lds, partials, scalars, ticket);
}

// derived stats + map totals from map sufficient stats only (used after set_map / reset)
__global__ __launch_bounds__(kBlock) void k_map_derive(const double* __restrict__ map, double* derived, int B,
                                                       double* partials, double* scalars, uint32_t* ticket) {
  __shared__ double lds[kWaves * kTotNV];
  double tot[kTotNV];
#pragma unroll
  for (int k = 0; k < kTotNV; ++k) tot[k] = 0.0;
  const size_t Bs = (size_t)B;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < B; b += gridDim.x * kBlock) {
    double sd[3], sp[3], spp[9];
    for (int k = 0; k < 3; ++k) { sd[k] = map[(MF_SD + k) * Bs + b]; sp[k] = map[(MF_SP + k) * Bs + b]; }
    for (int k = 0; k < 9; ++k) { spp[k] = map[(MF_SPP + k) * Bs + b]; tot[k] += map[(MF_S + k) * Bs + b]; }
    tot[9] += map[MF_ND * Bs + b];
    derive_bin(sd, map[MF_ND * Bs + b], map[MF_NP * Bs + b], sp, spp, derived, Bs, b);
  }
  map_totals_finish(tot, lds, partials, scalars, ticket);
}

// ---------------------------------------------------------------- launchers
static int grid_for(long n, int cap_blocks) {
  long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > cap_blocks ? cap_blocks : g);
}
int push_blocks(int n_bins) { return grid_for(n_bins, 4096); }

hipError_t launch_budget(const BudgetArgs& a, int nblk, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_budget, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a);
  return hipGetLastError();
}

hipError_t launch_points(const PointKernelArgs& a, bool scale, double* partials, int nblk, hipStream_t s, hipEvent_t e0,
                         hipEvent_t e1) {
  if (scale) {
    switch (a.k) {
      case 8: hipExtLaunchKernelGGL(k_points<true, 8>, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a, partials); break;
      case 16: hipExtLaunchKernelGGL(k_points<true, 16>, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a, partials); break;
      case 32: hipExtLaunchKernelGGL(k_points<true, 32>, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a, partials); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    hipExtLaunchKernelGGL(k_points<false, 1>, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, a, partials);
  }
  return hipGetLastError();
}

int scan_tiles(int n_bins) { return (n_bins + kScanTile - 1) / kScanTile; }

hipError_t launch_bucketing(const BucketArgs& b, int n, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_scan, dim3(scan_tiles(b.n_bins)), dim3(kBlock), 0, s, e0, nullptr, 0,
                        (const uint32_t*)b.counts, b.n_bins, b.scan_status, b.scan_ticket, b.starts);
  hipLaunchKernelGGL(k_place, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, (const uint32_t*)b.keys,
                     (const uint32_t*)b.slots, (const uint32_t*)b.starts, n, b.n_bins, b.slot_idx);
  hipLaunchKernelGGL(k_bucket_rank, dim3((b.n_bins + kBlock - 1) / kBlock), dim3(kBlock), 0, s, b);
  hipLaunchKernelGGL(k_bucket_mid, dim3(256), dim3(kBlock), 0, s, b, n);
  hipExtLaunchKernelGGL(k_gather, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s, nullptr, e1, 0,
                        (const uint32_t*)b.keys, (const uint32_t*)b.dest, n, b.n_bins, (const PointRec*)b.recs,
                        b.recs_s);
  return hipGetLastError();
}

int bins_scale_blocks(int n_bins) { return (n_bins + kTile - 1) / kTile; }
int bins_partial_nv() { return kBinNV; }

hipError_t launch_bins_scale(const BinKernelArgs& a, double* partials, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_bins_scale, dim3(bins_scale_blocks(a.n_bins)), dim3(kBlock), 0, s, e0, e1, 0, a, partials);
  return hipGetLastError();
}

hipError_t launch_dense(const BinKernelArgs& a, double* bin_partials, double* partials, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1) {
  int nchunks = (a.cap + kBlock - 1) / kBlock;
  hipExtLaunchKernelGGL(k_dense_accum, dim3(nchunks), dim3(kBlock), 0, s, e0, nullptr, 0, a, bin_partials);
  int nblk = (a.n_bins + kBlock - 1) / kBlock;
  hipExtLaunchKernelGGL(k_dense_finalize, dim3(nblk), dim3(kBlock), 0, s, nullptr, e1, 0, a,
                        (const double*)bin_partials, nchunks, partials);
  return hipGetLastError();
}

hipError_t launch_mf(const double* scan, const double* map, int B, double* partials, int nblk, double* scalars,
                     uint32_t* ticket, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_mf, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, scan, map, B, partials, scalars, ticket);
  return hipGetLastError();
}

hipError_t launch_pt(const double* scan, const double* map, const double* derived, int B, double* partials, int nblk,
                     double* scalars, uint32_t* ticket, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_pt, dim3(nblk), dim3(kBlock), 0, s, e0, e1, 0, scan, map, derived, B, scalars, partials,
                        ticket);
  return hipGetLastError();
}

hipError_t launch_pushforward(const double* scan, double* map, double* derived, int B, const PushArgs& pa,
                              double* partials, double* scalars, uint32_t* ticket, hipStream_t s, hipEvent_t e0,
                              hipEvent_t e1) {
  hipExtLaunchKernelGGL(k_pushforward, dim3(push_blocks(B)), dim3(kBlock), 0, s, e0, e1, 0, scan, map, derived, B, pa,
                        partials, scalars, ticket);
  return hipGetLastError();
}

hipError_t launch_map_derive(const double* map, double* derived, int B, double* partials, double* scalars,
                             uint32_t* ticket, hipStream_t s) {
  hipLaunchKernelGGL(k_map_derive, dim3(push_blocks(B)), dim3(kBlock), 0, s, map, derived, B, partials, scalars,
                     ticket);
  return hipGetLastError();
}

}  // namespace gcs
