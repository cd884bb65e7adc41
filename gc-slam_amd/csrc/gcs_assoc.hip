// Primitive association by unbalanced optimal transport on gfx950 -- the live primitive path's
// second operator: associate_primitives_ot,
// FS/backend/operators/primitive_association.py:239-553.
//
//   k_as_prep      one lane per measurement row: mean position ((Lambda + eps I)^-1 theta, partial
//                  pivoting), resultant direction and kappa (measurement_batch.py:389-411), A_vmf of
//                  kappa, the MA-hex stencil tile ids (tiling.py:148-186, :309-336) and their index in
//                  the view's tile list (first match, -1 none: :338-344); one lane per view entry: A_vmf
//                  of its kappa and the valid count
//   k_as_pool      one workgroup per row: the row's pool (n_stencil x m_tile_view entries) costed
//                  (:351-365; ||dx||^2 + beta H^2_vMF, 1e12 where invalid or the tile is missing), the
//                  k_assoc smallest by (cost, pool position) -- lax.sort with num_keys=1 is stable on
//                  cost alone (:376) -- per-thread sorted lists merged by k rounds of a block argmin;
//                  then per candidate the unmasked cost + recency, row-min subtraction, addressing
//                  (:377-403)
//   k_as_sinkhorn  workgroup 0 (512 threads): marginals a (policy) and b (uniform), the optional median
//                  scaling, k_sinkhorn fixed unbalanced iterations (:105-138) with the K_mat rows in
//                  registers and the column sums in a fixed tree, pi, row masses, responsibilities and
//                  the OTCert / Support / Influence scalars (:465-551) into mapped host memory;
//                  workgroup 1, concurrently: the p95 order statistics of a and of the recency rows
//                  (8-pass radix selects)
// No floating-point atomics; every sum has a fixed order: bitwise reproducible.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <string>

#include "gcs_math.h"
#include "gcslam_hip.h"
#include "gcs_live.h"

namespace gcs {
namespace {

constexpr int kAsThreads = 256;
#ifndef GCS_POOL_THREADS
#define GCS_POOL_THREADS 128
#endif
constexpr int kPoolThreads = GCS_POOL_THREADS;
#ifndef GCS_POOL_FLAT
#define GCS_POOL_FLAT 1  // 0: each trip's position loads wait on its flag loads (A/B)
#endif
#ifndef GCS_POOL_PB
#define GCS_POOL_PB 8  // pool entries per thread and trip
#endif
// the Sinkhorn workgroup: 8 waves, 4 rows per thread at K <= 8 (K_mat rows in registers).  1024
// threads (4 waves per SIMD, 128 VGPRs: the rows spill) measured slower: 3.2 vs 3.0 us per iteration,
// 0.480 vs 0.422 ms per call (profiles/r03/assoc/)
#ifndef GCS_SH_THREADS
#define GCS_SH_THREADS 512
#endif
constexpr int kShThreads = GCS_SH_THREADS;
#ifndef GCS_SH_ONEBAR
// 1: v in every wave, one barrier per iteration -- no faster while v took a pow (profiles/r04/sh1/),
// 0.150 -> 0.144 ms per call with the Newton root (profiles/r05/assoc/); 0: v by wave 0 + a second barrier
#define GCS_SH_ONEBAR 1
#endif
#ifndef GCS_SH_LOGB
#define GCS_SH_LOGB 1  // 0: v = pow(b / K^T u, vb) with the quotient in every iteration (A/B)
#endif
#ifndef GCS_SH_TAB
#define GCS_SH_TAB 1  // 0: the loop's log / exp are log_fast / exp_fast (fdlibm forms with a divide; A/B)
#endif
#ifndef GCS_SH_ILV
#define GCS_SH_ILV 1  // 0: each row's u under its own branches (the chains one after another; A/B)
#endif
#ifndef GCS_SH_SPLIT
#define GCS_SH_SPLIT 1  // 0: log_tab / exp_tab called whole per row (their table reads not hoisted; A/B)
#endif
#ifndef GCS_SH_ZSKIP
#define GCS_SH_ZSKIP 1  // 0: zero-marginal rows take the fallback branch (A/B)
#endif
#ifndef GCS_SH_LOGA
#define GCS_SH_LOGA 1  // 0: u = pow(a / Kv, ua) with the quotient in every iteration (A/B)
#endif
#ifndef GCS_SH_DPP
#define GCS_SH_DPP 1  // 0: the Sinkhorn's reduce-scatter through ds_bpermute xor shuffles (A/B)
#endif
#ifndef GCS_SH_ROOT
#define GCS_SH_ROOT 1  // 0: no Newton root for exponents 1 / n (the log / exp tables every iteration; A/B)
#endif
constexpr int kShCR = 16 * 1024 / kShThreads;  // Sinkhorn row capacity: N <= kShCR * kShThreads / KM
constexpr int kMaxStencil = 64;
// GCS_SH_PROBE (timing probe builds only): wall-clock stamps of the Sinkhorn's phases, printed by the
// host call (stderr) -- workgroup 0: start, marginal, K_mat, loop end, end; workgroup 1: end
#ifndef GCS_SH_PROBE
#define GCS_SH_PROBE 0
#endif
#if GCS_SH_PROBE
__device__ unsigned long long g_sh_stamp[16];
#define SH_STAMP(k) do { if (threadIdx.x == 0) g_sh_stamp[k] = wall_clock64(); } while (0)
// the iteration's parts, summed over the iterations by thread 0 (u, K^T u + reduce-scatter, first
// barrier, v, second barrier + v read)
#define SH_ACC(k) do { const unsigned long long tn_ = wall_clock64(); sh_pa[k] += tn_ - sh_tp; sh_tp = tn_; } while (0)
#else
#define SH_STAMP(k) do { } while (0)
#define SH_ACC(k) do { } while (0)
#endif
constexpr double kLog4Pi = 2.5310242469692907;     // np.log(4.0 * np.pi)
constexpr double kLog2 = 0.6931471805599453;       // np.log(2.0)
constexpr double kSqrt3Half = 0.8660254037844386;  // jnp.sqrt(3.0) * 0.5 (:319)
constexpr double kCostInvalid = 1e12;              // :365
constexpr double kEigMin = 1e-12;                  // _compute_sparse_cost_matrix_jax eig_min
constexpr int kBitsPerAxis = 21;                   // tiling.py:80
constexpr int64_t kBias = 1LL << 20;               // tiling.py:81
constexpr int64_t kMask = (1LL << kBitsPerAxis) - 1;

struct AsParams {
  int n, m_view, m_shift, n_tiles, n_stencil, k, iters, m_pool;
  int s_center;  // the stencil entry (0, 0, 0): the row's own tile
  int a_policy, row_min, med;
  int fin_split;  // the finish (pi, responsibilities, certificate sums): GCS_SH_FINSPLIT's modes
  unsigned epoch; // this launch's hand-off value of the Sinkhorn's flag (never 0)
  double beta, eps, tau_a, tau_b, eps_mass, eps_lift, eps_dir, h, lam, eps_lam;
  long long scan_seq;
};

struct AsWork {
  double *pos, *dir, *kap, *A1, *A2, *dt;
  int32_t* tix;
  int32_t* cand;
  uint32_t* mvalid;       // this call's valid-entry count (k_as_prep adds, the Sinkhorn reads)
  uint32_t* mvalid_next;  // the next call's (zeroed by this call's Sinkhorn workgroup 0)
  float4* vc;             // k_as_stage: each view tile's valid entries, (x, y, z, slot) in f32 (k_as_pool_lds)
  int32_t* vcnt;          // k_as_stage: valid entries per view tile
  int32_t* order;         // k_as_stage: rows grouped by bucket, each bucket padded to a chunk (-1)
  int32_t *ctile, *cpre;  // k_as_stage: per chunk, its stencil tiles and the prefix of their valid counts (64 each)
  uint32_t* tcnt;         // k_as_prep: valid entries per view tile (read and re-armed by k_as_stage)
  double* kmat;           // the pools: K_mat = exp(-C / eps) beside the cost (read by the Sinkhorn when the
                          // median scaling is off: the exps run on the whole grid, not one workgroup)
  int chunk;              // rows per k_as_pool_lds workgroup (0: the buckets are not used)
  double* su;             // the Sinkhorn's scalings for k_as_finish: u (N), v (KM), sum a
  double* fpart;          // k_as_finish: per workgroup, its rows' certificate sums (7 + KM)
  uint32_t* ticket;       // k_as_finish: workgroups done (the last folds; re-armed by it)
  uint32_t* flag;         // the Sinkhorn workgroup's u / v hand-off to the finish workgroups (= epoch)
  uint32_t* cstat;        // the pools: per row, valid candidates | distinct tiles << 16 (cand_stats)
};

struct AsIn {
  const double *Lambdas, *thetas, *etas, *weights;
  const uint8_t* valid;
  int n_lobes;
  const int64_t* tile_ids;
  const double *vpos, *vdir, *vkap;
  const uint8_t* vvalid;
  const int64_t *vlast, *vtile;
  const int32_t* vslot;
};

struct AsOut {
  double *resp, *rmass, *cost;
  int32_t* cand;
  int64_t *tile, *slot;
  double* cert;  // mapped host
};

// A_vmf(k) = log(4 pi) + log sinh(k) - log k with the stable log-sinh (:141-149); k**3 is
// lax.integer_pow (k k k)
__device__ __forceinline__ double a_vmf(double k) {
#pragma clang fp contract(off)
  k = fmax(k, kEigMin);
  double ls;
  if (k > 20.0) ls = k - kLog2;
  else if (k >= 1e-2) ls = log(sinh(k));
  else ls = log(k + (k * k * k) / 6.0);
  return (kLog4Pi + ls) - log(k);
}

// cost of measurement (p, d, k, A1) against view entry e (:166-197)
__device__ __forceinline__ double pair_cost(const double* mp, const double* md, double mk, double A1,
                                            const double* __restrict__ vpos, const double* __restrict__ vdir,
                                            const double* __restrict__ vkap, const double* __restrict__ A2, int e,
                                            double beta) {
#pragma clang fp contract(off)
  const double dx = mp[0] - vpos[3 * e], dy = mp[1] - vpos[3 * e + 1], dz = mp[2] - vpos[3 * e + 2];
  const double d_pos = (dx * dx + dy * dy) + dz * dz;
  const double vk = vkap[e];
  const double s0 = mk * md[0] + vk * vdir[3 * e], s1 = mk * md[1] + vk * vdir[3 * e + 1],
               s2 = mk * md[2] + vk * vdir[3 * e + 2];
  const double km = 0.5 * sqrt((s0 * s0 + s1 * s1) + s2 * s2);
  const double bc = exp(a_vmf(fmax(km, kEigMin)) - 0.5 * (A1 + A2[e]));
  double d_dir = fmax(0.0, 1.0 - bc);
  if (!(mk > 0.0 && vk > 0.0)) d_dir = 0.0;
  return d_pos + beta * d_dir;
}

// total order of doubles as unsigned keys (NaN last, as lax.sort / numpy argsort place it)
__device__ __forceinline__ unsigned long long order_key(double x) {
  if (isnan(x)) return ~0ULL;
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}

// inverse of order_key (the empty key ~0 gives NaN, which compares false)
__device__ __forceinline__ double key_value(unsigned long long k) {
  if (k == ~0ULL) return NAN;
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k));
}

__device__ __forceinline__ int64_t pack_tile(int64_t c1, int64_t c2, int64_t cz) {
  return (((c1 + kBias) & kMask) << (2 * kBitsPerAxis)) | (((c2 + kBias) & kMask) << kBitsPerAxis) |
         ((cz + kBias) & kMask);
}

// x = (L + eps I)^-1 th: Gaussian elimination with partial pivoting (jnp.linalg.solve is LU)
__device__ __forceinline__ void solve3_pivot(const double* L, double eps, const double* th, double* x) {
#pragma clang fp contract(off)
  double A[3][4];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) A[r][c] = L[3 * r + c] + (r == c ? eps : 0.0);
    A[r][3] = th[r];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int pr = c;
#pragma unroll
    for (int r = c + 1; r < 3; ++r)
      if (fabs(A[r][c]) > fabs(A[pr][c])) pr = r;
    if (pr != c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double tmp = A[c][q];
        A[c][q] = A[pr][q];
        A[pr][q] = tmp;
      }
#pragma unroll
    for (int r = c + 1; r < 3; ++r) {
      const double f = A[r][c] / A[c][c];
#pragma unroll
      for (int q = c; q < 4; ++q) A[r][q] = A[r][q] - f * A[c][q];
    }
  }
  x[2] = A[2][3] / A[2][2];
  x[1] = (A[1][3] - A[1][2] * x[2]) / A[1][1];
  x[0] = ((A[0][3] - A[0][1] * x[1]) - A[0][2] * x[2]) / A[0][0];
}

// one lane of the prep: row lanes g < n (mean position, direction, kappa, A_vmf, the stencil tiles'
// view indices), view lanes n <= g < n + m_pool (A_vmf of the entry's kappa, the valid counts)
__device__ __forceinline__ void prep_lane(const AsIn& in, const AsParams& p, const AsWork& w,
                                          const int8_t* __restrict__ st, int g, const int64_t* s_tid, bool lds_tiles,
                                          bool count_tiles) {
#pragma clang fp contract(off)
  if (g < p.n) {
    const int i = g;
    double L[9], th[3], x[3];
    for (int k = 0; k < 9; ++k) L[k] = in.Lambdas[9 * i + k];
    for (int k = 0; k < 3; ++k) th[k] = in.thetas[3 * i + k];
    solve3_pivot(L, p.eps_lift, th, x);
    double es[3];
    for (int c = 0; c < 3; ++c) es[c] = in.etas[(size_t)i * in.n_lobes * 3 + c];
    for (int b = 1; b < in.n_lobes; ++b)
      for (int c = 0; c < 3; ++c) es[c] = es[c] + in.etas[((size_t)i * in.n_lobes + b) * 3 + c];
    const double kap = sqrt((es[0] * es[0] + es[1] * es[1]) + es[2] * es[2]);
    for (int c = 0; c < 3; ++c) {
      w.pos[3 * i + c] = x[c];
      w.dir[3 * i + c] = es[c] / (kap + p.eps_dir);
    }
    w.kap[i] = kap;
    w.A1[i] = a_vmf(fmax(kap, kEigMin));
    // stencil tiles (:317-336) and their view tile index (first match, :341-344)
    const double s1 = x[0];
    const double s2 = x[0] * 0.5 + x[1] * kSqrt3Half;
    const int64_t c1 = (int64_t)floor(s1 / p.h), c2 = (int64_t)floor(s2 / p.h), cz = (int64_t)floor(x[2] / p.h);
    // eight stencil tiles per sweep over the view's tile list (the first match of each kept): the
    // tile loads do not depend on a compare (a search per stencil tile with an early exit was a
    // chain of dependent loads)
    for (int s0 = 0; s0 < p.n_stencil; s0 += 8) {
      int64_t id[8];
      int hit[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s = s0 + j < p.n_stencil ? s0 + j : s0;
        id[j] = pack_tile(c1 + st[3 * s], c2 + st[3 * s + 1], cz + st[3 * s + 2]);
        hit[j] = -1;
      }
      for (int q = p.n_tiles - 1; q >= 0; --q) {  // backwards: the last write is the first match
        const int64_t v = lds_tiles ? s_tid[q] : in.tile_ids[q];
#pragma unroll
        for (int j = 0; j < 8; ++j) hit[j] = v == id[j] ? q : hit[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s0 + j < p.n_stencil) w.tix[(size_t)i * p.n_stencil + s0 + j] = hit[j];
      }
    }
  }
  // the view lanes: A_vmf of the entry's kappa; the valid count (and per view tile, for k_as_stage's
  // chunk records), one integer add per wave and tile (order-free)
  const int e = g - p.n;
  const bool vl = g >= p.n && g < p.n + p.m_pool;
  const bool vv = vl && in.vvalid[e] != 0;
  if (vl) w.A2[e] = a_vmf(fmax(in.vkap[e], kEigMin));
  const unsigned long long vm = __ballot(vv);
  const int lane = threadIdx.x & 63;
  if (vm != 0ull) {
    const int first = __ffsll((long long)vm) - 1;
    if (lane == first) atomicAdd(w.mvalid, (unsigned)__popcll(vm));
    if (w.chunk && count_tiles) {
      const int te = vv ? e / p.m_view : -1;
      const int t0 = __shfl(te, first, 64);
      if (__ballot(vv && te != t0) == 0ull) {
        if (lane == first) atomicAdd(&w.tcnt[t0], (unsigned)__popcll(vm));
      } else if (vv) {
        atomicAdd(&w.tcnt[te], 1u);
      }
    }
  }
}

__global__ __launch_bounds__(kAsThreads) void k_as_prep(AsIn in, AsParams p, AsWork w, const int8_t* __restrict__ st) {
  const int g = blockIdx.x * kAsThreads + threadIdx.x;
  // the view's tile ids in LDS (broadcast reads) for the stencil lookups of the row lanes
  constexpr int kLdsTiles = 256;
  __shared__ int64_t s_tid[kLdsTiles];
  const bool lds_tiles = p.n_tiles <= kLdsTiles;
  if (lds_tiles && blockIdx.x * kAsThreads < p.n) {
    for (int q = threadIdx.x; q < p.n_tiles; q += kAsThreads) s_tid[q] = in.tile_ids[q];
    __syncthreads();
  }
  prep_lane(in, p, w, st, g, s_tid, lds_tiles, true);
}

template <int KM>
__device__ __forceinline__ void list_insert(unsigned long long (&key)[KM], int (&idx)[KM], unsigned long long k, int p) {
  // sorted ascending by (key, idx); the new entry is dropped if it is not below the last
  if (k > key[KM - 1] || (k == key[KM - 1] && p >= idx[KM - 1])) return;
  key[KM - 1] = k;
  idx[KM - 1] = p;
#pragma unroll
  for (int j = KM - 1; j > 0; --j) {
    const bool sw = key[j] < key[j - 1] || (key[j] == key[j - 1] && idx[j] < idx[j - 1]);
    if (sw) {
      const unsigned long long tk = key[j];
      key[j] = key[j - 1];
      key[j - 1] = tk;
      const int ti = idx[j];
      idx[j] = idx[j - 1];
      idx[j - 1] = ti;
    }
  }
}

__device__ __forceinline__ bool kless(unsigned long long ka, int pa, unsigned long long kb, int pb) {
  return ka < kb || (ka == kb && pa < pb);
}

// one workgroup per measurement row: kPoolThreads = 128 (two waves) puts all 1,536 rows of the reference
// sizes in flight at once (eight workgroups per CU by registers and LDS); 256 threads took two rounds
// of workgroups (GCS_POOL_THREADS=256 for A/B; any split of the pool over the lanes gives the same
// candidates, see the merge below)
template <int KM>
__global__ __launch_bounds__(kPoolThreads) void k_as_pool(AsIn in, AsParams p, AsWork w, AsOut o) {
#pragma clang fp contract(off)
  __shared__ int s_tix[kMaxStencil];
  __shared__ unsigned long long s_wk[2][kPoolThreads / 64];
  __shared__ int s_wp[2][kPoolThreads / 64];
  __shared__ int s_sel[32];
  __shared__ double s_thr[kPoolThreads / 64];
  // per wave: the ring of entries past the threshold (d_pos, pool position, view index)
  constexpr unsigned kRing = 512;  // >= 63 pending + PB x 64 appended per trip
  __shared__ double s_rd[kPoolThreads / 64][kRing];
  __shared__ int s_rq[kPoolThreads / 64][kRing], s_re[kPoolThreads / 64][kRing];
  const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool row_valid = in.valid[i] != 0;
  if (t < p.n_stencil) s_tix[t] = w.tix[(size_t)i * p.n_stencil + t];
  __syncthreads();
  const double mp[3] = {w.pos[3 * i], w.pos[3 * i + 1], w.pos[3 * i + 2]};
  const double md[3] = {w.dir[3 * i], w.dir[3 * i + 1], w.dir[3 * i + 2]};
  const double mk = w.kap[i], A1 = w.A1[i];
  if (row_valid) {
    unsigned long long key[KM];
    int idx[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      key[j] = ~0ULL;
      idx[j] = 0x7fffffff;
    }
    const bool prune = p.beta >= 0.0;
    // PB pool entries per trip, in increasing pool position: their flag and position loads issue
    // together, none behind another's result (the pass is bound by L2 round trips, not VALU)
    constexpr int PB = GCS_POOL_PB;
    // Block threshold (beta >= 0): cost = d_pos + beta d_dir lies in [d_pos, d_pos + beta] (d_dir in
    // [0, 1], rounding monotone), so with D an upper bound of the row's K-th smallest valid d_pos at
    // least K entries cost <= D + beta: an entry with d_pos > D + beta cannot be selected and needs no
    // vMF term.  D: per thread the smallest d_pos of its share; per wave the K-th smallest of those
    // (K rounds of a wave min, K distinct entries at or below it); the block's smallest wave value.
    // Without it every thread's first K entries took full costs (2,048 per row).
    double thr = INFINITY;
    const int S = p.n_stencil, MV = p.m_view;
    if (prune) {
      // The bound from the row's own stencil tile first (its nearest entries are mostly there; a
      // bound from any subset of the pool is still an upper bound), from every stencil tile only
      // when that one leaves it infinite.  Tile-major: the stencil tile of a trip is uniform.
      for (int round = 0; round < 2 && thr == INFINITY; ++round) {
        double dmin = INFINITY;
        for (int sq = round == 0 ? p.s_center : 0; sq < (round == 0 ? p.s_center + 1 : S); ++sq) {
          const int ti = sq >= 0 ? s_tix[sq] : -1;
          if (ti < 0) continue;
          const size_t base = (size_t)ti * MV;
          for (int o = t; o < MV; o += PB * kPoolThreads) {
#if GCS_POOL_FLAT
            uint8_t vv[PB];
            double px[PB], py[PB], pz[PB];
#pragma unroll
            for (int u = 0; u < PB; ++u) {  // every load of the trip first (in-range entries only)
              const int oo = o + u * kPoolThreads;
              const size_t e = base + (oo < MV ? oo : 0);
              vv[u] = oo < MV ? in.vvalid[e] : 0;
              px[u] = in.vpos[3 * e];
              py[u] = in.vpos[3 * e + 1];
              pz[u] = in.vpos[3 * e + 2];
            }
#pragma unroll
            for (int u = 0; u < PB; ++u) {
              if (!vv[u]) continue;
              const double dx = mp[0] - px[u], dy = mp[1] - py[u], dz = mp[2] - pz[u];
              dmin = fmin(dmin, (dx * dx + dy * dy) + dz * dz);
            }
#else
#pragma unroll
            for (int u = 0; u < PB; ++u) {
              const int oo = o + u * kPoolThreads;
              if (oo >= MV) break;
              const size_t e = base + oo;
              if (!in.vvalid[e]) continue;
              const double dx = mp[0] - in.vpos[3 * e], dy = mp[1] - in.vpos[3 * e + 1],
                           dz = mp[2] - in.vpos[3 * e + 2];
              dmin = fmin(dmin, (dx * dx + dy * dy) + dz * dz);
            }
#endif
          }
        }
        double kth = INFINITY, cur = dmin;
        for (int r = 0; r < p.k; ++r) {  // the r-th smallest lane minimum, lanes popped in turn
          double m = cur;
#pragma unroll
          for (int sh = 32; sh >= 1; sh >>= 1) m = fmin(m, __shfl_xor(m, sh, 64));
          kth = m;
          const unsigned long long hit = __ballot(cur == m);
          if (lane == __ffsll((long long)hit) - 1) cur = INFINITY;  // one lane per round
        }
        if (lane == 0) s_thr[wid] = kth;
        __syncthreads();
        double d = s_thr[0];
#pragma unroll
        for (int v = 1; v < kPoolThreads / 64; ++v) d = fmin(d, s_thr[v]);
        __syncthreads();  // (s_thr is written again by a second round)
        thr = d + p.beta;  // (inf when every wave has fewer than K valid entries: the second round)
      }
    }
    // Second pass, compacted: the entries that pass the block threshold go into the wave's ring (in
    // increasing pool position) and are costed 64 at a time, one per lane, so the vMF term and the
    // list insert run with every lane busy instead of once per trip whenever any lane has one.  Any
    // partition of the entries over the lanes' lists gives the same K smallest (cost, position)
    // after the merge below; each lane still takes its entries in increasing position.  Entries
    // that are invalid or in a missing tile enter the visiting lane's list with the invalid cost.
    double* rd = s_rd[wid];
    int* rq = s_rq[wid];
    int* re = s_re[wid];
    unsigned head = 0, tail = 0;  // wave-uniform ring counters
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    auto take = [&](int n) {  // lanes < n cost ring entry head + lane
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < n) {
        const unsigned slot = (head + lane) & (kRing - 1);
        const double d_pos = rd[slot];
        const int q = rq[slot], e = re[slot];
        if (!(prune && d_pos > key_value(key[KM - 1])))
          list_insert<KM>(key, idx, order_key(pair_cost(mp, md, mk, A1, in.vpos, in.vdir, in.vkap, w.A2, e, p.beta)),
                          q);
      }
      head += n;
    };
    for (int sq = 0; sq < S; ++sq) {
      const int ti = s_tix[sq];
      const size_t base = (size_t)(ti < 0 ? 0 : ti) * MV;
      for (int ow = t & ~63; ow < MV; ow += PB * kPoolThreads) {  // wave-uniform trips (ballots inside)
#if GCS_POOL_FLAT
        uint8_t vv[PB];
        double px[PB], py[PB], pz[PB];
#pragma unroll
        for (int u = 0; u < PB; ++u) {  // every load of the trip first (a missing tile reads tile 0)
          const int oo = ow + lane + u * kPoolThreads;
          const size_t e = base + (oo < MV ? oo : 0);
          vv[u] = oo < MV && ti >= 0 ? in.vvalid[e] : 0;
          px[u] = in.vpos[3 * e];
          py[u] = in.vpos[3 * e + 1];
          pz[u] = in.vpos[3 * e + 2];
        }
#endif
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const int oo = ow + lane + u * kPoolThreads;
          const bool in_tile = oo < MV;
          const int q = sq * MV + oo;
          bool valid = false;
          double d_pos = 0.0;
#if GCS_POOL_FLAT
          if (in_tile && vv[u]) {
            const double dx = mp[0] - px[u], dy = mp[1] - py[u], dz = mp[2] - pz[u];
#else
          if (in_tile && ti >= 0 && in.vvalid[base + oo]) {
            const size_t e = base + oo;
            const double dx = mp[0] - in.vpos[3 * e], dy = mp[1] - in.vpos[3 * e + 1], dz = mp[2] - in.vpos[3 * e + 2];
#endif
            d_pos = (dx * dx + dy * dy) + dz * dz;
            valid = true;
          } else if (in_tile) {
            list_insert<KM>(key, idx, order_key(kCostInvalid), q);
          }
          // cost = d_pos + beta d_dir >= d_pos (beta >= 0, d_dir >= 0): past the threshold no entry
          // can be selected
          const bool keep = valid && !(prune && d_pos > thr);
          const unsigned long long m = __ballot(keep);
          if (keep) {
            const unsigned slot = (tail + (unsigned)__popcll(m & lt_mask)) & (kRing - 1);
            rd[slot] = d_pos;
            rq[slot] = q;
            re[slot] = (int)(base + oo);
          }
          tail += (unsigned)__popcll(m);
        }
        while (tail - head >= 64u) take(64);
      }
    }
    if (tail != head) take((int)(tail - head));
    // k rounds of a block argmin over the lists' heads; the winner's owner pops its head
    for (int r = 0; r < p.k; ++r) {
      unsigned long long bk = key[0];
      int bp = idx[0];
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) {
        const unsigned long long ok = __shfl_xor(bk, sh, 64);
        const int op = __shfl_xor(bp, sh, 64);
        if (kless(ok, op, bk, bp)) {
          bk = ok;
          bp = op;
        }
      }
      const int buf = r & 1;
      if (lane == 0) {
        s_wk[buf][wid] = bk;
        s_wp[buf][wid] = bp;
      }
      __syncthreads();
      bk = s_wk[buf][0];
      bp = s_wp[buf][0];
#pragma unroll
      for (int v = 1; v < kPoolThreads / 64; ++v)
        if (kless(s_wk[buf][v], s_wp[buf][v], bk, bp)) {
          bk = s_wk[buf][v];
          bp = s_wp[buf][v];
        }
      if (t == 0) s_sel[r] = bp;
      if (idx[0] == bp && key[0] == bk) {  // pool positions are unique: exactly one owner
#pragma unroll
        for (int j = 0; j < KM - 1; ++j) {
          key[j] = key[j + 1];
          idx[j] = idx[j + 1];
        }
        key[KM - 1] = ~0ULL;
        idx[KM - 1] = 0x7fffffff;
      }
    }
    __syncthreads();
  }
  if (wid != 0) return;
  // per candidate (lane k < K): view index, unmasked cost + recency, row min (:377-403)
  const bool act = lane < p.k;
  int e = 0;
  if (act && row_valid) {
    const int q = s_sel[lane];
    const int ti = s_tix[q / p.m_view];
    e = (ti < 0 ? 0 : ti) * p.m_view + q % p.m_view;
  }
  double c = INFINITY, dt = 0.0;
  if (act) {
    c = pair_cost(mp, md, mk, A1, in.vpos, in.vdir, in.vkap, w.A2, e, p.beta);
    const long long last = (long long)in.vlast[e];
    dt = (double)(p.scan_seq - last > 0 ? p.scan_seq - last : 0);
    c = c + p.eps_lam * dt;
  }
  double mn = c;
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) mn = fmin(mn, __shfl_xor(mn, sh, 64));
  if (act) {
    if (p.row_min) c = c - mn;
    const size_t o_ = (size_t)i * p.k + lane;
    o.cost[o_] = c;
    if (!p.med) w.kmat[o_] = exp(-c / fmax(p.eps, 1e-12));  // (the Sinkhorn's own expression)
    w.cand[o_] = e;
    w.dt[o_] = dt;
    if (o.cand) o.cand[o_] = e;
    if (o.tile) o.tile[o_] = in.vtile[e];
    if (o.slot) o.slot[o_] = (int64_t)in.vslot[e];
  }
  {  // the MapUpdateCert's per-row candidate statistics (cand_stats): valid candidates, distinct tiles
    const bool cv = act && row_valid && in.vvalid[e] != 0;
    const long long tile = cv ? (long long)in.vtile[e] : -1;
    bool seen = false;
    for (int k2 = 0; k2 < p.k; ++k2) {  // (every lane: the shuffles read lanes < K)
      const long long t2 = __shfl(tile, k2, 64);
      seen = seen || (k2 < lane && t2 != -1 && t2 == tile);
    }
    const unsigned cnt = (unsigned)__popcll(__ballot(cv));
    const unsigned dist = (unsigned)__popcll(__ballot(cv && tile != -1 && !seen));
    if (lane == 0) w.cstat[i] = cnt | (dist << 16);
  }
}

// The pool by center-tile bucket (GCS_POOL_LDS).  Rows whose own tile is view tile c share their
// stencil's view tiles (the stencil is a fixed offset set around the row's cell), so the rows are
// grouped by c (k_as_stage lays them out, each bucket padded to a chunk of kPoolLdsWaves rows) and a
// workgroup of kPoolLdsWaves waves stages its chunk's stencil tiles in LDS once and each wave selects
// one row's K candidates from them (k_as_pool, one workgroup per row, re-read 25 B per entry from L2
// for every row).  The staged tiles hold only their VALID entries (k_as_stage compacts each view tile:
// f32 position + the entry's slot in the tile, 16 B), so a row's pass visits the ~30 % of the pool
// that can be selected.  Invalid entries and missing tiles carry the invalid cost (1e12) and enter
// the selection only when fewer than K valid entries cost less than that: the row's K-th selected key
// then reaches order_key(1e12) and the row is selected again over every pool position, exactly as
// k_as_pool does (a rare slow path).  Rows whose own tile is not in the view (bucket -1) or stencils
// too large for LDS read the compacted table from L2.
//
// The f32 distances only prune; what is selected is decided on the exact f64 costs, so the
// candidates are k_as_pool's (bit-exact indices).  With m32, v32 the f32 roundings (2^-24 relative
// per axis), |v| <= |m| + |m - v|, the f32 difference and sum of squares (a few 2^-24 relative), the
// exact distance de and the table distance da = sqrt(d32) satisfy, with E = 2^-20 |m|_1 + 1e-30:
//   de <= (da + E)(1 + 2^-19),  de >= (da - E)(1 - 2^-19)   (margins ~4x the rounding terms).
// The bound D (an upper bound of the row's K-th smallest valid d_pos) comes from upper bounds of the
// table distances (an order statistic of entrywise upper bounds bounds the exact one); an entry is
// pruned only when its lower bound exceeds D + beta (threshold rounded up into f32); the list-max skip
// uses the exact d_pos.  One wave per row: the lists' merge needs no block barrier.
#ifndef GCS_POOL_LDS
#define GCS_POOL_LDS 1
#endif
constexpr int kPoolLdsWaves = 8;
constexpr int kLRing = 256;  // per wave: >= 63 pending + kLdsPB x 64 appended per trip
constexpr int kLdsPB = 2;
constexpr int kPoolLdsMaxView = (160 * 1024 - kPoolLdsWaves * kLRing * 8) / 16;  // 9,216 stencil slots
constexpr int kMaxBuckets = 4096;
constexpr int kBucketRows = 4;
// GCS_POOL_PROBE (timing probe builds only): per row, wall-clock stamps of k_as_pool_lds's phases
// (block start, staged, pass 1, ring + costing, merge, slow path, end) and the ring count, printed by
// the host collect (stderr)
#ifndef GCS_POOL_PROBE
#define GCS_POOL_PROBE 0
#endif
#if GCS_POOL_PROBE
__device__ unsigned long long g_pool_probe[4096 * 10];
#define PP_STAMP(k) do { if (lane == 0) g_pool_probe[(size_t)i * 10 + (k)] = wall_clock64(); } while (0)
#else
#define PP_STAMP(k) do { } while (0)
#endif  // rows per k_as_stage thread: <= 4,096 rows (the Sinkhorn caps them at 2,048)

// workgroups 0..n_tiles-1: view tile b's valid entries in slot order (a block scan of wave ballots)
// into vc[b MV ..] as (x, y, z, slot) in f32, their count in vcnt[b].  Workgroup n_tiles: each row's
// slot in its bucket (LDS counters), bucket b's padded start (exclusive scan of ceil(count / chunk) x
// chunk), the order list (-1 everywhere first), every row at its bucket's start + its slot.
// view tile tb's valid entries in slot order (a block scan of wave ballots, 1,024 threads) into
// vc[tb MV ..] as (x, y, z, slot) in f32, their count in vcnt[tb]
__device__ __forceinline__ void compact_tile(const AsIn& in, const AsParams& p, const AsWork& w, int tb,
                                             uint32_t* s_wsum /*16*/) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int MV = p.m_view;
  uint32_t base = 0;
  for (int c0 = 0; c0 < MV; c0 += 1024) {
    const int oo = c0 + t;
    const size_t e = (size_t)tb * MV + oo;
    const bool v = oo < MV && in.vvalid[e] != 0;
    const unsigned long long bm = __ballot(v);
    if (lane == 0) s_wsum[wid] = (uint32_t)__popcll(bm);
    __syncthreads();
    uint32_t off = base + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull)), tot = 0;
    for (int q = 0; q < 16; ++q) {
      const uint32_t c = s_wsum[q];
      if (q < wid) off += c;
      tot += c;
    }
    if (v)
      w.vc[(size_t)tb * MV + off] = make_float4((float)in.vpos[3 * e], (float)in.vpos[3 * e + 1],
                                                (float)in.vpos[3 * e + 2], (float)oo);
    base += tot;
    __syncthreads();  // (s_wsum is rewritten by the next chunk)
  }
  if (t == 0) w.vcnt[tb] = (int32_t)base;
}

__global__ __launch_bounds__(1024) void k_as_stage(AsIn in, AsParams p, AsWork w, int nb, int cap) {
  __shared__ uint32_t s_wsum[16];
  __shared__ uint32_t s_cnt[kMaxBuckets];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int MV = p.m_view;
  if ((int)blockIdx.x < p.n_tiles) {
    compact_tile(in, p, w, blockIdx.x, s_wsum);
    return;
  }
  const int C = w.chunk, S = p.n_stencil;
  constexpr int kPer = kMaxBuckets / 1024;
  __shared__ uint32_t s_tc[kMaxBuckets];  // valid entries per view tile
  for (int b = t; b < nb; b += 1024) s_cnt[b] = 0u;
  for (int q = t; q < cap; q += 1024) w.order[q] = -1;
  __syncthreads();
  for (int b = t; b < p.n_tiles; b += 1024) {  // k_as_prep's per-tile valid counts, re-armed for the next call
    s_tc[b] = w.tcnt[b];
    w.tcnt[b] = 0u;
  }
  int rb[kBucketRows];
  uint32_t rs[kBucketRows];
#pragma unroll
  for (int j = 0; j < kBucketRows; ++j) {
    const int i = t + j * 1024;
    rb[j] = 0;
    rs[j] = 0u;
    if (i < p.n) {
      rb[j] = (p.s_center >= 0 ? w.tix[(size_t)i * S + p.s_center] : -1) + 1;
      rs[j] = atomicAdd(&s_cnt[rb[j]], 1u);  // (arrival order: any -- each row's result is its own)
    }
  }
  __syncthreads();
  uint32_t pc[kPer], mine = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = t * kPer + q;
    pc[q] = b < nb ? (s_cnt[b] + (uint32_t)C - 1u) / (uint32_t)C * (uint32_t)C : 0u;
    mine += pc[q];
  }
  uint32_t inc = mine;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) s_wsum[wid] = inc;
  __syncthreads();
  uint32_t run = inc - mine;
  for (int v = 0; v < wid; ++v) run += s_wsum[v];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = t * kPer + q;
    if (b < nb) s_cnt[b] = run << 12;  // (the bucket's first slot in the order list)
    run += pc[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBucketRows; ++j) {
    const int i = t + j * 1024;
    if (i < p.n) w.order[(s_cnt[rb[j]] >> 12) + rs[j]] = i;
  }
  __syncthreads();
  // every chunk's record -- its stencil tiles (its first row's tix: rows of a bucket share them) and
  // the inclusive prefix of their valid counts -- so k_as_pool_lds reads one record and the compacted
  // entries (two round trips).  One (chunk, slot) per thread and pass: the loads of a pass are
  // independent (no store between them)
  const int nch = cap / C, np = nch * S;
  for (int q = t; q < np; q += 1024) {
    const int c = q / S, sq = q - c * S;
    const int row = w.order[c * C];
    w.ctile[(size_t)c * 64 + sq] = row >= 0 ? w.tix[(size_t)row * S + sq] : -1;
  }
  __syncthreads();
  for (int q = t; q < np; q += 1024) {
    const int c = q / S, sq = q - c * S;
    int pre = 0;
    for (int s2 = 0; s2 <= sq; ++s2) {
      const int tj = w.ctile[(size_t)c * 64 + s2];
      pre += tj >= 0 ? (int)s_tc[tj] : 0;
    }
    w.cpre[(size_t)c * 64 + sq] = pre;
  }
}

// GCS_PREP_FUSED: k_as_prep and k_as_stage as one launch for views of at most kFusedTiles tiles
// (1,024-thread blocks): the prep's row and view lanes, one block per view tile compacting it, and one
// block that buckets the rows.  That block cannot read the row lanes' results (same launch), so it
// recomputes what it needs from the inputs with the same device code: each row's mean position and
// own tile (bitwise the row lanes' values), the view tiles' valid counts, and per bucket the stencil
// tiles of its cell (rows of a bucket share the cell modulo the 21-bit tile id fields).  Measured
// slower (profiles/r05/assoc/prepfused_*: the launch 29 us against 8.6 + 7.7 us for the two, the bucket
// block's serial recomputation being the longest lane of it; C-ABI 0.156 vs 0.145 ms): off by default,
// GCSLAM_PREP_FUSED=1 for A/B.
#ifndef GCS_PREP_FUSED
#define GCS_PREP_FUSED 0
#endif
constexpr int kFusedTiles = 256;
constexpr int kFusedBuckets = kFusedTiles + 1;
__global__ __launch_bounds__(1024) void k_as_prep_fused(AsIn in, AsParams p, AsWork w, const int8_t* __restrict__ st,
                                                        int lane_blocks, int cap) {
#pragma clang fp contract(off)
  __shared__ int64_t s_tid[kFusedTiles];
  __shared__ uint32_t s_wsum[16];
  __shared__ uint32_t s_cnt[kFusedBuckets], s_off[kFusedBuckets], s_tc[kFusedTiles];
  __shared__ int32_t s_bcell[kFusedBuckets * 3];
  __shared__ int32_t s_btix[kFusedBuckets * kMaxStencil];
  __shared__ int16_t s_cbk[kMaxBuckets];  // chunk -> bucket (chunks <= rows / 8 + buckets)
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int b = blockIdx.x;
  const int NT = p.n_tiles, S = p.n_stencil, MV = p.m_view, C = w.chunk;
  if (b < lane_blocks) {
    if (b * 1024 < p.n) {
      for (int q = t; q < NT; q += 1024) s_tid[q] = in.tile_ids[q];
      __syncthreads();
    }
    prep_lane(in, p, w, st, b * 1024 + t, s_tid, true, false);
    return;
  }
  if (b < lane_blocks + NT) {
    compact_tile(in, p, w, b - lane_blocks, s_wsum);
    return;
  }
  // ---- the bucket block
  const int nb = NT + 1;
  for (int q = t; q < NT; q += 1024) {
    s_tid[q] = in.tile_ids[q];
    s_tc[q] = 0u;
  }
  for (int q = t; q < nb; q += 1024) s_cnt[q] = 0u;
  for (int q = t; q < cap; q += 1024) w.order[q] = -1;
  __syncthreads();
  {  // the view tiles' valid counts (loads first, then one LDS add per tile run of the thread's bytes)
    const int tot = NT * MV;
    constexpr int kB = 32;  // bytes per thread and pass
    for (int e0 = t * kB; e0 < tot; e0 += 1024 * kB) {
      uint8_t v[kB];
#pragma unroll
      for (int u = 0; u < kB; ++u) v[u] = e0 + u < tot ? in.vvalid[e0 + u] : 0;
      int run_t = e0 / MV;
      uint32_t run_n = 0u;
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        if (e0 + u >= tot) break;
        const int tb = (e0 + u) / MV;
        if (tb != run_t) {
          if (run_n) atomicAdd(&s_tc[run_t], run_n);
          run_t = tb;
          run_n = 0u;
        }
        run_n += v[u] != 0 ? 1u : 0u;
      }
      if (run_n) atomicAdd(&s_tc[run_t], run_n);
    }
  }
  // each row's own tile: the row lanes' solve and cell (the same code), its first match in the view
  int rb[kBucketRows];
  uint32_t rs[kBucketRows];
#pragma unroll
  for (int j = 0; j < kBucketRows; ++j) {
    const int i = t + j * 1024;
    rb[j] = 0;
    rs[j] = 0u;
    if (i < p.n) {
      double L[9], th[3], x[3];
      for (int k = 0; k < 9; ++k) L[k] = in.Lambdas[9 * i + k];
      for (int k = 0; k < 3; ++k) th[k] = in.thetas[3 * i + k];
      solve3_pivot(L, p.eps_lift, th, x);
      const double s1 = x[0];
      const double s2 = x[0] * 0.5 + x[1] * kSqrt3Half;
      const int64_t c1 = (int64_t)floor(s1 / p.h), c2 = (int64_t)floor(s2 / p.h), cz = (int64_t)floor(x[2] / p.h);
      int cb = -1;
      if (p.s_center >= 0) {
        const int sc = p.s_center;
        const int64_t id = pack_tile(c1 + st[3 * sc], c2 + st[3 * sc + 1], cz + st[3 * sc + 2]);
        for (int q = NT - 1; q >= 0; --q) cb = s_tid[q] == id ? q : cb;
      }
      rb[j] = cb + 1;
      rs[j] = atomicAdd(&s_cnt[rb[j]], 1u);  // (arrival order: any -- each row's result is its own)
      if (rs[j] == 0u) {  // the bucket's cell (any row's: they agree in the tile id's 21-bit fields)
        s_bcell[3 * rb[j]] = (int32_t)(c1 & kMask);
        s_bcell[3 * rb[j] + 1] = (int32_t)(c2 & kMask);
        s_bcell[3 * rb[j] + 2] = (int32_t)(cz & kMask);
      }
    }
  }
  __syncthreads();
  // buckets' padded starts (exclusive scan of ceil(count / C) x C over the <= 257 buckets)
  {
    const uint32_t pc = t < nb ? (s_cnt[t] + (uint32_t)C - 1u) / (uint32_t)C * (uint32_t)C : 0u;
    uint32_t inc = pc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, off, 64);
      if (lane >= off) inc += y;
    }
    if (lane == 63) s_wsum[wid] = inc;
    __syncthreads();
    uint32_t run = inc - pc;
    for (int v2 = 0; v2 < wid; ++v2) run += s_wsum[v2];
    if (t < nb) s_off[t] = run;
  }
  __syncthreads();
  // the order list, the chunk -> bucket map, per bucket its stencil tiles' view indices
#pragma unroll
  for (int j = 0; j < kBucketRows; ++j) {
    const int i = t + j * 1024;
    if (i < p.n) w.order[s_off[rb[j]] + rs[j]] = i;
  }
  const int nch = cap / C;
  for (int q = t; q < nch; q += 1024) s_cbk[q] = -1;
  __syncthreads();
  for (int bk = t; bk < nb; bk += 1024) {
    const int c0 = (int)(s_off[bk] / (uint32_t)C), nc = (int)((s_cnt[bk] + (uint32_t)C - 1u) / (uint32_t)C);
    for (int c = 0; c < nc; ++c) s_cbk[c0 + c] = (int16_t)bk;
  }
  for (int q = t; q < nb * S; q += 1024) {
    const int bk = q / S, sq = q - bk * S;
    int hit = -1;
    if (s_cnt[bk] > 0u) {
      const int64_t id = pack_tile((int64_t)s_bcell[3 * bk] + st[3 * sq], (int64_t)s_bcell[3 * bk + 1] + st[3 * sq + 1],
                                   (int64_t)s_bcell[3 * bk + 2] + st[3 * sq + 2]);
      for (int qq = NT - 1; qq >= 0; --qq) hit = s_tid[qq] == id ? qq : hit;
    }
    s_btix[bk * S + sq] = hit;
  }
  __syncthreads();
  // every chunk's record: its bucket's stencil tiles and the inclusive prefix of their valid counts
  for (int q = t; q < nch * S; q += 1024) {
    const int c = q / S, sq = q - c * S;
    const int bk = s_cbk[c];
    if (bk < 0) continue;
    int pre = 0;
    for (int s2 = 0; s2 <= sq; ++s2) {
      const int tj = s_btix[bk * S + s2];
      pre += tj >= 0 ? (int)s_tc[tj] : 0;
    }
    w.ctile[(size_t)c * 64 + sq] = s_btix[bk * S + sq];
    w.cpre[(size_t)c * 64 + sq] = pre;
  }
}

// Cross-lane exchange for wave reductions without the LDS crossbar (ds_bpermute: ~100+ cycles per
// step on a row's latency chain): step 0, 1 quad_perm [1,0,3,2] / [2,3,0,1] (xor 1, 2), step 2, 3
// row_half_mirror / row_mirror (DPP), step 4, 5 v_permlane16_swap / v_permlane32_swap (the other row /
// half).  Not an xor for steps 2 and 3, but each step pairs every lane of one aligned group of
// 2^step lanes with a lane of the neighbouring group, so after a reduction's step s every aligned
// group of 2^(s+1) lanes holds its reduction (min / argmin: commutative, associative, idempotent).
template <int STEP>
__device__ __forceinline__ unsigned xlane(unsigned x, int lane) {
  if constexpr (STEP == 0) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
  else if constexpr (STEP == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
  else if constexpr (STEP == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
  else if constexpr (STEP == 3) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
  else if constexpr (STEP == 4) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (lane & 32) ? r[0] : r[1];
  }
}
template <int STEP>
__device__ __forceinline__ void argmin_step(unsigned long long& k, int& p, int lane) {
  const unsigned lo = xlane<STEP>((unsigned)k, lane), hi = xlane<STEP>((unsigned)(k >> 32), lane);
  const int op = (int)xlane<STEP>((unsigned)p, lane);
  const unsigned long long ok = ((unsigned long long)hi << 32) | lo;
  if (kless(ok, op, k, p)) {
    k = ok;
    p = op;
  }
}
// the wave's smallest (key, position): in every lane
__device__ __forceinline__ void wave_argmin(unsigned long long& k, int& p, int lane) {
  argmin_step<0>(k, p, lane);
  argmin_step<1>(k, p, lane);
  argmin_step<2>(k, p, lane);
  argmin_step<3>(k, p, lane);
  argmin_step<4>(k, p, lane);
  argmin_step<5>(k, p, lane);
}
template <int STEP>
__device__ __forceinline__ float fmin_step(float x, int lane) {
  return fminf(x, __uint_as_float(xlane<STEP>(__float_as_uint(x), lane)));
}
template <int STEP>
__device__ __forceinline__ double dmin_step(double x, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = xlane<STEP>((unsigned)b, lane), hi = xlane<STEP>((unsigned)(b >> 32), lane);
  return fmin(x, __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)));
}
__device__ __forceinline__ double wave_min_f64(double x, int lane) {
  x = dmin_step<0>(x, lane);
  x = dmin_step<1>(x, lane);
  x = dmin_step<2>(x, lane);
  x = dmin_step<3>(x, lane);
  x = dmin_step<4>(x, lane);
  return dmin_step<5>(x, lane);
}
// a double through xlane<st> (st folds to a constant in unrolled loops)
__device__ __forceinline__ double xlane_d(double x, int st, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  unsigned lo, hi;
  switch (st) {
    case 0: lo = xlane<0>((unsigned)b, lane); hi = xlane<0>((unsigned)(b >> 32), lane); break;
    case 1: lo = xlane<1>((unsigned)b, lane); hi = xlane<1>((unsigned)(b >> 32), lane); break;
    case 2: lo = xlane<2>((unsigned)b, lane); hi = xlane<2>((unsigned)(b >> 32), lane); break;
    case 3: lo = xlane<3>((unsigned)b, lane); hi = xlane<3>((unsigned)(b >> 32), lane); break;
    case 4: lo = xlane<4>((unsigned)b, lane); hi = xlane<4>((unsigned)(b >> 32), lane); break;
    default: lo = xlane<5>((unsigned)b, lane); hi = xlane<5>((unsigned)(b >> 32), lane); break;
  }
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float wave_min_f32(float x, int lane) {
  x = fmin_step<0>(x, lane);
  x = fmin_step<1>(x, lane);
  x = fmin_step<2>(x, lane);
  x = fmin_step<3>(x, lane);
  x = fmin_step<4>(x, lane);
  return fmin_step<5>(x, lane);
}

// the wave's K rounds of argmin over the lanes' sorted lists (the winner's lane pops its head): lane r
// receives the r-th selected position; returns the K-th selected key (wave-uniform)
template <int KM>
__device__ __forceinline__ unsigned long long wave_merge(unsigned long long (&key)[KM], int (&idx)[KM], int K, int lane,
                                                         int& my_sel) {
  unsigned long long last = ~0ULL;
  for (int r = 0; r < K; ++r) {
    unsigned long long bk = key[0];
    int bp = idx[0];
    wave_argmin(bk, bp, lane);
    if (lane == r) my_sel = bp;
    last = bk;
    if (idx[0] == bp && key[0] == bk) {  // pool positions are unique: exactly one owner
#pragma unroll
      for (int j = 0; j < KM - 1; ++j) {
        key[j] = key[j + 1];
        idx[j] = idx[j + 1];
      }
      key[KM - 1] = ~0ULL;
      idx[KM - 1] = 0x7fffffff;
    }
  }
  return last;
}

// one row's selection (one wave); LDS: the chunk's compacted stencil tiles are staged in s_vp (else
// read from L2) -- two instantiations, so neither path's loads go through generic pointers
template <int KM, bool LDS>
__device__ __forceinline__ void pool_row(const AsIn& in, const AsParams& p, const AsWork& w, const AsOut& o,
                                         const float4* s_vp, int* rq, int* re, int i, int lane, int my_tix,
                                         int my_cnt) {
#pragma clang fp contract(off)
  const int MV = p.m_view, S = p.n_stencil;
  const bool row_valid = in.valid[i] != 0;
  auto ld = [&](int sq, int ti, int j) -> float4 {
    if constexpr (LDS) return s_vp[sq * MV + j];
    else return w.vc[(size_t)ti * MV + j];
  };
  const double mp[3] = {w.pos[3 * i], w.pos[3 * i + 1], w.pos[3 * i + 2]};
  const double md[3] = {w.dir[3 * i], w.dir[3 * i + 1], w.dir[3 * i + 2]};
  const double mk = w.kap[i], A1 = w.A1[i];
  int my_sel = 0;
  if (row_valid) {
    unsigned long long key[KM];
    int idx[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      key[j] = ~0ULL;
      idx[j] = 0x7fffffff;
    }
    const bool prune = p.beta >= 0.0;
    const double E = 0x1p-20 * ((fabs(mp[0]) + fabs(mp[1])) + fabs(mp[2])) + 1e-30;
    const double rup = 1.0 + 0x1p-19, rdn = 1.0 - 0x1p-19;
    const float m0 = (float)mp[0], m1 = (float)mp[1], m2 = (float)mp[2];
    auto d32 = [&](const float4& v) {
      const float dx = m0 - v.x, dy = m1 - v.y, dz = m2 - v.z;
      return (dx * dx + dy * dy) + dz * dz;
    };
    float thrA = INFINITY;  // prune an entry whose table distance^2 exceeds this
    PP_STAMP(2);
    if (prune) {
      double thr = INFINITY;
      for (int round = 0; round < 2 && thr == INFINITY; ++round) {
        float dmin = INFINITY;
        for (int sq = round == 0 ? p.s_center : 0; sq < (round == 0 ? p.s_center + 1 : S); ++sq) {
          const int ti = sq >= 0 ? __shfl(my_tix, sq, 64) : -1;
          const int n = sq >= 0 ? __shfl(my_cnt, sq, 64) : 0;
          if (ti < 0) continue;
          for (int j = lane; j < n; j += 64) dmin = fminf(dmin, d32(ld(sq, ti, j)));
        }
        float kth = INFINITY, cur = dmin;
        for (int r = 0; r < p.k; ++r) {  // the r-th smallest lane minimum, lanes popped in turn
          const float m = wave_min_f32(cur, lane);
          kth = m;
          const unsigned long long hit = __ballot(cur == m);
          if (lane == __ffsll((long long)hit) - 1) cur = INFINITY;
        }
        if (kth < INFINITY) {
          const double du = (sqrt((double)kth) + E) * rup;
          thr = du * du * (1.0 + 0x1p-40) + p.beta;
        }
      }
      if (thr < INFINITY) {
        const double dl = sqrt(thr) / rdn + E;
        thrA = (float)(dl * dl * (1.0 + 0x1p-20));  // (rounded to f32: still above the f64 value)
      }
    }
    PP_STAMP(3);
    unsigned head = 0, tail = 0;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    auto take = [&](int n) {  // lanes < n cost ring entry head + lane (exact f64)
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < n) {
        const unsigned slot = (head + lane) & (kLRing - 1);
        const int q = rq[slot], e = re[slot];
        const double dx = mp[0] - in.vpos[3 * e], dy = mp[1] - in.vpos[3 * e + 1], dz = mp[2] - in.vpos[3 * e + 2];
        const double d_pos = (dx * dx + dy * dy) + dz * dz;
        if (!(prune && d_pos > key_value(key[KM - 1])))
          list_insert<KM>(key, idx, order_key(pair_cost(mp, md, mk, A1, in.vpos, in.vdir, in.vkap, w.A2, e, p.beta)),
                          q);
      }
      head += n;
    };
    for (int sq = 0; sq < S; ++sq) {
      const int ti = __shfl(my_tix, sq, 64);
      const int n = __shfl(my_cnt, sq, 64);  // (0 for a missing tile)
      for (int j0 = 0; j0 < n; j0 += kLdsPB * 64) {
        float4 vv[kLdsPB];
#pragma unroll
        for (int u = 0; u < kLdsPB; ++u) {
          const int j = j0 + lane + u * 64;
          vv[u] = j < n ? ld(sq, ti, j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < kLdsPB; ++u) {
          const int j = j0 + lane + u * 64;
          const bool keep = j < n && !(prune && d32(vv[u]) > thrA);
          const unsigned long long m = __ballot(keep);
          if (keep) {
            const int oo = (int)vv[u].w;
            const unsigned slot = (tail + (unsigned)__popcll(m & lt_mask)) & (kLRing - 1);
            rq[slot] = sq * MV + oo;
            re[slot] = ti * MV + oo;
          }
          tail += (unsigned)__popcll(m);
        }
        while (tail - head >= 64u) take(64);
      }
    }
    if (tail != head) take((int)(tail - head));
    PP_STAMP(4);
#if GCS_POOL_PROBE
    if (lane == 0) g_pool_probe[(size_t)i * 10 + 8] = tail;
#endif
    const unsigned long long kth_key = wave_merge<KM>(key, idx, p.k, lane, my_sel);
    PP_STAMP(5);
    if (kth_key >= order_key(kCostInvalid)) {
      // Fewer than K valid entries cost less than the invalid cost.  No valid entry was pruned here
      // (a finite threshold has K valid entries at or below it, and a pruned one is above them all),
      // so the K selected are the K smallest valid (cost, position); the invalid entries and missing
      // tiles all cost 1e12, ordered by position: the K smallest of both sets are the K first invalid
      // positions (wave-ordered ballots over the pool) merged with the selected ones.
      // lane r < K: the r-th selected key again (the merge popped it; empty: ~0, position 0x7fffffff)
      const bool has = lane < p.k && my_sel != 0x7fffffff;
      const int sel_t = __shfl(my_tix, has ? my_sel / MV : 0, 64);
      unsigned long long my_key = ~0ULL;
      if (has)
        my_key = order_key(pair_cost(mp, md, mk, A1, in.vpos, in.vdir, in.vkap, w.A2, sel_t * MV + my_sel % MV, p.beta));
      int inv_pos = 0x7fffffff;  // lane r < K: the r-th invalid position
      int found = 0;
      for (int sq = 0; sq < S && found < p.k; ++sq) {
        const int ti = __shfl(my_tix, sq, 64);
        for (int o0 = 0; o0 < MV && found < p.k; o0 += 64) {
          const int oo = o0 + lane;
          const bool inv = oo < MV && (ti < 0 || !in.vvalid[(size_t)ti * MV + oo]);
          const unsigned long long bm = __ballot(inv);
          const int rank = found + (int)__popcll(bm & ((1ull << lane) - 1ull));
          if (inv && rank < p.k) rq[rank] = sq * MV + oo;  // (the wave's ring as scratch: no take pending)
          found += (int)__popcll(bm);
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < std::min(found, p.k)) inv_pos = rq[lane];
      // lanes 0..K-1: the selected (key, position); lanes K..2K-1: the invalid positions at 1e12
      unsigned long long ck = my_key;
      int cp = lane < p.k ? my_sel : 0x7fffffff;
      if (lane >= p.k) ck = ~0ULL;
      const int il = lane - p.k;
      const int ipos = __shfl(inv_pos, il >= 0 && il < 64 ? il : 0, 64);
      if (il >= 0 && il < p.k && il < found) {
        ck = order_key(kCostInvalid);
        cp = ipos;
      }
      for (int r = 0; r < p.k; ++r) {
        unsigned long long bk = ck;
        int bp = cp;
        wave_argmin(bk, bp, lane);
        if (lane == r) my_sel = bp;
        if (ck == bk && cp == bp) {  // (positions are unique: one owner)
          ck = ~0ULL;
          cp = 0x7fffffff;
        }
      }
#if GCS_POOL_PROBE
      if (lane == 0) g_pool_probe[(size_t)i * 10 + 9] = 1;
#endif
    }
  }
  PP_STAMP(6);
  // per candidate (lane k < K): view index, unmasked cost + recency, row min (:377-403)
  const bool act = lane < p.k;
  const int sel_ti = __shfl(my_tix, row_valid && act ? my_sel / MV : 0, 64);
  int e = 0;
  if (act && row_valid) e = (sel_ti < 0 ? 0 : sel_ti) * MV + my_sel % MV;
  double c = INFINITY, dt = 0.0;
  if (act) {
    c = pair_cost(mp, md, mk, A1, in.vpos, in.vdir, in.vkap, w.A2, e, p.beta);
    const long long last = (long long)in.vlast[e];
    dt = (double)(p.scan_seq - last > 0 ? p.scan_seq - last : 0);
    c = c + p.eps_lam * dt;
  }
  const double mn = wave_min_f64(c, lane);
  if (act) {
    if (p.row_min) c = c - mn;
    const size_t o_ = (size_t)i * p.k + lane;
    o.cost[o_] = c;
    if (!p.med) w.kmat[o_] = exp(-c / fmax(p.eps, 1e-12));  // (the Sinkhorn's own expression)
    w.cand[o_] = e;
    w.dt[o_] = dt;
    if (o.cand) o.cand[o_] = e;
    if (o.tile) o.tile[o_] = in.vtile[e];
    if (o.slot) o.slot[o_] = (int64_t)in.vslot[e];
  }
  {  // the MapUpdateCert's per-row candidate statistics (cand_stats): valid candidates, distinct tiles
    const bool cv = act && row_valid && in.vvalid[e] != 0;
    const long long tile = cv ? (long long)in.vtile[e] : -1;
    bool seen = false;
    for (int k2 = 0; k2 < p.k; ++k2) {  // (every lane: the shuffles read lanes < K)
      const long long t2 = __shfl(tile, k2, 64);
      seen = seen || (k2 < lane && t2 != -1 && t2 == tile);
    }
    const unsigned cnt = (unsigned)__popcll(__ballot(cv));
    const unsigned dist = (unsigned)__popcll(__ballot(cv && tile != -1 && !seen));
    if (lane == 0) w.cstat[i] = cnt | (dist << 16);
  }
  PP_STAMP(7);
}

template <int KM>
__global__ __launch_bounds__(kPoolLdsWaves * 64) void k_as_pool_lds(AsIn in, AsParams p, AsWork w, AsOut o,
                                                                    int lds_slots) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* s_vp = (float4*)smem;
  const int MV = p.m_view, S = p.n_stencil;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#if GCS_POOL_PROBE
  const unsigned long long t_start = wall_clock64();
#endif
  const int r0 = w.order[blockIdx.x * kPoolLdsWaves];
  const int i = w.order[blockIdx.x * kPoolLdsWaves + wid];
  const int my_st = lane < S ? w.ctile[(size_t)blockIdx.x * 64 + lane] : -1;  // (S <= 64: in every wave)
  const int my_pre = lane < S ? w.cpre[(size_t)blockIdx.x * 64 + lane] : 0;
  if (r0 < 0) return;  // a chunk past the last bucket (every thread: before the block barrier)
  const int cb = p.s_center >= 0 ? __shfl(my_st, p.s_center, 64) : -1;
  const bool lds = cb >= 0 && lds_slots > 0;  // (uniform)
  if (lds) {
    // each stencil tile's valid entries at sq MV, the tiles' entries concatenated over the threads:
    // eight 16-B loads in flight per thread, then their LDS stores (one round trip, not one per tile)
    const int tot = __shfl(my_pre, S - 1, 64);
    for (int g0 = 0; g0 < tot; g0 += 8 * kPoolLdsWaves * 64) {
      float4 v[8];
      int dst[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int g = g0 + u * kPoolLdsWaves * 64 + t;
        // the stencil slot holding concatenated entry g: the first whose inclusive prefix exceeds g
        int sq = -1, base = 0, ti = 0, prev = 0;
        for (int q = 0; q < S; ++q) {
          const int pre = __builtin_amdgcn_readlane(my_pre, q), tq = __builtin_amdgcn_readlane(my_st, q);
          if (sq < 0 && g < pre) {
            sq = q;
            base = prev;
            ti = tq;
          }
          prev = pre;
        }
        dst[u] = -1;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g < tot && sq >= 0) {
          dst[u] = sq * MV + (g - base);
          v[u] = w.vc[(size_t)ti * MV + (g - base)];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (dst[u] >= 0) s_vp[dst[u]] = v[u];
    }
  }
  __syncthreads();
  if (i < 0) return;  // a bucket's padding (after the only block barrier)
#if GCS_POOL_PROBE
  if (lane == 0) {
    g_pool_probe[(size_t)i * 10 + 0] = t_start;
    g_pool_probe[(size_t)i * 10 + 1] = wall_clock64();
    for (int q = 2; q < 10; ++q) g_pool_probe[(size_t)i * 10 + q] = 0;
  }
#endif
  int* rq = (int*)(smem + (size_t)lds_slots * 16) + wid * 2 * kLRing;
  int* re = rq + kLRing;
  if (lds) {  // the row's stencil tiles are the chunk's (lane s: tile, valid count)
    const int prv = __shfl_up(my_pre, 1, 64);
    pool_row<KM, true>(in, p, w, o, s_vp, rq, re, i, lane, my_st, lane == 0 ? my_pre : my_pre - prv);
  } else {
    const int my_tix = lane < S ? w.tix[(size_t)i * S + lane] : -1;
    const int my_cnt = lane < S && my_tix >= 0 ? w.vcnt[my_tix] : 0;
    pool_row<KM, false>(in, p, w, o, s_vp, rq, re, i, lane, my_tix, my_cnt);
  }
}

// ---------------------------------------------------------------- single-workgroup Sinkhorn
template <int NV>
__device__ __forceinline__ void bsum(double (&v)[NV], double* lds /*16*NV*/) {
  // fixed xor tree in each wave, then the 16 wave rows in order (valid in every thread)
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], sh, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[wid * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = lds[k];
    for (int q = 1; q < kShThreads / 64; ++q) s += lds[q * NV + k];
    v[k] = s;
  }
}

// k-th smallest (0-based) of the values the threads hold (slot j of a thread counts when bit j of
// its mask is set), MSB-first radix select over the total-order keys, 8 bits per pass; the result
// is returned in every thread
template <int CAP>
__device__ __forceinline__ double radix_select(const double (&vals)[CAP], uint32_t okmask, int k, uint32_t* hist /*256*/,
                               uint32_t* sel /*4*/) {
  static_assert(CAP <= 32, "slot mask is 32 bits");
  unsigned long long prefix = 0, mask = 0;
  const int t = threadIdx.x, lane = t & 63;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    __syncthreads();
    if (t < 256) hist[t] = 0u;
    __syncthreads();
    // Histogram adds aggregated before the LDS atomics: runs of one digit within a thread's values
    // are counted in a register, and a thread's last run is merged across the wave when every lane's
    // run has the same digit.  The b-row and a-marginal values repeat (uniform marginals, equal
    // recency), and one LDS address took every add of a pass (N K serialised atomics x 8 passes).
    uint32_t run_d = 0u, run_n = 0u;
#pragma unroll
    for (int j = 0; j < CAP; ++j)
      if ((okmask >> j) & 1u) {
        const unsigned long long kk = order_key(vals[j]);
        if ((kk & mask) == prefix) {
          const uint32_t d = (uint32_t)((kk >> shift) & 255ULL);
          if (run_n != 0u && d != run_d) {
            atomicAdd(&hist[run_d], run_n);
            run_n = 0u;
          }
          run_d = d;
          ++run_n;
        }
      }
    {
      const bool have = run_n != 0u;
      const unsigned long long hm = __ballot(have);
      if (hm != 0ull) {
        const int first = __ffsll((long long)hm) - 1;
        const uint32_t d0 = (uint32_t)__shfl((int)run_d, first, 64);
        if (__ballot(have && run_d != d0) == 0ull) {  // one digit across the wave: one add
          uint32_t tot = run_n;
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) tot += (uint32_t)__shfl_xor((int)tot, off, 64);
          if (lane == first) atomicAdd(&hist[d0], tot);
        } else if (have) {
          atomicAdd(&hist[run_d], run_n);
        }
      }
    }
    __syncthreads();
    if (t < 64) {
      const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
      const uint32_t mine = h0 + h1 + h2 + h3;
      uint32_t inc = mine;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
      }
      const uint32_t exc = inc - mine;
      if ((uint32_t)k >= exc && (uint32_t)k < inc) {  // exactly one lane
        uint32_t below = exc, d = 4 * lane;
        const uint32_t hs[4] = {h0, h1, h2, h3};
        for (int q = 0; q < 4; ++q) {
          if ((uint32_t)k < below + hs[q]) {
            d = 4 * lane + q;
            break;
          }
          below += hs[q];
        }
        sel[0] = d;
        sel[1] = below;
      }
    }
    __syncthreads();
    prefix |= (unsigned long long)sel[0] << shift;
    mask |= 255ULL << shift;
    k -= (int)sel[1];
  }
  // invert the key map
  const unsigned long long b = (prefix >> 63) ? (prefix & 0x7fffffffffffffffULL) : ~prefix;
  return prefix == ~0ULL ? NAN : __longlong_as_double((long long)b);
}

// recency-weighted b rows (:441-446): exp(-lambda dt) normalised per row
template <int KM, int RPT>
__device__ __forceinline__ void recency_rows(const AsParams& p, const AsWork& w, int N, int K, int t,
                                             double (&brow)[RPT * KM], uint32_t& okb) {
#pragma clang fp contract(off)
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = t + j * kShThreads;
    double dsum = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      double dd = 0.0;
      if (r < N && k < K) {
        dd = exp(-p.lam * w.dt[(size_t)r * K + k]);
        dd = dd > 0.0 ? dd : 0.0;
        okb |= 1u << (j * KM + k);
      }
      brow[j * KM + k] = dd;
      dsum += dd;
    }
    const double den = fmax(dsum, p.eps_mass);
#pragma unroll
    for (int k = 0; k < KM; ++k) brow[j * KM + k] = brow[j * KM + k] / den;
  }
}

enum CertSlot : int {
  CE_DEFECT_A, CE_DEFECT_B, CE_MASS_TOTAL, CE_SUM_A, CE_SUM_B, CE_SUM_M, CE_SUM_NOVEL, CE_P95_A, CE_P95_B,
  CE_NONZERO_A, CE_NONZERO_B, CE_B_P95, CE_ESS, CE_MASS_EPS, CE_TOTAL_COST, CE_SUPPORT, CE_EXACT, CE_MVALID,
  CE_CAND_TILES, CE_CAND_PRIMS, CE_CAND_PRIMS_P95,
  CE_COUNT
};
static_assert(CE_COUNT == GCS_ASSOC_CERT_LEN, "certificate slots");

// The map branch's candidate statistics of the MapUpdateCert (pipeline.py:879-905) from the selected
// candidates: per valid measurement row, the candidates whose view entry is valid (count) and their
// distinct tile ids other than -1; the means of both over the valid rows (denominator max(rows,
// eps_mass)) and the p95 order statistic of the counts with invalid rows at -1 (jnp.sort, index
// min(int(0.95 n), n - 1)).  Every sum is of small integers, so the values are exact in any order; one
// workgroup, LDS integer counters.  e_of(q): the view entry of candidate q.
// (cstat: per row, cnt | dist << 16 from the pool kernel -- each row's candidates sit in its wave's
// lanes there, so the count and the distinct tiles take a few shuffles; the per-row loop below
// walked K^2 dependent loads per row, ~50 us of this workgroup; null: computed here)
template <int NT, class EOF_>
__device__ __forceinline__ void cand_stats(const AsIn& in, const AsParams& p, double eps_mass, EOF_ e_of, double* cert,
                                           const uint32_t* cstat = nullptr) {
  __shared__ unsigned long long s_cs[3];  // valid rows, sum counts, sum distinct tiles
  __shared__ uint32_t s_ch[33];            // histogram of the valid rows' counts (K <= 32)
  const int t = threadIdx.x, K = p.k, N = p.n;
  if (t < 3) s_cs[t] = 0ull;
  if (t < 33) s_ch[t] = 0u;
  __syncthreads();
  uint32_t nv = 0, sc = 0, sd = 0;
  const bool no_view = (long long)p.n_tiles * p.m_view <= 0;  // no entry to index: nothing valid
  for (int r = t; r < N; r += NT) {
    if (!in.valid[r]) continue;
    int cnt = 0, dist = 0;
    if (cstat) {
      const uint32_t cs = cstat[r];
      cnt = (int)(cs & 0xffffu);
      dist = (int)(cs >> 16);
    }
    for (int k = 0; k < K && !no_view && !cstat; ++k) {
      const int e = e_of((size_t)r * K + k);
      if (!in.vvalid[e]) continue;
      ++cnt;
      const long long tile = (long long)in.vtile[e];
      if (tile == -1) continue;
      bool seen = false;
      for (int k2 = 0; k2 < k; ++k2) {
        const int e2 = e_of((size_t)r * K + k2);
        seen = seen || (in.vvalid[e2] && (long long)in.vtile[e2] == tile);
      }
      dist += seen ? 0 : 1;
    }
    ++nv;
    sc += (uint32_t)cnt;
    sd += (uint32_t)dist;
    atomicAdd(&s_ch[cnt], 1u);
  }
  atomicAdd(&s_cs[0], (unsigned long long)nv);
  atomicAdd(&s_cs[1], (unsigned long long)sc);
  atomicAdd(&s_cs[2], (unsigned long long)sd);
  __syncthreads();
  if (t == 0) {
    double tiles = 0.0, prims = 0.0, p95 = 0.0;
    const unsigned long long nvalid = s_cs[0];
    if (nvalid > 0 && N > 0) {
      const double den = fmax((double)nvalid, eps_mass);
      tiles = (double)s_cs[2] / den;
      prims = (double)s_cs[1] / den;
      const long long i95 = std::min((long long)(0.95 * (double)N), (long long)N - 1);
      long long at = (long long)N - (long long)nvalid;  // the -1 entries sort first
      p95 = -1.0;
      for (int c = 0; c <= K && at <= i95; ++c) {
        at += s_ch[c];
        if (at > i95) p95 = (double)c;
      }
    }
    cert[CE_CAND_TILES] = tiles;
    cert[CE_CAND_PRIMS] = prims;
    cert[CE_CAND_PRIMS_P95] = p95;
  }
}

// The scaling updates' arithmetic (the Sinkhorn loop is VALU-bound on one CU: ~600 f64 operations
// per thread and iteration at two waves per SIMD).  gcs_math.h's log_short / exp_short with the
// polynomials in fma Horner form and the quotients from v_rcp_f64 + two Newton steps + one residual
// correction (d > 0 normal, n finite: within an ulp of the IEEE quotient) -- a third fewer
// operations than the contraction-off form with IEEE divides, a few ulps apart from it.
__device__ __forceinline__ double div_fast(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  const double q = n * r;
  return fma(fma(-d, q, n), r, q);
}
__device__ __forceinline__ double log_fast(double x) {  // x > 0, finite, normal
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int e;
  double m = frexp(x, &e);
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  const double f = m - 1.0;
  const double hfsq = 0.5 * f * f;
  const double sq = div_fast(f, 2.0 + f);
  const double dk = (double)e;
  const double z = sq * sq, w = z * z;
  const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  return fma(dk, ln2_hi, -((hfsq - fma(sq, hfsq + R, dk * ln2_lo)) - f));
}
__device__ __forceinline__ double exp_fast(double x) {  // |x| < 700
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
  const int k = (int)fma(invln2, x, x < 0.0 ? -0.5 : 0.5);
  const double t = (double)k;
  const double hi = fma(-t, ln2_hi, x), lo = t * ln2_lo;
  const double r = hi - lo;
  const double rr = r * r;
  const double c = fma(-rr, fma(rr, fma(rr, fma(rr, fma(rr, P5, P4), P3), P2), P1), r);
  const double y = 1.0 - ((lo - div_fast(r * c, 2.0 - c)) - hi);
  return ldexp(y, k);
}
// x^(-1/n) for a uniform integer n >= 1 and x in [2^-100, 2^100]: an f32 seed (v_log_f32 / v_exp_f32,
// a few e-7 relative) and two Newton steps y <- y ((n + 1) - x y^n) / n in f64 (the error squares per
// step: ~3e-11, then below the f64 rounding), y^n by squaring.  The Sinkhorn's scaling exponents
// ua = 1 / (1 + tau_a / eps), vb = 1 / (1 + tau_b / eps) are fl(1 / n) for the reference defaults
// (tau 0.5, eps 0.1: n = 6), so (a / x)^ua = a^ua x^(-1/n) -- a^ua once per call -- replaces a log
// and an exp per row and iteration (a few ulps apart from the pow: the tests' 1e-9 bars)
constexpr double kRootLo = 7.888609052210118e-31;  // 2^-100
constexpr double kRootHi = 1.2676506002282294e30;  // 2^100
__device__ __forceinline__ double ipow_u(double y, int n) {  // y^n, n >= 1 (uniform)
  double r = 1.0;
  for (;;) {
    if (n & 1) r *= y;
    n >>= 1;
    if (!n) return r;
    y *= y;
  }
}
__device__ __forceinline__ double root_seed(double x, float inv_n) {
  return (double)__builtin_amdgcn_exp2f(-inv_n * __builtin_amdgcn_logf((float)x));
}
__device__ __forceinline__ double root_step(double y, double x, int n, double inv_n) {
  return (y * fma(-x, ipow_u(y, n), (double)(n + 1))) * inv_n;
}
template <int N>
__device__ __forceinline__ double ipow_c(double y) {
  if constexpr (N == 1) return y;
  else if constexpr (N % 2 == 0) { const double h = ipow_c<N / 2>(y); return h * h; }
  else return ipow_c<N - 1>(y) * y;
}
template <int N>
__device__ __forceinline__ double root_step_c(double y, double x, double inv_n) {
  return (y * fma(-x, ipow_c<N>(y), (double)(N + 1))) * inv_n;
}
// x^y as pow_sinkhorn (0 at x = 0; the library pow outside the short path's range)
__device__ __forceinline__ double pow_fast(double x, double y) {
  if (x == 0.0) return 0.0;
  if (!(x >= 2.2250738585072014e-308) || !(x <= 1.7976931348623157e308)) return pow_lib(x, y);
  const double a = y * log_fast(x);
  if (!(fabs(a) < 700.0)) return pow_lib(x, y);
  return exp_fast(a);
}

// GCS_SH_FINSPLIT: the Sinkhorn's finish over several workgroups, one row per thread -- pi = u K v, the
// responsibilities and row masses, and the certificate sums (per workgroup in a fixed tree, then the
// workgroups in index order by the last one to finish).  1 (default): extra workgroups of the Sinkhorn
// launch, which load their rows' costs while workgroup 0 iterates and wait for its u / v hand-off
// (sc1 stores + a flag); 2: a launch of its own after the Sinkhorn (k_as_finish); 0: workgroup 0
// finishes alone (~13 us: three rows per thread, their loads and stores on one CU).
#ifndef GCS_SH_FINSPLIT
#define GCS_SH_FINSPLIT 1
#endif
template <int STEP>
__device__ __forceinline__ double dsum_step(double x, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = xlane<STEP>((unsigned)b, lane), hi = xlane<STEP>((unsigned)(b >> 32), lane);
  return x + __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kFinThreads = 256;
// one block of the finish: rows blk NT + t.  The rows' cost / K_mat loads issue first, then wait()
// (the in-kernel form polls the Sinkhorn workgroup's flag there), then u, v and sum a -- sc1 loads
// (the in-kernel form's hand-off; harmless across a launch boundary).  The block's sums (a fixed
// tree) are written sc1 and drained before the ticket; the last block folds them in block order with
// sc1 loads and writes the certificate.
template <int KM, int NT, class Wait>
__device__ __forceinline__ void finish_block(const AsIn& in, const AsParams& p, const AsWork& w, const AsOut& o, int blk,
                                             int nblk, double* s_red /*(NT / 64) x (7 + KM)*/, Wait wait) {
#pragma clang fp contract(off)
  constexpr int NV = 7 + KM;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, N = p.n, K = p.k;
  const double eps = fmax(p.eps, 1e-12);
  const double bk = 1.0 / (double)K;
  const int r = blk * NT + t;
  bool rv = false;
  double va = 0.0, Cr[KM], Xr[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) Cr[k] = Xr[k] = 0.0;
  if (r < N) {
    rv = in.valid[r] != 0;
    va = rv ? 1.0 : 0.0;
    if (p.a_policy == 1) va = va * in.weights[r];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      Cr[k] = k < K && !p.med ? o.cost[(size_t)r * K + k] : 0.0;
      Xr[k] = k < K && !p.med ? w.kmat[(size_t)r * K + k] : 0.0;
    }
  }
  if (!wait()) return;
  if (p.med && r < N)  // the median-scaled costs: written by the Sinkhorn workgroup (sc1) before its hand-off
#pragma unroll
    for (int k = 0; k < KM; ++k)
      Cr[k] = k < K ? __hip_atomic_load(&o.cost[(size_t)r * K + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
  const double sum_a = __hip_atomic_load(&w.su[N + KM], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double v[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) v[k] = k < K ? __hip_atomic_load(&w.su[N + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
  // acc: [sum rm, sum rm^2, sum novel, defect_a^2, sum pi C, nonzero_a, sum pi | col masses K]
  double acc[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) acc[q] = 0.0;
  if (r < N) {
    va = va / sum_a;
    const double u = __hip_atomic_load(&w.su[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double rm = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= K) continue;
      const double X = p.med ? exp(-Cr[k] / eps) : Xr[k];
      const double pik = (u * X) * v[k];
      rm += pik;
      acc[4] += pik * Cr[k];
      acc[6] += pik;
      acc[7 + k] += pik;
      o.resp[(size_t)r * K + k] = rv ? pik : 0.0;
    }
    o.rmass[r] = rm;
    acc[0] += rm;
    acc[1] += rm * rm;
    acc[2] += fmax(va - rm, 0.0);
    acc[3] += (rm - va) * (rm - va);
    acc[5] += va > p.eps_mass ? 1.0 : 0.0;
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double x = acc[q];
    x = dsum_step<0>(x, lane);
    x = dsum_step<1>(x, lane);
    x = dsum_step<2>(x, lane);
    x = dsum_step<3>(x, lane);
    x = dsum_step<4>(x, lane);
    x = dsum_step<5>(x, lane);
    acc[q] = x;
  }
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) s_red[wid * NV + q] = acc[q];
  __syncthreads();
  if (wid != 0) return;
  // wave 0: this block's sums (lane q), the ticket, and -- in the last block -- the fold.  The sums are
  // write-through (sc1) stores drained before the ticket (the guide's R1 publish: no release fence,
  // whose L2 write-back costs more than the finish); the last block reads them with sc1 loads
  if (lane < NV) {
    double sum = s_red[lane];
    for (int g = 1; g < NT / 64; ++g) sum += s_red[g * NV + lane];
    __hip_atomic_store(&w.fpart[(size_t)blk * NV + lane], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned tk = 0;
  if (lane == 0) tk = __hip_atomic_fetch_add(w.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tk = (unsigned)__shfl((int)tk, 0, 64);
  if (tk != (unsigned)nblk - 1u) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (keeps the loads below the ticket)
  double f = 0.0;
  if (lane < NV)
    for (int g = 0; g < nblk; ++g)
      f += __hip_atomic_load(&w.fpart[(size_t)g * NV + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double tot[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) tot[q] = __shfl(f, q, 64);
  double db = 0.0;  // (every lane: the shuffles read lanes 7 ..)
  for (int k = 0; k < K; ++k) {
    const double ck = __shfl(f, 7 + k, 64);
    db += (ck - bk) * (ck - bk);
  }
  if (lane == 0) {
    const double tm = tot[6];
    o.cert[CE_DEFECT_A] = sqrt(tot[3]);
    o.cert[CE_DEFECT_B] = sqrt(db);
    o.cert[CE_MASS_TOTAL] = tm;
    o.cert[CE_SUM_A] = sum_a;
    o.cert[CE_SUM_B] = bk * (double)K;
    o.cert[CE_SUM_M] = tot[0];
    o.cert[CE_SUM_NOVEL] = tot[2];
    o.cert[CE_P95_B] = bk;  // b uniform: every entry is 1 / K
    o.cert[CE_NONZERO_A] = tot[5];
    o.cert[CE_NONZERO_B] = bk > p.eps_mass ? (double)K : 0.0;
    o.cert[CE_ESS] = tot[0] * tot[0] / (tot[1] + p.eps_mass);
    o.cert[CE_MASS_EPS] = p.eps_mass / (tm + p.eps_mass);
    o.cert[CE_TOTAL_COST] = tot[4];
    o.cert[CE_SUPPORT] = tot[5] / (double)std::max(N, 1);
    o.cert[CE_EXACT] = 0.0;
    o.cert[CE_MVALID] = (double)*w.mvalid;
    *w.mvalid_next = 0u;  // the next call's counter, armed
    __hip_atomic_store(w.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
  }
}

// GCSLAM_SH_FINSPLIT=2: the finish as its own launch after the Sinkhorn (A/B of the in-kernel form)
template <int KM>
__global__ __launch_bounds__(kFinThreads) void k_as_finish(AsIn in, AsParams p, AsWork w, AsOut o, int n_valid_host,
                                                           const int32_t* n_valid_dev) {
  __shared__ double s_red[(kFinThreads / 64) * (7 + KM)];
  if ((n_valid_dev ? *n_valid_dev : n_valid_host) == 0 || *w.mvalid == 0u) return;  // the Sinkhorn's empty result
  finish_block<KM, kFinThreads>(in, p, w, o, blockIdx.x, gridDim.x, s_red, [] { return true; });
}

template <int KM, int RPT>
__global__ __launch_bounds__(kShThreads) void k_as_sinkhorn(AsIn in, AsParams p, AsWork w, AsOut o, int n_valid_host,
                                                            const int32_t* n_valid_dev) {
#pragma clang fp contract(off)
  __shared__ double s_red[16 * (KM + 8)];
#if GCS_SH_ONEBAR
  __shared__ double s_colp2[2][(kShThreads / 64) * KM];  // alternate iterations (one barrier each)
#else
  __shared__ double s_colp[(kShThreads / 64) * KM];
  __shared__ double s_v[KM];
#endif
  __shared__ uint32_t s_hist[256], s_sel[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int N = p.n, K = p.k;
  if (blockIdx.x == 0) SH_STAMP(0);
  const bool empty = (n_valid_dev ? *n_valid_dev : n_valid_host) == 0 || *w.mvalid == 0u;
  if (empty) {  // :272-287 -- zeros, exact cert (workgroup 0)
    if (blockIdx.x != 0) return;
    for (int q = t; q < N * K; q += kShThreads) {
      o.resp[q] = 0.0;
      o.cost[q] = 0.0;
      if (o.cand) o.cand[q] = 0;
      if (o.tile) o.tile[q] = 0;
      if (o.slot) o.slot[q] = 0;
    }
    for (int q = t; q < N; q += kShThreads) o.rmass[q] = 0.0;
    if (t < CE_CAND_TILES) o.cert[t] = t == CE_EXACT ? 1.0 : (t == CE_MVALID ? (double)*w.mvalid : 0.0);
    if (t == 0) *w.mvalid_next = 0u;  // the next call's counter, armed (no per-call memset)
    // the empty result selects view entry 0 for every candidate (the outputs above)
    cand_stats<kShThreads>(in, p, p.eps_mass, [](size_t) { return 0; }, o.cert);
    return;
  }
  if (blockIdx.x >= 2) {  // a finish workgroup (GCS_SH_FINSPLIT 1): its rows' costs, then workgroup 0's u, v
    __shared__ double s_fin[(kShThreads / 64) * (7 + KM)];
    __shared__ int s_ok;
    auto wait = [&]() -> bool {
      if (t == 0) {
        bool ok = false;
        for (unsigned it = 0; it < (1u << 22) && !ok; ++it) {  // bounded: a lost hand-off fails loudly
          ok = __hip_atomic_load(w.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.epoch;
          if (!ok) __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) o.cert[CE_MASS_TOTAL] = NAN;
        s_ok = ok ? 1 : 0;
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (keeps the hand-off's sc1 loads below)
      return s_ok != 0;
    };
    finish_block<KM, kShThreads>(in, p, w, o, blockIdx.x - 2, gridDim.x - 2, s_fin, wait);
    return;
  }
  if (blockIdx.x == 1) {
    // The certificate's p95 order statistics (:445-446, :488-493) depend on the marginal a and the
    // recency rows only, not on the scalings: a second workgroup computes them on another CU while
    // workgroup 0 iterates.
    double va1[RPT];
    double part1[1] = {0.0};
    uint32_t oka1 = 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int r = t + j * kShThreads;
      va1[j] = 0.0;
      if (r < N) {
        va1[j] = in.valid[r] ? 1.0 : 0.0;
        if (p.a_policy == 1) va1[j] = va1[j] * in.weights[r];
        oka1 |= 1u << j;
      }
      part1[0] += va1[j];
    }
    bsum<1>(part1, s_red);
    const double sum_a1 = fmax(part1[0], p.eps_mass);
#pragma unroll
    for (int j = 0; j < RPT; ++j) va1[j] = va1[j] / sum_a1;
    double brow1[RPT * KM];
    uint32_t okb1 = 0;
    recency_rows<KM, RPT>(p, w, N, K, t, brow1, okb1);
    const double p95_a = radix_select<RPT>(va1, oka1, std::min((int)(0.95 * (double)N), N - 1), s_hist, s_sel);
    const int nbt = N * K;
    const double p95_b_row = radix_select<RPT * KM>(brow1, okb1, std::min((int)(0.95 * (double)nbt), nbt - 1), s_hist, s_sel);
    SH_STAMP(5);
    if (t == 0) {
      o.cert[CE_P95_A] = p95_a;
      o.cert[CE_B_P95] = p95_b_row;
    }
    // this workgroup ends well inside workgroup 0's iterations: the MapUpdateCert's candidate
    // statistics ride here, with no host sync of their own
    const int32_t* cand = w.cand;
    cand_stats<kShThreads>(in, p, p.eps_mass, [cand](size_t q) { return (int)cand[q]; }, o.cert, w.cstat);
    return;
  }
#if GCS_SH_TAB
  // the loop's log / exp tables (gcs_sh_tables.h) in LDS: per-lane indexed reads at LDS latency
  __shared__ double s_lt[kShLogTabLen], s_et[kShExpTabLen];
  for (int q = t; q < kShLogTabLen; q += kShThreads) s_lt[q] = kShLogTab[q];
  for (int q = t; q < kShExpTabLen; q += kShThreads) s_et[q] = kShExpTab[q];  // (bsum's barriers publish them)
#define SH_LOG(x) log_tab((x), s_lt)
#define SH_EXP(x) exp_tab((x), s_et)
#else
#define SH_LOG(x) log_fast(x)
#define SH_EXP(x) exp_fast(x)
#endif
  // marginal a (:412-424)
  double va[RPT], X[RPT * KM];  // X: the cost rows, then K_mat = exp(-C / eps) in place
  double part[1] = {0.0};
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = t + j * kShThreads;
    va[j] = 0.0;
    if (r < N) {
      va[j] = in.valid[r] ? 1.0 : 0.0;
      if (p.a_policy == 1) va[j] = va[j] * in.weights[r];
    }
    part[0] += va[j];
  }
  bsum<1>(part, s_red);
  const double sum_a = fmax(part[0], p.eps_mass);
  SH_STAMP(1);
#pragma unroll
  for (int j = 0; j < RPT; ++j) va[j] = va[j] / sum_a;
#if GCS_SH_LOGA
  // log a once: each iteration's u = (a / Kv)^ua is exp(ua (log a - log Kv)) -- the quotient (and its
  // rcp / Newton / residual steps) leaves the loop (rounding-level change; the tests' 1e-9 bars)
  double lva[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    lva[j] = va[j] >= 2.2250738585072014e-308 && va[j] <= 1.7976931348623157e308 ? log_fast(va[j]) : NAN;
#endif
  uint32_t okm = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j)
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int r = t + j * kShThreads;
      const bool ok = r < N && k < K;
      X[j * KM + k] = ok ? (p.med ? o.cost[(size_t)r * K + k] : w.kmat[(size_t)r * K + k]) : 0.0;
      if (ok) okm |= 1u << (j * KM + k);
    }
  if (p.med) {  // cost_scale_by_median (:405-407)
    const int tot = N * K;
    double med;
    if (tot & 1) {
      med = radix_select<RPT * KM>(X, okm, tot / 2, s_hist, s_sel);
    } else {
      const double lo = radix_select<RPT * KM>(X, okm, tot / 2 - 1, s_hist, s_sel);
      const double hi = radix_select<RPT * KM>(X, okm, tot / 2, s_hist, s_sel);
      med = (lo + hi) * 0.5;  // jnp.median: mean of the two middle values
    }
#pragma unroll
    for (int q = 0; q < RPT * KM; ++q) {
      X[q] = X[q] / (med + 1e-12);
      if ((okm >> q) & 1u)  // result.cost_matrix (sc1: the finish workgroups read it after the hand-off)
        __hip_atomic_store(&o.cost[(size_t)(t + (q / KM) * kShThreads) * K + q % KM], X[q], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const double eps = fmax(p.eps, 1e-12);
  const double ua = 1.0 / (1.0 + p.tau_a / eps), vb = 1.0 / (1.0 + p.tau_b / eps);
  const double bk = 1.0 / (double)K;
  // exponents of the form fl(1 / n): the Newton root (uniform)
  auto root_n = [](double e) {
    const double r = 1.0 / e;
    const int n = r >= 1.0 && r <= 64.0 ? (int)rint(r) : 0;
    return n >= 1 && 1.0 / (double)n == e ? n : 0;
  };
  const int na = GCS_SH_ROOT ? root_n(ua) : 0, nb = GCS_SH_ROOT ? root_n(vb) : 0;
  const double ina = na ? 1.0 / (double)na : 0.0, inb = nb ? 1.0 / (double)nb : 0.0;
  const float ina_f = (float)ina, inb_f = (float)inb;
  double apow[RPT];  // a^ua (the row's factor of u on the root path)
#pragma unroll
  for (int j = 0; j < RPT; ++j) apow[j] = na ? pow_fast(va[j], ua) : 0.0;
  const double bpow = nb ? pow_fast(bk, vb) : 0.0;
#if GCS_SH_LOGB
  // v = (b / (K^T u + 1e-12))^vb as exp(vb (log b - log K^T u)): log b once per call, no quotient in
  // the loop (as u; the short log / exp outside their ranges fall back to the quotient form)
  const double lbk = log(bk);
  auto v_scale = [&](double sum) {
    const double ss = sum + 1e-12;
    if (nb && ss >= kRootLo && ss <= kRootHi) {
      double y = root_seed(ss, inb_f);
      y = nb == 6 ? root_step_c<6>(y, ss, inb) : root_step(y, ss, nb, inb);
      y = nb == 6 ? root_step_c<6>(y, ss, inb) : root_step(y, ss, nb, inb);
      return bpow * y;
    }
    const double b_ = vb * (lbk - SH_LOG(ss));
    return ss >= 2.2250738585072014e-308 && ss <= 1.7976931348623157e308 && fabs(b_) < 700.0
               ? SH_EXP(b_)
               : pow_fast(div_fast(bk, ss), vb);
  };
#else
  auto v_scale = [&](double sum) { return pow_fast(div_fast(bk, sum + 1e-12), vb); };
#endif
  if (p.med)  // (else the pool kernel wrote K_mat)
#pragma unroll
    for (int q = 0; q < RPT * KM; ++q) X[q] = ((okm >> q) & 1u) ? exp(-X[q] / eps) : 0.0;
  SH_STAMP(2);
  double u[RPT], v[KM];
#pragma unroll
  for (int j = 0; j < RPT; ++j) u[j] = 1.0;
#pragma unroll
  for (int k = 0; k < KM; ++k) v[k] = 1.0;
  // K^T u from the row-major K_mat rows each thread already holds (no column-major copy: that copy,
  // 2 x RPT x KM doubles of registers, spilled): per thread its rows' column partials, then a
  // reduce-scatter across the wave (log2 KM halving exchanges leave lane L the column of its bits
  // 5..6-log2 KM, then xor adds inside each KM-lane group), then the waves in order.  Fixed order.
  static_assert(KM == 8 || KM == 16 || KM == 32, "reduce-scatter over 64 lanes");
  constexpr int LG = KM == 8 ? 3 : (KM == 16 ? 4 : 5);  // halving steps
  int col = 0;  // the column this lane ends up holding
#pragma unroll
  for (int s = 0; s < LG; ++s) col |= ((lane >> (5 - s)) & 1) << (LG - 1 - s);
#if GCS_SH_PROBE
  unsigned long long sh_pa[5] = {0, 0, 0, 0, 0}, sh_tp = wall_clock64();
#endif
  for (int it = 0; it < p.iters; ++it) {
    // u = (a / (K v + 1e-12))^ua, one lane per row (K v in column order)
    // ua = fl(1 / na): u = a^ua (K v + 1e-12)^(-1/na), the rows side by side (na = 6, the reference
    // defaults, with y^6 unrolled: the runtime-n squaring loop kept the rows' chains apart)
    auto root_rows = [&](auto nc) {
      constexpr int NC = decltype(nc)::value;
      double kvv[RPT], y[RPT];
      bool ok[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        double kv = 0.0;
#pragma unroll
        for (int k = 0; k < KM; ++k) kv = fma(X[j * KM + k], v[k], kv);
        kvv[j] = kv + 1e-12;
        ok[j] = kvv[j] >= kRootLo && kvv[j] <= kRootHi;
        y[j] = root_seed(ok[j] ? kvv[j] : 1.0, ina_f);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
          const double x = ok[j] ? kvv[j] : 1.0;
          y[j] = NC ? root_step_c<NC>(y[j], x, ina) : root_step(y[j], x, na, ina);
        }
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int r = t + j * kShThreads;
        double uj = apow[j] * y[j];
        if (!ok[j] && va[j] != 0.0) uj = pow_fast(div_fast(va[j], kvv[j]), ua);  // (rare: K v out of range)
        u[j] = r < N && va[j] != 0.0 ? uj : 0.0;
      }
    };
    if (na == 6) {
      root_rows(std::integral_constant<int, 6>{});
    } else if (na) {
      root_rows(std::integral_constant<int, 0>{});
    } else {
#if GCS_SH_LOGA && GCS_SH_ILV
    // the rows' chains side by side, branch-free (log and exp of an in-range stand-in where the row's
    // arguments are out of range), the rare fallback rows after them: the per-row branches serialised
    // the RPT chains (K v -> log -> exp), which is the loop's critical path
    {
      double kvv[RPT], a_[RPT], ue[RPT];
      bool ok[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        double kv = 0.0;
#pragma unroll
        for (int k = 0; k < KM; ++k) kv = fma(X[j * KM + k], v[k], kv);
        kvv[j] = kv + 1e-12;
        ok[j] = kvv[j] >= 2.2250738585072014e-308 && kvv[j] <= 1.7976931348623157e308;
      }
#if GCS_SH_TAB && GCS_SH_SPLIT
      // every row's table reads first, then the polynomials
      double lm[RPT], li[RPT], lh[RPT], ll[RPT];
      int le[RPT], lj[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        log_tab_reduce(ok[j] ? kvv[j] : 1.0, lm[j], le[j], lj[j]);
        li[j] = s_lt[3 * lj[j]];
        lh[j] = s_lt[3 * lj[j] + 1];
        ll[j] = s_lt[3 * lj[j] + 2];
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        a_[j] = ua * (lva[j] - log_tab_poly(lm[j], le[j], li[j], lh[j], ll[j]));
        ok[j] = ok[j] && fabs(a_[j]) < 700.0;
      }
      double er[RPT], eh[RPT], el[RPT];
      int em[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        int ej;
        exp_tab_reduce(ok[j] ? a_[j] : 0.0, er[j], ej, em[j]);
        eh[j] = s_et[2 * ej];
        el[j] = s_et[2 * ej + 1];
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) ue[j] = exp_tab_poly(er[j], em[j], eh[j], el[j]);
#else
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        a_[j] = ua * (lva[j] - SH_LOG(ok[j] ? kvv[j] : 1.0));
        // (NaN lva: a zero or denormal marginal; |a_| >= 700; NaN a_ fails the compare)
        ok[j] = ok[j] && fabs(a_[j]) < 700.0;
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) ue[j] = SH_EXP(ok[j] ? a_[j] : 0.0);
#endif
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int r = t + j * kShThreads;
        double uj = ue[j];
        // a zero marginal (an invalid row) gives u = 0 exactly (pow_sinkhorn(0, ua)) without the
        // fallback branch, so waves holding invalid rows do not diverge into it every iteration
#if GCS_SH_ZSKIP
        if (!ok[j] && va[j] != 0.0) uj = pow_fast(div_fast(va[j], kvv[j]), ua);
        u[j] = r < N && va[j] != 0.0 ? uj : 0.0;
#else
        if (!ok[j]) uj = pow_fast(div_fast(va[j], kvv[j]), ua);
        u[j] = r < N ? uj : 0.0;
#endif
      }
    }
#else
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int r = t + j * kShThreads;
      double kv = 0.0;
#pragma unroll
      for (int k = 0; k < KM; ++k) kv = fma(X[j * KM + k], v[k], kv);
#if GCS_SH_LOGA
      const double kvv = kv + 1e-12;
      double uj = 0.0;
      if (r < N) {
        const double a_ = ua * (lva[j] - SH_LOG(kvv));
        // (NaN lva: a zero or denormal marginal; a Kv outside the short log's range; |a_| >= 700)
        uj = kvv >= 2.2250738585072014e-308 && kvv <= 1.7976931348623157e308 && fabs(a_) < 700.0
                 ? SH_EXP(a_)
                 : pow_fast(div_fast(va[j], kvv), ua);
      }
      u[j] = uj;
#else
      u[j] = r < N ? pow_fast(div_fast(va[j], kv + 1e-12), ua) : 0.0;
#endif
    }
#endif
    }
    SH_ACC(0);
    double c[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      double sacc = 0.0;
#pragma unroll
      for (int j = 0; j < RPT; ++j) sacc = fma(X[j * KM + k], u[j], sacc);
      c[k] = sacc;
    }
    // reduce-scatter: step s exchanges half of the live values with a lane of the other half of its
    // 64 >> s group (GCS_SH_DPP: xlane's DPP / permlane pairings -- xor 32, 16, then the mirrors -- in
    // place of the ds_bpermute xor shuffles: each lane still ends with its column summed over all 64)
#pragma unroll
    for (int s = 0, n = KM; s < LG; ++s, n >>= 1) {
      const int h = n >> 1;
      const bool up = (lane >> (5 - s)) & 1;
#pragma unroll
      for (int i = 0; i < KM / 2; ++i) {
        if (i < h) {
          const double send = up ? c[i] : c[i + h];
          const double keep = up ? c[i + h] : c[i];
#if GCS_SH_DPP
          c[i] = keep + xlane_d(send, 5 - s, lane);
#else
          c[i] = keep + __shfl_xor(send, 32 >> s, 64);
#endif
        }
      }
    }
    double cs = c[0];
#if GCS_SH_DPP
#pragma unroll
    for (int st = 5 - LG; st >= 0; --st) cs += xlane_d(cs, st, lane);
#else
#pragma unroll
    for (int sh = (64 >> LG) / 2; sh >= 1; sh >>= 1) cs += __shfl_xor(cs, sh, 64);
#endif
#if GCS_SH_ONEBAR
    // every wave finishes v itself: lane k (< KM) sums column k over the waves in order and takes its
    // power, then v[k] comes from lane k.  The partials alternate between two buffers, so one barrier
    // per iteration separates a buffer's writes from its reads and from its next writes (a wave
    // rewriting it two iterations on has passed the barrier every reader reached after reading)
    double* cp = s_colp2[it & 1];
    if ((lane & ((64 >> LG) - 1)) == 0) cp[wid * KM + col] = cs;
    __syncthreads();
    double vk = 0.0;
    {
      const int kk = lane & (KM - 1);
      double sum = cp[kk];
#pragma unroll
      for (int g = 1; g < kShThreads / 64; ++g) sum += cp[g * KM + kk];
      if (kk < K) vk = v_scale(sum);
    }
    // v is wave-uniform: lane k's value read into scalar registers (no cross-lane permute)
    const unsigned long long vbits = (unsigned long long)__double_as_longlong(vk);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const unsigned lo = __builtin_amdgcn_readlane((unsigned)vbits, k);
      const unsigned hi = __builtin_amdgcn_readlane((unsigned)(vbits >> 32), k);
      v[k] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    }
#else
    if ((lane & ((64 >> LG) - 1)) == 0) s_colp[wid * KM + col] = cs;
    SH_ACC(1);
    __syncthreads();
    SH_ACC(2);
    if (t < K) {  // v = (b / (K^T u + 1e-12))^vb: column t over the waves in order
      double sum = s_colp[t];
#pragma unroll
      for (int g = 1; g < kShThreads / 64; ++g) sum += s_colp[g * KM + t];
      s_v[t] = v_scale(sum);
    }
    SH_ACC(3);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KM; ++k) v[k] = k < K ? s_v[k] : 0.0;
    SH_ACC(4);
#endif
  }
  SH_STAMP(3);
#if GCS_SH_PROBE
  if (t == 0)
    for (int k = 0; k < 5; ++k) g_sh_stamp[8 + k] = sh_pa[k];
#endif
#undef SH_LOG
#undef SH_EXP
  if (p.fin_split) {  // the finish runs in other workgroups: hand them u, v and sum a
    // (sc1 stores drained by every storing wave, then one flag store: the guide's R1 publish)
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int r = t + j * kShThreads;
      if (r < N) __hip_atomic_store(&w.su[r], u[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < KM; ++k) __hip_atomic_store(&w.su[N + k], v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&w.su[N + KM], sum_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p.fin_split == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) __hip_atomic_store(w.flag, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // pi, row masses, responsibilities and the cert sums
  // acc: [sum rm, sum rm^2, sum novel, defect_a^2, sum pi C, nonzero_a, sum pi | col masses K]
  double acc[7 + KM];
#pragma unroll
  for (int q = 0; q < 7 + KM; ++q) acc[q] = 0.0;
  // the cost rows and the row flags first, all loads in flight together: in the loop below every
  // load would wait behind the preceding resp store it may alias (8.6 us of serial round trips)
  // (the reference shape, 3 rows x 8 candidates; the wider instantiations keep the direct loads:
  // their registers are already at the limit)
  constexpr bool kPre = RPT * KM <= 24;
  double Cr[kPre ? RPT * KM : 1];
  bool rvj[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = t + j * kShThreads;
    rvj[j] = r < N && in.valid[r] != 0;
    if constexpr (kPre) {
#pragma unroll
      for (int k = 0; k < KM; ++k) Cr[j * KM + k] = r < N && k < K ? o.cost[(size_t)r * K + k] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = t + j * kShThreads;
    if (r >= N) continue;
    const bool rv = rvj[j];
    double rm = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= K) continue;
      const double pik = (u[j] * X[j * KM + k]) * v[k];
      rm += pik;
      if constexpr (kPre) acc[4] += pik * Cr[j * KM + k];
      else acc[4] += pik * o.cost[(size_t)r * K + k];
      acc[6] += pik;
      acc[7 + k] += pik;
      o.resp[(size_t)r * K + k] = rv ? pik : 0.0;
    }
    o.rmass[r] = rm;
    acc[0] += rm;
    acc[1] += rm * rm;
    acc[2] += fmax(va[j] - rm, 0.0);
    acc[3] += (rm - va[j]) * (rm - va[j]);
    acc[5] += va[j] > p.eps_mass ? 1.0 : 0.0;
  }
  SH_STAMP(6);
  bsum<7 + KM>(acc, s_red);
  SH_STAMP(7);
  if (t == 0) {
    double db = 0.0;
    for (int k = 0; k < K; ++k) db += (acc[7 + k] - bk) * (acc[7 + k] - bk);
    const double tm = acc[6];
    o.cert[CE_DEFECT_A] = sqrt(acc[3]);
    o.cert[CE_DEFECT_B] = sqrt(db);
    o.cert[CE_MASS_TOTAL] = tm;
    o.cert[CE_SUM_A] = sum_a;
    o.cert[CE_SUM_B] = bk * (double)K;
    o.cert[CE_SUM_M] = acc[0];
    o.cert[CE_SUM_NOVEL] = acc[2];
    o.cert[CE_P95_B] = bk;  // b uniform: every entry is 1 / K
    o.cert[CE_NONZERO_A] = acc[5];
    o.cert[CE_NONZERO_B] = bk > p.eps_mass ? (double)K : 0.0;
    o.cert[CE_ESS] = acc[0] * acc[0] / (acc[1] + p.eps_mass);
#if GCS_SH_PROBE
    g_sh_stamp[4] = wall_clock64();
#endif
    o.cert[CE_MASS_EPS] = p.eps_mass / (tm + p.eps_mass);
    o.cert[CE_TOTAL_COST] = acc[4];
    o.cert[CE_SUPPORT] = acc[5] / (double)std::max(N, 1);
    o.cert[CE_EXACT] = 0.0;
    o.cert[CE_MVALID] = (double)*w.mvalid;
    *w.mvalid_next = 0u;  // the next call's counter, armed (no per-call memset)
  }
}

// ---------------------------------------------------------------- visual pose evidence
// visual_pose_evidence (FS/backend/operators/visual_pose_evidence.py:260-412) over the first n_meas
// valid rows: one 1024-thread workgroup, each thread sums its strided rows in order, then a fixed
// tree.  Per row i (body mean p, direction u, kappa k, Lambda_reg = Lambda + eps I) and candidate j
// (view position m, direction v, kappa kv, responsibility r):
//   L_t += (sum_j r) Lambda_reg; h_t += Lambda_reg sum_j r (m - R p); cost_t += r q^T Lambda_reg q,
//   q = m - R p - t (:121-148);  w = r sqrt(k kv + 1e-12), S += w v u^T, cost_r += w (1 - (R u).v)
//   (:209-222).  out: L_t 9, h_t 3, cost_t, S 9, cost_r, sum row masses, rows used, map valid count.
#ifndef GCS_VPE_THREADS
#define GCS_VPE_THREADS 512  // 1024 capped the kernel at 128 VGPRs (73 spilled); at 512 it takes 193, no spills
#endif
constexpr int kVpeThreads = GCS_VPE_THREADS;
constexpr int kVpeVals = 27;
struct VpeIn {
  const double *Lambdas, *thetas, *etas;
  const uint8_t* valid;
  int n, n_lobes, n_meas;
  const int32_t* n_meas_dev;  // (may be null) the count on the device, read instead of n_meas
  const double *vpos, *vdir, *vkap;
  const uint8_t* vvalid;
  int m_view;
  const double *resp, *rmass;
  const int32_t* cand;
  int k;
  double R[9], t[3], eps_lift, eps_mass;
};

// the 25 sums of row i (L_t 9, h_t 3, cost_t, S 9, cost_r, row mass, 1), in the kernel's operation order
constexpr int kVpeRowVals = 25;
__device__ __forceinline__ void vpe_row(const VpeIn& in, int i, double* o) {
#pragma clang fp contract(off)
  double p[3];
  solve3_pivot(in.Lambdas + 9 * (size_t)i, in.eps_lift, in.thetas + 3 * (size_t)i, p);
  double es[3] = {0.0, 0.0, 0.0};
  for (int b = 0; b < in.n_lobes; ++b)
    for (int c = 0; c < 3; ++c) {
      const double e = in.etas[(size_t)3 * in.n_lobes * i + 3 * b + c];
      es[c] = b == 0 ? e : es[c] + e;
    }
  const double kap = sqrt((es[0] * es[0] + es[1] * es[1]) + es[2] * es[2]);
  const double u[3] = {es[0] / (kap + in.eps_mass), es[1] / (kap + in.eps_mass), es[2] / (kap + in.eps_mass)};
  double Lr[9];
  for (int c = 0; c < 9; ++c) Lr[c] = in.Lambdas[9 * (size_t)i + c] + ((c % 4) == 0 ? in.eps_lift : 0.0);
  double Rp[3], Ru[3];
  for (int r = 0; r < 3; ++r) {
    Rp[r] = (in.R[3 * r] * p[0] + in.R[3 * r + 1] * p[1]) + in.R[3 * r + 2] * p[2];
    Ru[r] = (in.R[3 * r] * u[0] + in.R[3 * r + 1] * u[1]) + in.R[3 * r + 2] * u[2];
  }
  double rs = 0.0, wt[3] = {0.0, 0.0, 0.0}, ct = 0.0, cr = 0.0, S[9];
  for (int c = 0; c < 9; ++c) S[c] = 0.0;
  for (int j = 0; j < in.k; ++j) {
    const double r = in.resp[(size_t)i * in.k + j];
    const int e = in.cand[(size_t)i * in.k + j];
    const double m[3] = {in.vpos[3 * (size_t)e], in.vpos[3 * (size_t)e + 1], in.vpos[3 * (size_t)e + 2]};
    const double vd[3] = {in.vdir[3 * (size_t)e], in.vdir[3 * (size_t)e + 1], in.vdir[3 * (size_t)e + 2]};
    rs = rs + r;
    double q[3], Lq[3];
    for (int c = 0; c < 3; ++c) {
      wt[c] = wt[c] + r * (m[c] - Rp[c]);
      q[c] = (m[c] - Rp[c]) - in.t[c];
    }
    for (int a = 0; a < 3; ++a) Lq[a] = (Lr[3 * a] * q[0] + Lr[3 * a + 1] * q[1]) + Lr[3 * a + 2] * q[2];
    ct = ct + r * ((q[0] * Lq[0] + q[1] * Lq[1]) + q[2] * Lq[2]);
    const double w = r * sqrt(kap * in.vkap[e] + 1e-12);
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) S[3 * a + b] = S[3 * a + b] + (w * vd[a]) * u[b];
    cr = cr + w * (1.0 - ((Ru[0] * vd[0] + Ru[1] * vd[1]) + Ru[2] * vd[2]));
  }
  for (int c = 0; c < 9; ++c) o[c] = rs * Lr[c];
  for (int a = 0; a < 3; ++a) o[9 + a] = (Lr[3 * a] * wt[0] + Lr[3 * a + 1] * wt[1]) + Lr[3 * a + 2] * wt[2];
  o[12] = ct;
  for (int c = 0; c < 9; ++c) o[13 + c] = S[c];
  o[22] = cr;
  o[23] = in.rmass[i];
  o[24] = 1.0;
}

// GCS_VPE_SPLIT (default): every valid row's sums computed by its own lane over the grid (k_as_vpe_rows,
// rows x 25 in rowv), then k_as_vpe adds them in its per-thread row order -- the same additions on the
// same values as the one-workgroup form (whose threads each walked three rows' candidate loads in
// series: 29 us at the reference sizes).
#ifndef GCS_VPE_SPLIT
#define GCS_VPE_SPLIT 1
#endif
__global__ __launch_bounds__(256) void k_as_vpe_rows(VpeIn in, double* __restrict__ rowv) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= in.n || !in.valid[i]) return;
  double o[kVpeRowVals];
  vpe_row(in, i, o);
#pragma unroll
  for (int q = 0; q < kVpeRowVals; ++q) rowv[(size_t)q * in.n + i] = o[q];
}

__global__ __launch_bounds__(kVpeThreads) void k_as_vpe(VpeIn in, const double* __restrict__ rowv, double* out) {
#pragma clang fp contract(off)
  __shared__ int s_w[kVpeThreads / 64];
  __shared__ double lds_all[(kVpeThreads / 64) * kVpeVals];
  double acc[kVpeVals];
  for (int q = 0; q < kVpeVals; ++q) acc[q] = 0.0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n_meas = in.n_meas_dev ? max(0, *in.n_meas_dev) : in.n_meas;
  int base = 0;  // valid rows before this chunk
  for (int c0 = 0; c0 < in.n; c0 += kVpeThreads) {
    const int i = c0 + threadIdx.x;
    const int v = i < in.n && in.valid[i] ? 1 : 0;
    int x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    int rank = base + x - v;
    for (int w = 0; w < wid; ++w) rank += s_w[w];
    int tot = 0;
    for (int w = 0; w < kVpeThreads / 64; ++w) tot += s_w[w];
    base += tot;
    if (!v || rank >= n_meas) continue;
    double o[kVpeRowVals];
    if (rowv) {
#pragma unroll
      for (int q = 0; q < kVpeRowVals; ++q) o[q] = rowv[(size_t)q * in.n + i];
    } else {
      vpe_row(in, i, o);
    }
#pragma unroll
    for (int q = 0; q < kVpeRowVals; ++q) acc[q] += o[q];
  }
  for (int e = threadIdx.x; e < in.m_view; e += kVpeThreads) acc[25] += in.vvalid[e] ? 1.0 : 0.0;
  // all 27 sums at once: the same xor tree per value in every wave, then thread q adds value q's wave
  // rows in wave order (the per-value form paid two barriers per value)
#pragma unroll
  for (int q = 0; q < kVpeVals; ++q)
    for (int off = 32; off >= 1; off >>= 1) acc[q] += __shfl_xor(acc[q], off, 64);
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < kVpeVals; ++q) lds_all[wid * kVpeVals + q] = acc[q];
  __syncthreads();
  if (threadIdx.x < kVpeVals) {
    const int q = threadIdx.x;
    double sum = lds_all[q];
    for (int w = 1; w < kVpeThreads / 64; ++w) sum += lds_all[w * kVpeVals + q];
    out[q] = sum;
  }
}

}  // namespace
}  // namespace gcs

using namespace gcs;

struct gcs_assoc_ctx {
  int device = 0;
  int max_meas = 0, max_pool = 0, max_k = 0;
  std::string err;
  hipStream_t own = nullptr, stream = nullptr;
  double *d_pos = nullptr, *d_dir = nullptr, *d_kap = nullptr, *d_A1 = nullptr, *d_A2 = nullptr, *d_dt = nullptr;
  int32_t *d_tix = nullptr, *d_cand = nullptr;
  uint32_t* d_mvalid = nullptr;  // two valid-entry counters, by call parity: a call's Sinkhorn zeroes the next's
  int mv_parity = 0;
  int st_ns = -1, st_rxy = -1, st_rz = -1;  // the stencil table in d_st
  int8_t* d_st = nullptr;
  double* h_cert = nullptr;  // pinned, mapped
  double* h_cert_dev = nullptr;
  double* h_vpe = nullptr;   // pinned, mapped: k_as_vpe's sums
  double* h_vpe_dev = nullptr;
  double* d_vpe_rows = nullptr;  // k_as_vpe_rows: 25 sums per row (field-major, max_meas rows)
  float4* d_vc = nullptr;        // k_as_stage: the view tiles' valid entries in f32 (max_pool entries)
  int32_t* d_vcnt = nullptr;     // k_as_stage: valid entries per view tile (kMaxBuckets)
  int32_t* d_order = nullptr;    // k_as_stage's row order: max_meas + kMaxBuckets x chunk
  double* d_kmat = nullptr;      // the pools' K_mat (max_meas x max_k)
  int32_t *d_ctile = nullptr, *d_cpre = nullptr;  // k_as_stage's chunk records (64 each per chunk)
  uint32_t* d_tcnt = nullptr;    // k_as_prep's per-view-tile valid counts (kMaxBuckets; zero between calls)
  double *d_su = nullptr, *d_fpart = nullptr;  // k_as_finish: u, v, sum a; per-workgroup sums
  uint32_t* d_ticket = nullptr;
  int fin_split = GCS_SH_FINSPLIT;  // GCSLAM_SH_FINSPLIT: 0 the Sinkhorn workgroup, 2 a launch of its own (A/B)
  uint32_t* d_flag = nullptr;        // the Sinkhorn's hand-off flag
  uint32_t* d_cstat = nullptr;       // the pools' per-row candidate statistics
  unsigned epoch = 0;
  bool pool_lds = GCS_POOL_LDS != 0;  // GCSLAM_POOL_LDS=0: k_as_pool from L2 for every view (A/B)
  bool prep_fused = GCS_PREP_FUSED != 0;  // GCSLAM_PREP_FUSED=1: k_as_prep and k_as_stage as one launch (A/B)
  bool vpe_split = GCS_VPE_SPLIT != 0;  // GCSLAM_VPE_SPLIT=0: the one-workgroup form (A/B, bitwise test)
  int probe_iters = 0;       // GCS_SH_PROBE builds: the last launch's Sinkhorn iterations
  int probe_rows = 0;        // GCS_POOL_PROBE builds: the last launch's rows
};

namespace {
int as_fail(gcs_assoc_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}
#define ASCHK(ctx, expr)                                                                          \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return as_fail((ctx), GCS_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

// rows per Sinkhorn thread for k_assoc <= KM: the K_mat rows stay in registers (both layouts)
constexpr int rpt_for(int km) { return kShCR / km > 1 ? kShCR / km : 1; }  // rows per Sinkhorn thread
constexpr int max_rows_for(int max_k) { return kShCR * kShThreads / (max_k <= 8 ? 8 : (max_k <= 16 ? 16 : 32)); }
}  // namespace

extern "C" {

int gcs_debug_short_log_exp(const double* x, int32_t n, double y, double* log_out, double* exp_out, double* pow_out) {
  if (n < 0 || (n > 0 && (!x || !log_out || !exp_out || !pow_out))) return GCS_ERR_ARG;
  for (int i = 0; i < n; ++i) {
    log_out[i] = x[i] > 0.0 ? gcs::log_short(x[i]) : NAN;
    exp_out[i] = fabs(x[i]) < 700.0 ? gcs::exp_short(x[i]) : NAN;
    pow_out[i] = gcs::pow_sinkhorn(x[i], y);
  }
  return GCS_OK;
}

int gcs_debug_tab_log_exp(const double* x, int32_t n, double* log_out, double* exp_out) {
  if (n < 0 || (n > 0 && (!x || !log_out || !exp_out))) return GCS_ERR_ARG;
  for (int i = 0; i < n; ++i) {
    log_out[i] = x[i] >= 2.2250738585072014e-308 && x[i] <= 1.7976931348623157e308 ? gcs::log_tab(x[i], gcs::kShLogTab)
                                                                                  : NAN;
    exp_out[i] = fabs(x[i]) < 700.0 ? gcs::exp_tab(x[i], gcs::kShExpTab) : NAN;
  }
  return GCS_OK;
}

int gcs_assoc_config_defaults(gcs_assoc_config* c) {
  if (!c) return GCS_ERR_ARG;
  memset(c, 0, sizeof(*c));
  c->k_assoc = 8;       // GC_K_ASSOC, constants.py:356
  c->k_sinkhorn = 50;   // GC_K_SINKHORN, constants.py:357
  c->beta = 0.5;        // primitive_association.py:219-222
  c->epsilon = 0.1;
  c->tau_a = 0.5;
  c->tau_b = 0.5;
  c->cost_subtract_row_min = 1;
  c->cost_scale_by_median = 0;
  c->a_policy = GCS_ASSOC_A_UNIFORM;
  c->b_policy = GCS_ASSOC_B_UNIFORM;
  c->eps_mass = 1e-12;  // GC_EPS_MASS
  c->eps_lift = 1e-9;   // GC_EPS_LIFT
  c->eps_mass_dir = 1e-12;
  c->h_tile = 2.0;      // GC_H_TILE, constants.py:408
  c->r_stencil_tiles_xy = 1;  // constants.py:415-416
  c->r_stencil_tiles_z = 0;
  c->scan_seq = 0;
  c->recency_decay_lambda = 0.02;  // GC_RECENCY_DECAY_LAMBDA, constants.py:419
  return GCS_OK;
}

const char* gcs_assoc_last_error(const gcs_assoc_ctx* c) { return c ? c->err.c_str() : "null association context"; }

int gcs_assoc_ctx_destroy(gcs_assoc_ctx* c) {
  if (!c) return GCS_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_pos, c->d_dir, c->d_kap, c->d_A1, c->d_A2, c->d_dt, c->d_tix, c->d_cand, c->d_mvalid, c->d_st,
                  c->d_vpe_rows, c->d_vc, c->d_vcnt, c->d_order, c->d_kmat, c->d_su, c->d_fpart, c->d_ticket, c->d_ctile, c->d_cpre, c->d_tcnt, c->d_flag, c->d_cstat};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->h_cert) (void)hipHostFree(c->h_cert);
  if (c->h_vpe) (void)hipHostFree(c->h_vpe);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return GCS_OK;
}

int gcs_assoc_ctx_create(int32_t max_meas, int32_t max_pool, int32_t max_k, int32_t device, gcs_assoc_ctx** out) {
  if (!out) return GCS_ERR_ARG;
  *out = nullptr;
  if (max_meas < 1 || max_pool < 1 || max_k < 1 || max_k > 32 || max_meas > max_rows_for(max_k))
    return GCS_ERR_ARG;
  auto* c = new gcs_assoc_ctx();
  c->device = device;
  c->max_meas = max_meas;
  c->max_pool = max_pool;
  c->max_k = max_k;
  auto bad = [](hipError_t e) { return e != hipSuccess; };
  const size_t N = (size_t)max_meas, M = (size_t)max_pool, NK = N * (size_t)max_k;
  if (bad(hipSetDevice(device)) || bad(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) ||
      bad(hipMalloc(&c->d_pos, N * 3 * 8)) || bad(hipMalloc(&c->d_dir, N * 3 * 8)) || bad(hipMalloc(&c->d_kap, N * 8)) ||
      bad(hipMalloc(&c->d_A1, N * 8)) || bad(hipMalloc(&c->d_A2, M * 8)) || bad(hipMalloc(&c->d_dt, NK * 8)) ||
      bad(hipMalloc(&c->d_tix, N * kMaxStencil * 4)) || bad(hipMalloc(&c->d_cand, NK * 4)) ||
      bad(hipMalloc(&c->d_mvalid, 8)) || bad(hipMalloc(&c->d_st, kMaxStencil * 3)) ||
      bad(hipMalloc(&c->d_vpe_rows, N * kVpeRowVals * 8)) || bad(hipMalloc(&c->d_vc, M * sizeof(float4))) || bad(hipMalloc(&c->d_kmat, NK * 8)) ||
      bad(hipMalloc(&c->d_su, (N + 40) * 8)) || bad(hipMalloc(&c->d_fpart, ((N + kFinThreads - 1) / kFinThreads) * 40 * 8)) ||
      bad(hipMalloc(&c->d_ticket, 4)) ||
      bad(hipMalloc(&c->d_ctile, (N / kPoolLdsWaves + kMaxBuckets + 1) * 64 * 4)) ||
      bad(hipMalloc(&c->d_cpre, (N / kPoolLdsWaves + kMaxBuckets + 1) * 64 * 4)) || bad(hipMalloc(&c->d_tcnt, kMaxBuckets * 4)) || bad(hipMalloc(&c->d_flag, 4)) || bad(hipMalloc(&c->d_cstat, N * 4)) || bad(hipMalloc(&c->d_vcnt, kMaxBuckets * 4)) ||
      bad(hipMalloc(&c->d_order, (N + (size_t)kMaxBuckets * kPoolLdsWaves) * 4)) ||
      bad(hipHostMalloc(&c->h_cert, GCS_ASSOC_CERT_LEN * sizeof(double), hipHostMallocMapped)) ||
      bad(hipHostGetDevicePointer((void**)&c->h_cert_dev, c->h_cert, 0)) ||
      bad(hipHostMalloc(&c->h_vpe, 32 * sizeof(double), hipHostMallocMapped)) ||
      bad(hipHostGetDevicePointer((void**)&c->h_vpe_dev, c->h_vpe, 0))) {
    gcs_assoc_ctx_destroy(c);
    return GCS_ERR_HIP;
  }
  if (bad(hipMemset(c->d_mvalid, 0, 8)) || bad(hipMemset(c->d_ticket, 0, 4)) || bad(hipMemset(c->d_tcnt, 0, kMaxBuckets * 4)) || bad(hipMemset(c->d_flag, 0, 4)) ||
      bad(hipStreamSynchronize(nullptr))) {  // (null-stream clears: done before the context's stream runs)
    gcs_assoc_ctx_destroy(c);
    return GCS_ERR_HIP;
  }
  if (const char* e = getenv("GCSLAM_VPE_SPLIT")) c->vpe_split = atoi(e) != 0;
  if (const char* e = getenv("GCSLAM_POOL_LDS")) c->pool_lds = atoi(e) != 0;
  if (const char* e = getenv("GCSLAM_PREP_FUSED")) c->prep_fused = atoi(e) != 0;
  if (const char* e = getenv("GCSLAM_SH_FINSPLIT")) c->fin_split = atoi(e);
  // the LDS pool's dynamic LDS reaches 160 KB (the view table + the waves' rings)
  (void)hipFuncSetAttribute((const void*)k_as_pool_lds<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipGetLastError();
  (void)hipFuncSetAttribute((const void*)k_as_pool_lds<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)k_as_pool_lds<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  c->stream = c->own;
  *out = c;
  return GCS_OK;
}

int gcs_assoc_ctx_set_stream(gcs_assoc_ctx* c, void* stream) {
  if (!c) return GCS_ERR_ARG;
  hipStream_t ns = stream ? (hipStream_t)stream : c->own;
  if (ns == c->stream) return GCS_OK;
  ASCHK(c, hipSetDevice(c->device));
  ASCHK(c, hipStreamSynchronize(c->stream));  // work queued on the old stream completes first
  c->stream = ns;
  return GCS_OK;
}

}  // extern "C"

namespace gcs {
namespace live {
int assoc_launch(gcs_assoc_ctx* c, const gcs_assoc_config* cfg, const gcs_assoc_meas* m, const gcs_assoc_view* v,
                 gcs_assoc_outputs* o, const int32_t* n_valid_dev) {
  if (!c || !cfg || !m || !v || !o) return GCS_ERR_ARG;
  if (!o->responsibilities || !o->row_masses || !o->cost_matrix)
    return as_fail(c, GCS_ERR_ARG, "responsibilities, row_masses and cost_matrix are required outputs");
  const int K = cfg->k_assoc;
  if (K < 1 || K > c->max_k) return as_fail(c, GCS_ERR_ARG, "k_assoc outside [1, max_k] of the context");
  if (m->n_total < 1 || m->n_total > c->max_meas) return as_fail(c, GCS_ERR_ARG, "n_total outside [1, max_meas]");
  if (m->n_lobes < 1) return as_fail(c, GCS_ERR_ARG, "n_lobes < 1");
  // an unsupported policy raises only past the empty-case return, as in the reference (:272 vs :413-437)
  const char* bad_policy = nullptr;
  if (cfg->a_policy != GCS_ASSOC_A_UNIFORM && cfg->a_policy != GCS_ASSOC_A_WEIGHT)
    bad_policy = "Unsupported measurement mass policy: only UNIFORM and WEIGHT_PROPORTIONAL are implemented";
  else if (cfg->b_policy != GCS_ASSOC_B_UNIFORM)
    bad_policy = "Unsupported map mass policy: only UNIFORM is implemented";
  if (v->m_tile_view <= 0) return as_fail(c, GCS_ERR_ARG, "m_tile_view must be > 0");
  if (v->n_tiles < 1) return as_fail(c, GCS_ERR_ARG, "the view needs at least one tile");
  const long pool = (long)v->n_tiles * v->m_tile_view;
  if (pool > c->max_pool) return as_fail(c, GCS_ERR_ARG, "view entries exceed max_pool");
  if (cfg->r_stencil_tiles_xy < 0 || cfg->r_stencil_tiles_z < 0 || cfg->k_sinkhorn < 0)
    return as_fail(c, GCS_ERR_ARG, "negative stencil radius or iteration count");
  // stencil offsets, z slab outer, sorted axial disk inner (tiling.py:171-186; :309-336)
  int8_t st[kMaxStencil * 3];
  int ns = 0;
  const int rxy = cfg->r_stencil_tiles_xy, rz = cfg->r_stencil_tiles_z;
  for (int z = -rz; z <= rz; ++z)
    for (int q = -rxy; q <= rxy; ++q)
      for (int r = std::max(-rxy, -q - rxy); r <= std::min(rxy, -q + rxy); ++r) {
        if (ns >= kMaxStencil) return as_fail(c, GCS_ERR_ARG, "stencil exceeds 64 tiles");
        st[3 * ns] = (int8_t)q;
        st[3 * ns + 1] = (int8_t)r;
        st[3 * ns + 2] = (int8_t)z;
        ++ns;
      }
  if ((long)ns * v->m_tile_view < K) return as_fail(c, GCS_ERR_ARG, "pool smaller than k_assoc");
  int s_center = -1;
  for (int q = 0; q < ns; ++q)
    if (st[3 * q] == 0 && st[3 * q + 1] == 0 && st[3 * q + 2] == 0) s_center = q;
  ASCHK(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  AsParams p{};
  p.n = m->n_total;
  p.m_view = v->m_tile_view;
  p.m_shift = -1;
  for (int b = 0; b < 31; ++b)
    if ((1 << b) == p.m_view) p.m_shift = b;
  p.n_tiles = v->n_tiles;
  p.n_stencil = ns;
  p.k = K;
  p.iters = cfg->k_sinkhorn;
  p.m_pool = (int)pool;
  p.s_center = s_center;
  p.a_policy = cfg->a_policy == GCS_ASSOC_A_WEIGHT ? 1 : 0;
  p.row_min = cfg->cost_subtract_row_min != 0;
  p.med = cfg->cost_scale_by_median != 0;
  p.fin_split = !bad_policy && c->fin_split >= 1 && c->fin_split <= 2 ? c->fin_split : 0;
  if (++c->epoch == 0u) c->epoch = 1u;
  p.epoch = c->epoch;
  p.beta = cfg->beta;
  p.eps = cfg->epsilon;
  p.tau_a = cfg->tau_a;
  p.tau_b = cfg->tau_b;
  p.eps_mass = cfg->eps_mass;
  p.eps_lift = cfg->eps_lift;
  p.eps_dir = cfg->eps_mass_dir;
  p.h = std::max(cfg->h_tile, 1e-12);
  p.lam = cfg->recency_decay_lambda;
  p.eps_lam = cfg->epsilon * cfg->recency_decay_lambda;  // float(epsilon) * float(lambda) first (:397)
  p.scan_seq = (long long)cfg->scan_seq;
  AsIn in{m->Lambdas, m->thetas, m->etas, m->weights, m->valid_mask, m->n_lobes, v->tile_ids, v->positions,
          v->directions, v->kappas, v->valid_mask, v->last_supported_scan_seq, v->candidate_tile_ids,
          v->candidate_slots};
  uint32_t* mv = c->d_mvalid + c->mv_parity;
  uint32_t* mv_next = c->d_mvalid + (c->mv_parity ^ 1);
  c->mv_parity ^= 1;
  // the bucketed pool (k_as_pool_lds) for views of at most kMaxBuckets - 1 tiles
  const bool bucketed = c->pool_lds && !bad_policy && v->n_tiles + 1 <= kMaxBuckets && m->n_total <= kBucketRows * 1024;
  AsWork w{c->d_pos, c->d_dir, c->d_kap, c->d_A1, c->d_A2, c->d_dt, c->d_tix, c->d_cand, mv, mv_next, c->d_vc, c->d_vcnt,
           c->d_order, c->d_ctile, c->d_cpre, c->d_tcnt, c->d_kmat, bucketed ? kPoolLdsWaves : 0, c->d_su, c->d_fpart, c->d_ticket, c->d_flag, c->d_cstat};
  AsOut out{o->responsibilities, o->row_masses, o->cost_matrix, o->candidate_pool_indices, o->candidate_tile_ids,
            o->candidate_slots, c->h_cert_dev};
  if (ns != c->st_ns || rxy != c->st_rxy || rz != c->st_rz) {  // the stencil table changes with the radii only
    ASCHK(c, hipStreamSynchronize(s));
    ASCHK(c, hipMemcpy(c->d_st, st, (size_t)ns * 3, hipMemcpyHostToDevice));
    ASCHK(c, hipStreamSynchronize(nullptr));  // (a pageable copy may return before its DMA lands)
    c->st_ns = ns;
    c->st_rxy = rxy;
    c->st_rz = rz;
  }
  // (the valid-entry counter k_as_prep adds to is re-armed by the Sinkhorn kernel that reads it)
  const int nprep = (int)((p.n + pool + kAsThreads - 1) / kAsThreads);
  // (the fused prep: prep + stage in one launch -- bucketed pools on views of <= kFusedTiles tiles)
  const bool fused_prep = bucketed && c->prep_fused && v->n_tiles <= kFusedTiles &&
                          (long)p.n + (long)(v->n_tiles + 1) * kPoolLdsWaves <= (long)kMaxBuckets * 8;
  if (fused_prep) {
    const int lane_blocks = (int)((p.n + pool + 1023) / 1024);
    const int cap = p.n + (v->n_tiles + 1) * kPoolLdsWaves;
    hipLaunchKernelGGL(k_as_prep_fused, dim3(lane_blocks + v->n_tiles + 1), dim3(1024), 0, s, in, p, w,
                       (const int8_t*)c->d_st, lane_blocks, cap);
  } else {
    hipLaunchKernelGGL(k_as_prep, dim3(nprep), dim3(kAsThreads), 0, s, in, p, w, (const int8_t*)c->d_st);
  }
  // every return between here and the Sinkhorn's launch skips the kernel that zeroes the next
  // call's counter: this guard zeroes it instead (the next call would otherwise start from the
  // count of the call before this one)
  struct RearmNext {
    uint32_t* next;
    bool armed = true;
    ~RearmNext() {
      if (armed) {
        (void)hipMemset(next, 0, 4);
        (void)hipStreamSynchronize(nullptr);  // (the null stream does not order the context's stream)
      }
    }
  } rearm{mv_next};
  const int km = K <= 8 ? 8 : (K <= 16 ? 16 : 32);
  // the pool: the whole view staged in LDS when it fits (one wave per row, as many waves per
  // workgroup as spread the rows over 256 workgroups), else one 128-thread workgroup per row from L2
  auto launch_pool = [&](auto k_l2, auto k_lds) {
    if (bucketed) {
      const int nb = v->n_tiles + 1;
      const int cap = p.n + nb * kPoolLdsWaves;  // rows + every bucket's padding, at most
      if (!fused_prep) hipLaunchKernelGGL(k_as_stage, dim3(v->n_tiles + 1), dim3(1024), 0, s, in, p, w, nb, cap);
      const int lds_slots = (long)ns * p.m_view <= kPoolLdsMaxView ? ns * p.m_view : 0;
      const size_t lds = (size_t)lds_slots * 16 + (size_t)kPoolLdsWaves * kLRing * 8;
      hipLaunchKernelGGL(k_lds, dim3((cap + kPoolLdsWaves - 1) / kPoolLdsWaves), dim3(kPoolLdsWaves * 64), lds, s, in, p,
                         w, out, lds_slots);
    } else {
      hipLaunchKernelGGL(k_l2, dim3(p.n), dim3(kPoolThreads), 0, s, in, p, w, out);
    }
  };
  if (bad_policy) {
    uint32_t mvh = 0;
    int32_t nvh = m->n_valid;
    ASCHK(c, hipMemcpyAsync(&mvh, mv, 4, hipMemcpyDeviceToHost, s));
    if (n_valid_dev) ASCHK(c, hipMemcpyAsync(&nvh, n_valid_dev, 4, hipMemcpyDeviceToHost, s));
    ASCHK(c, hipStreamSynchronize(s));
    if (nvh != 0 && mvh != 0) return as_fail(c, GCS_ERR_ARG, bad_policy);  // rearm zeroes the next counter
    // empty: the Sinkhorn kernel's zero path writes the reference's empty result
  }
  const int nfin = (p.n + kFinThreads - 1) / kFinThreads;  // (GCS_SH_FINSPLIT 2)
  const int gsh = 2 + (p.fin_split == 1 ? (p.n + kShThreads - 1) / kShThreads : 0);  // the Sinkhorn's grid
  if (bad_policy) {
    hipLaunchKernelGGL((k_as_sinkhorn<8, rpt_for(8)>), dim3(2), dim3(kShThreads), 0, s, in, p, w, out, 0, (const int32_t*)nullptr);
  } else if (km == 8) {
    launch_pool(k_as_pool<8>, k_as_pool_lds<8>);
    // three rows per thread when they cover the rows (the reference's 1,536 = 3 x 512): no padding
    // row in the K v / K^T u sums
    if (3 * kShThreads < rpt_for(8) * kShThreads && p.n <= 3 * kShThreads)
      hipLaunchKernelGGL((k_as_sinkhorn<8, 3>), dim3(gsh), dim3(kShThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
    else
      hipLaunchKernelGGL((k_as_sinkhorn<8, rpt_for(8)>), dim3(gsh), dim3(kShThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
    if (p.fin_split == 2)
      hipLaunchKernelGGL(k_as_finish<8>, dim3(nfin), dim3(kFinThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
  } else if (km == 16) {
    launch_pool(k_as_pool<16>, k_as_pool_lds<16>);
    hipLaunchKernelGGL((k_as_sinkhorn<16, rpt_for(16)>), dim3(gsh), dim3(kShThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
    if (p.fin_split == 2)
      hipLaunchKernelGGL(k_as_finish<16>, dim3(nfin), dim3(kFinThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
  } else {
    launch_pool(k_as_pool<32>, k_as_pool_lds<32>);
    hipLaunchKernelGGL((k_as_sinkhorn<32, rpt_for(32)>), dim3(gsh), dim3(kShThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
    if (p.fin_split == 2)
      hipLaunchKernelGGL(k_as_finish<32>, dim3(nfin), dim3(kFinThreads), 0, s, in, p, w, out, m->n_valid, n_valid_dev);
  }
  ASCHK(c, hipGetLastError());
  rearm.armed = false;  // the Sinkhorn is queued: it zeroes mv_next
  c->probe_iters = p.iters;
  c->probe_rows = p.n;
  return GCS_OK;
}

int assoc_bind_stream(gcs_assoc_ctx* c, void* s) {
  if ((hipStream_t)s == c->stream) return GCS_OK;
  ASCHK(c, hipSetDevice(c->device));
  ASCHK(c, hipStreamSynchronize(c->stream));
  c->stream = (hipStream_t)s;
  return GCS_OK;
}

void assoc_collect(gcs_assoc_ctx* c, gcs_assoc_outputs* o) {
#if GCS_SH_PROBE
  {
    unsigned long long h[16];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sh_stamp), sizeof(h));
    fprintf(stderr, "sh_probe us: marginal %.2f kmat %.2f loop %.2f finish %.2f (pi %.2f bsum %.2f cert %.2f) | wg1 %.2f\n",
            (h[1] - h[0]) / 100.0, (h[2] - h[1]) / 100.0, (h[3] - h[2]) / 100.0, (h[4] - h[3]) / 100.0,
            (h[6] - h[3]) / 100.0, (h[7] - h[6]) / 100.0, (h[4] - h[7]) / 100.0, (h[5] - h[0]) / 100.0);
    const double it = c->probe_iters > 0 ? 100.0 * c->probe_iters : 1.0;  // per iteration, us
    fprintf(stderr, "sh_probe per iteration us: u %.3f KTu+scatter %.3f barrier1 %.3f v %.3f barrier2+read %.3f\n",
            h[8] / it, h[9] / it, h[10] / it, h[11] / it, h[12] / it);
  }
#endif
#if GCS_POOL_PROBE
  {
    static unsigned long long h[4096 * 10];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pool_probe), sizeof(h));
    const int n = std::min(c->probe_rows, 4096);
    double sum[8] = {0}, mx[8] = {0}, ring = 0, rmax = 0;
    int slow = 0, cnt = 0;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int i = 0; i < n; ++i) {
      const unsigned long long* r = h + (size_t)i * 10;
      if (!r[0] || !r[7]) continue;  // invalid rows skip stamps 2..6
      ++cnt;
      t0 = std::min(t0, r[0]);
      t1 = std::max(t1, r[7]);
      for (int k = 1; k < 8; ++k) {
        unsigned long long prev = r[k - 1];
        for (int j = k - 1; j >= 0 && !prev; --j) prev = r[j];
        const double d = r[k] ? (double)(r[k] - prev) / 100.0 : 0.0;
        sum[k] += d;
        mx[k] = std::max(mx[k], d);
      }
      ring += (double)r[8];
      rmax = std::max(rmax, (double)r[8]);
      slow += (int)r[9];
    }
    if (cnt)
      fprintf(stderr, "pool_probe rows %d span %.2f us | mean/max us: stage %.2f/%.2f pro %.2f/%.2f pass1 %.2f/%.2f "
              "ring %.2f/%.2f merge %.2f/%.2f slow %.2f/%.2f final %.2f/%.2f | ring %.1f/%.0f slow rows %d\n",
              cnt, (t1 - t0) / 100.0, sum[1] / cnt, mx[1], sum[2] / cnt, mx[2], sum[3] / cnt, mx[3], sum[4] / cnt, mx[4],
              sum[5] / cnt, mx[5], sum[6] / cnt, mx[6], sum[7] / cnt, mx[7], ring / cnt, rmax, slow);
  }
#endif
  for (int q = 0; q < GCS_ASSOC_CERT_LEN; ++q) o->cert[q] = c->h_cert[q];
  o->exact = c->h_cert[CE_EXACT] != 0.0;
  o->n_map_valid = (int32_t)c->h_cert[CE_MVALID];
}
}  // namespace live
}  // namespace gcs

extern "C" {
int gcs_associate_primitives_ot(gcs_assoc_ctx* c, const gcs_assoc_config* cfg, const gcs_assoc_meas* m,
                                const gcs_assoc_view* v, gcs_assoc_outputs* o) {
  if (int rc = gcs::live::assoc_launch(c, cfg, m, v, o)) return rc;
  ASCHK(c, hipStreamSynchronize(c->stream));
  gcs::live::assoc_collect(c, o);
  return GCS_OK;
}

int gcs_visual_pose_evidence(gcs_assoc_ctx* c, const gcs_assoc_meas* m, const gcs_assoc_view* v,
                             const double* responsibilities, const int32_t* candidate_pool_indices,
                             const double* row_masses, int32_t k_assoc, const double* z_lin_pose, double eps_lift,
                             double eps_mass, gcs_vpe_outputs* o) {
  if (!o) return GCS_ERR_ARG;
  if (int rc = gcs::live::vpe_launch(c, m, v, responsibilities, candidate_pool_indices, row_masses, k_assoc,
                                     z_lin_pose, eps_lift, eps_mass))
    return rc;
  ASCHK(c, hipStreamSynchronize(c->stream));
  gcs::live::vpe_collect(c, m->n_valid, k_assoc, z_lin_pose, eps_lift, o);
  return GCS_OK;
}
}  // extern "C"

namespace gcs {
namespace live {
int vpe_launch(gcs_assoc_ctx* c, const gcs_assoc_meas* m, const gcs_assoc_view* v, const double* responsibilities,
               const int32_t* candidate_pool_indices, const double* row_masses, int32_t k_assoc,
               const double* z_lin_pose, double eps_lift, double eps_mass, const int32_t* n_valid_dev) {
  if (!c || !m || !v || !z_lin_pose) return GCS_ERR_ARG;
  if (m->n_total < 1 || k_assoc < 1 || !responsibilities || !candidate_pool_indices || !row_masses || !m->Lambdas ||
      !m->thetas || !m->etas || !m->valid_mask || !v->positions || !v->directions || !v->kappas || !v->valid_mask)
    return as_fail(c, GCS_ERR_ARG, "visual_pose_evidence: missing measurement, view or association array");
  ASCHK(c, hipSetDevice(c->device));
  VpeIn in{};
  in.Lambdas = m->Lambdas;
  in.thetas = m->thetas;
  in.etas = m->etas;
  in.valid = m->valid_mask;
  in.n = m->n_total;
  in.n_lobes = m->n_lobes;
  in.n_meas = std::max(0, m->n_valid);
  in.n_meas_dev = n_valid_dev;
  in.vpos = v->positions;
  in.vdir = v->directions;
  in.vkap = v->kappas;
  in.vvalid = v->valid_mask;
  in.m_view = v->n_tiles * v->m_tile_view;
  in.resp = responsibilities;
  in.rmass = row_masses;
  in.cand = candidate_pool_indices;
  in.k = k_assoc;
  so3_exp(z_lin_pose + 3, in.R);
  for (int q = 0; q < 3; ++q) in.t[q] = z_lin_pose[q];
  in.eps_lift = eps_lift;
  in.eps_mass = eps_mass;
  if (c->vpe_split && in.n <= c->max_meas) {
    hipLaunchKernelGGL(k_as_vpe_rows, dim3((in.n + 255) / 256), dim3(256), 0, c->stream, in, c->d_vpe_rows);
    hipLaunchKernelGGL(k_as_vpe, dim3(1), dim3(kVpeThreads), 0, c->stream, in, (const double*)c->d_vpe_rows,
                       c->h_vpe_dev);
  } else {
    hipLaunchKernelGGL(k_as_vpe, dim3(1), dim3(kVpeThreads), 0, c->stream, in, (const double*)nullptr, c->h_vpe_dev);
  }
  ASCHK(c, hipGetLastError());
  return GCS_OK;
}

void vpe_collect(gcs_assoc_ctx* c, int32_t n_valid, int32_t k_assoc, const double* z_lin_pose, double eps_lift,
                 gcs_vpe_outputs* o) {
  double Rz[9];
  so3_exp(z_lin_pose + 3, Rz);
  const double* a = c->h_vpe;
  memset(o, 0, sizeof(*o));
  for (int q = 0; q < 22; ++q) o->L_pose[23 * q] = eps_lift;
  const int rows = (int)a[24];
  if (n_valid == 0 || rows == 0 || a[25] == 0.0) {  // the empty case (:293-318)
    o->exact = 1;
    return;
  }
  for (int q = 0; q < 9; ++q) o->L_trans[q] = a[q] + ((q % 4) == 0 ? eps_lift : 0.0);
  for (int q = 0; q < 3; ++q) o->h_trans[q] = a[9 + q];
  // rotation: SVD of the scatter, det-fixed U V^T, R_delta = R_scatter R_pred^T, h = diag(s + eps) log(R_delta)
  double U[9], sv[3], V[9];
  svd3(a + 13, U, sv, V);
  double Rs[9];
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q) Rs[3 * r + q] = (U[3 * r] * V[3 * q] + U[3 * r + 1] * V[3 * q + 1]) + U[3 * r + 2] * V[3 * q + 2];
  if (det3(Rs) < 0.0)
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q)
        Rs[3 * r + q] = (U[3 * r] * V[3 * q] + U[3 * r + 1] * V[3 * q + 1]) - U[3 * r + 2] * V[3 * q + 2];
  double Rd[9];
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q)
      Rd[3 * r + q] = (Rs[3 * r] * Rz[3 * q] + Rs[3 * r + 1] * Rz[3 * q + 1]) + Rs[3 * r + 2] * Rz[3 * q + 2];
  double w[3];
  so3_log(Rd, w);
  for (int q = 0; q < 3; ++q) {
    o->L_rot[4 * q] = sv[q] + eps_lift;
    o->h_rot[q] = o->L_rot[4 * q] * w[q];
  }
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q) {
      o->L_pose[22 * r + q] = o->L_trans[3 * r + q];
      o->L_pose[22 * (3 + r) + 3 + q] = o->L_rot[3 * r + q];
    }
  for (int q = 0; q < 3; ++q) {
    o->h_pose[q] = o->h_trans[q];
    o->h_pose[3 + q] = o->h_rot[q];
  }
  o->total_weighted_cost = a[12] + a[22];
  o->n_associations = rows * k_assoc;
  o->mean_transported_mass = a[23] / (double)rows;
  o->ess_total = a[23];
  o->support_frac = (double)rows / (double)std::max(n_valid, 1);
  o->exact = 0;
}
}  // namespace live
}  // namespace gcs

extern "C" {

}  // extern "C"
