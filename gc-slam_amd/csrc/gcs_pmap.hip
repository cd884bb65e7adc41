// The primitive map resident in HBM and its maintenance operators on gfx950 -- the live primitive
// path's map side, FS/backend/structures/primitive_map.py:
//
//   storage        max_tiles tiles x m_tile slots; per field [tile][slot][width] (the reference's
//                  PrimitiveMapTile array shapes, :98-174), f64 / i64 / u8
//   k_pm_keys      one lane per slot: the single sort key of _select_topk_slots_fixed (-score, :316-319)
//                  or _select_lowest_mass_slots_fixed (retention, :345-351) in order-preserving u64 bits
//                  (-0.0 and 0.0 equal, as lax.sort's comparator), value = slot; then a stable
//                  radix sort (rocPRIM) of all listed tiles' keys followed by a stable radix sort on the
//                  tile position: per tile, the key order with ties by slot
//   k_pm_view      one lane per view entry: the tile's r-th slot, mean (LU solve of Lambda + eps I),
//                  covariance, resultant direction and kappa (:474-498)
//   k_pm_insert    one workgroup: tile by tile, the masked proposals into the K lowest-retention slots,
//                  ids by a prefix over the mask from next_global_id (:852-934)
//   fuse           rows keyed by (tile, slot) (masked rows dropped), stable radix sort, one lane per key
//                  run sums its rows in input order (the reference's .at[].add order) and adds the sums
//                  to the slot (:1037-1123); every listed tile's rgb is rebuilt and the rows' slots get
//                  the timestamp (:1097-1112)
//   k_pm_cull / k_pm_recency / k_pm_forget  one workgroup per tile (fixed-order sums) / elementwise
//   merge          per-slot mean / covariance / det, all triu pairs' Bhattacharyya distance
//                  (:1907-1930), max_pairs rounds of a (distance, pair index) argmin over eligible pairs
//                  -- the greedy walk of the stable argsort (:1554-1585) -- then the moment-matched
//                  merges of the selected (disjoint) pairs (:1603-1707)
// No floating-point atomics; every sum has a fixed order.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gcs_math.h"
#include "gcslam_hip.h"
#include "gcs_live.h"

namespace gcs {
namespace {

constexpr int kPmThreads = 256;
constexpr int kNL = 3;  // vMF lobes per primitive (GC_VMF_N_LOBES, constants.py:463); the context requires it
constexpr int kPmRed = 1024;  // one-workgroup-per-tile reductions
constexpr uint32_t kNoKey = 0xffffffffu;

struct PmStore {
  double *lam, *th, *eta, *w, *ts, *cts, *col, *cam, *lid, *acc, *den, *rgb;
  int64_t *lsup, *lupd, *ids;
  uint8_t* valid;
  int M, nl;  // slots per tile, vMF lobes
};

__device__ __forceinline__ size_t sidx(const PmStore& s, int t, int q) { return (size_t)t * s.M + q; }

// ascending order of a double as unsigned bits; -0.0 folds onto 0.0 (lax.sort's float comparator)
__device__ __forceinline__ uint64_t ord_key(double x) {
  if (x == 0.0) x = 0.0;
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

// LU with partial pivoting on A + eps I (jnp.linalg.solve / inv / det are LU), n_rhs right-hand sides
__device__ void lu3(const double* A, double eps, double (&a)[3][3], int (&perm)[3], double& det) {
#pragma clang fp contract(off)
  for (int r = 0; r < 3; ++r) {
    perm[r] = r;
    for (int c = 0; c < 3; ++c) a[r][c] = A[3 * r + c] + (r == c ? eps : 0.0);
  }
  double sgn = 1.0;
  for (int c = 0; c < 3; ++c) {
    int pr = c;
    for (int r = c + 1; r < 3; ++r)
      if (fabs(a[r][c]) > fabs(a[pr][c])) pr = r;
    if (pr != c) {
      for (int q = 0; q < 3; ++q) {
        const double t = a[c][q];
        a[c][q] = a[pr][q];
        a[pr][q] = t;
      }
      const int t = perm[c];
      perm[c] = perm[pr];
      perm[pr] = t;
      sgn = -sgn;
    }
    for (int r = c + 1; r < 3; ++r) {
      a[r][c] = a[r][c] / a[c][c];
      for (int q = c + 1; q < 3; ++q) a[r][q] = a[r][q] - a[r][c] * a[c][q];
    }
  }
  det = sgn * (a[0][0] * a[1][1] * a[2][2]);
}

__device__ void lu3_solve(const double (&a)[3][3], const int (&perm)[3], const double* b, double* x) {
#pragma clang fp contract(off)
  double y[3];
  for (int r = 0; r < 3; ++r) {
    double v = b[perm[r]];
    for (int q = 0; q < r; ++q) v = v - a[r][q] * y[q];
    y[r] = v;
  }
  for (int r = 2; r >= 0; --r) {
    double v = y[r];
    for (int q = r + 1; q < 3; ++q) v = v - a[r][q] * x[q];
    x[r] = v / a[r][r];
  }
}

__device__ void lu3_inv(const double (&a)[3][3], const int (&perm)[3], double* inv) {
  for (int c = 0; c < 3; ++c) {
    const double e[3] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0};
    double x[3];
    lu3_solve(a, perm, e, x);
    for (int r = 0; r < 3; ++r) inv[3 * r + c] = x[r];
  }
}

__device__ __forceinline__ double clip01(double x) { return fmin(fmax(x, 0.0), 1.0); }

// fixed-order block sum (thread-strided partials, xor tree, waves in order); result in all threads
template <int NT>
__device__ double block_sum_d(double v, double* lds) {
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double s = lds[0];
  for (int w = 1; w < NT / 64; ++w) s += lds[w];
  return s;
}

__global__ __launch_bounds__(kPmThreads) void k_pm_clear(PmStore st, int t) {
  const int q = blockIdx.x * kPmThreads + threadIdx.x;
  if (q >= st.M) return;
  const size_t i = sidx(st, t, q);
  for (int k = 0; k < 9; ++k) st.lam[9 * i + k] = 0.0;
  for (int k = 0; k < 3; ++k) {
    st.th[3 * i + k] = 0.0;
    st.col[3 * i + k] = 0.0;
    st.acc[3 * i + k] = 0.0;
    st.rgb[3 * i + k] = 0.5;
  }
  for (int k = 0; k < 3 * kNL; ++k) st.eta[(size_t)3 * kNL * i + k] = 0.0;
  st.w[i] = st.ts[i] = st.cts[i] = st.cam[i] = st.lid[i] = st.den[i] = 0.0;
  st.lsup[i] = st.lupd[i] = st.ids[i] = 0;
  st.valid[i] = 0;
}

// mode 0: -score (score = w, -1e30 where invalid), mode 1: retention w exp(-lam dt) (-inf where invalid)
// other_bm (may be null): bit g set where the key is not the mode's empty-slot key (k_pm_topk_sparse),
// one 32-bit word per half wave (g is wave-aligned: 64 consecutive g per wave)
// below (with other_bm, mode 1): per tile, the keys under the empty-slot key (a NaN retention with the
// sign bit: none in practice) -- k_pm_topk_sparse's dense-tile shortcut needs there to be none
__global__ __launch_bounds__(kPmThreads) void k_pm_keys(PmStore st, const int32_t* tiles, int n, int mode,
                                                        long long seq, double lam, uint64_t* keys, uint32_t* vals,
                                                        uint32_t* other_bm, uint32_t* below) {
  const long g = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= (long)n * st.M) return;
  const int t = (int)(g / st.M), q = (int)(g % st.M);
  const int ti = tiles[t];
  bool v = false;
  double w = 0.0;
  long long last = 0;
  if (ti >= 0) {
    const size_t i = sidx(st, ti, q);
    v = st.valid[i] != 0;
    w = st.w[i];
    last = st.lsup[i];
  }
  double key;
  if (mode == 0) {
    key = -(v ? w : -1e30);
  } else {
    const long long dt = max(0ll, seq - last);
    const double decay = exp(-lam * (double)dt);
    key = v ? w * decay : -INFINITY;
  }
  const uint64_t kb = ord_key(key);
  keys[g] = kb;
  vals[g] = (uint32_t)g;  // tile position x M + slot
  if (other_bm) {
    const uint64_t E = ord_key(mode == 0 ? 1e30 : -INFINITY);
    const uint64_t b = __ballot(kb != E);
    if ((threadIdx.x & 31) == 0) other_bm[g >> 5] = (uint32_t)(b >> (threadIdx.x & 32));
    if (mode == 1 && kb < E) atomicAdd(&below[t], 1u);
  }
}

// the first k (<= kSelMax) entries of each tile's stable key order without sorting the tile: one
// workgroup per tile finds the k-th smallest key T by an MSB radix select (6 passes of 11 bits over
// the tile's keys), collects the keys below T and the first ties at T in slot order (exactly the
// entries a stable sort puts first), and orders those k by (key, slot) with a bitonic sort in LDS.
// Writes sorted[t M + r] = t M + slot for r < k (what k_pm_view / k_pm_insert read).
constexpr int kSelMax = 1024;
constexpr int kSelBits = 11;  // digit width of the select passes (6 passes over 64-bit keys)
__global__ __launch_bounds__(kPmRed) void k_pm_select(const uint64_t* __restrict__ keys, int M, int k,
                                                       uint32_t* __restrict__ sorted) {
  __shared__ uint32_t s_hist[1 << kSelBits];
  __shared__ uint64_t s_key[kSelMax];
  __shared__ uint32_t s_slot[kSelMax];
  __shared__ uint32_t s_wl[kPmRed / 64], s_we[kPmRed / 64];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint64_t* kt = keys + (size_t)t * M;
  uint64_t prefix = 0, pmask = 0;
  uint32_t need = (uint32_t)k;  // rank (1-based) of T among the keys that match the prefix
  for (int hi = 64; hi > 0; hi -= kSelBits) {
    const int bits = hi < kSelBits ? hi : kSelBits, shift = hi - bits;
    const uint32_t dmask = (1u << bits) - 1u;
    for (int i = tid; i < (1 << kSelBits); i += kPmRed) s_hist[i] = 0u;
    __syncthreads();
    for (int q0 = 0; q0 < M; q0 += kPmRed) {  // block-uniform trip count (the wave votes below)
      const int q = q0 + tid;
      const uint64_t x = q < M ? kt[q] : 0ull;
      const bool act = q < M && (x & pmask) == prefix;
      const uint32_t dg = (uint32_t)(x >> shift) & dmask;
      // wave-aggregated when every counted lane has the same digit (an empty or freshly activated tile
      // holds one key value everywhere: per-lane atomics on one LDS word serialise the whole tile)
      const uint64_t am = __ballot(act);
      if (am) {
        const int l0 = __ffsll((long long)am) - 1;
        const uint32_t d0 = (uint32_t)__shfl((int)dg, l0, 64);
        if (__ballot(act && dg != d0) == 0ull) {
          if (lane == l0) atomicAdd(&s_hist[d0], (uint32_t)__popcll(am));
        } else if (act) {
          atomicAdd(&s_hist[dg], 1u);
        }
      }
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: the digit whose cumulative count reaches need (kSelPer bins per lane)
      constexpr int kSelPer = (1 << kSelBits) / 64;
      uint32_t sum = 0;
      for (int j = 0; j < kSelPer; ++j) sum += s_hist[kSelPer * tid + j];
      uint32_t inc = sum;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
      }
      const uint32_t exc = inc - sum;
      if (exc < need && inc >= need) {
        uint32_t c = exc;
        int d = kSelPer * tid;
        for (int j = 0; j < kSelPer; ++j) {
          const uint32_t h = s_hist[kSelPer * tid + j];
          if (c + h >= need) {
            d = kSelPer * tid + j;
            break;
          }
          c += h;
        }
        s_need = need - c;
        s_prefix = prefix | ((uint64_t)d << shift);
      }
    }
    __syncthreads();
    need = s_need;
    prefix = s_prefix;
    pmask |= (uint64_t)dmask << shift;
    __syncthreads();
  }
  // keys < T: exactly k - need of them; keys == T: the first `need` in slot order
  const uint32_t nless = (uint32_t)k - need;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t base_l = 0, base_e = 0;
  for (int c0 = 0; c0 < M; c0 += kPmRed) {
    const int q = c0 + tid;
    const uint64_t x = q < M ? kt[q] : ~0ull;
    const bool lt = q < M && x < prefix, eq = q < M && x == prefix;
    const uint64_t bl = __ballot(lt), be = __ballot(eq);
    if (lane == 0) {
      s_wl[wid] = (uint32_t)__popcll(bl);
      s_we[wid] = (uint32_t)__popcll(be);
    }
    __syncthreads();
    uint32_t ol = 0, oe = 0, tl = 0, te = 0;
    for (int w = 0; w < kPmRed / 64; ++w) {
      if (w < wid) {
        ol += s_wl[w];
        oe += s_we[w];
      }
      tl += s_wl[w];
      te += s_we[w];
    }
    if (lt) {
      const uint32_t pos = base_l + ol + (uint32_t)__popcll(bl & below);
      s_key[pos] = x;
      s_slot[pos] = (uint32_t)q;
    }
    if (eq) {
      const uint32_t r = base_e + oe + (uint32_t)__popcll(be & below);
      if (r < need) {
        s_key[nless + r] = x;
        s_slot[nless + r] = (uint32_t)q;
      }
    }
    base_l += tl;
    base_e += te;
    __syncthreads();
  }
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = k + tid; i < P; i += kPmRed) {
    s_key[i] = ~0ull;
    s_slot[i] = ~0u;
  }
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      const int i = tid, j = tid ^ stride;
      if (i < P && j > i) {
        const uint64_t ki = s_key[i], kj = s_key[j];
        const uint32_t si = s_slot[i], sj = s_slot[j];
        const bool gt = ki > kj || (ki == kj && si > sj);
        if (gt == ((i & size) == 0)) {
          s_key[i] = kj;
          s_key[j] = ki;
          s_slot[i] = sj;
          s_slot[j] = si;
        }
      }
    }
  __syncthreads();
  for (int r = tid; r < k; r += kPmRed) sorted[(size_t)t * M + r] = (uint32_t)((size_t)t * M) + s_slot[r];
}

// The same select with the high 32 bits of the tile's keys held in registers (KPT per thread, slots
// tid + j * kPmRed): one global pass loads them, the digit passes over the high word and the
// collection run on registers and LDS; the low word is read from memory only for keys whose high word
// equals the k-th key's (ties of the high word: typically a handful).  Histogram adds are
// wave-aggregated when every counted lane of the wave has the same digit (an empty or freshly
// activated tile has one key value everywhere: per-lane atomics on one LDS word serialise the tile),
// else one LDS atomic per key.
template <int KPT, int NT>
__global__ __launch_bounds__(NT) void k_pm_select_reg(const uint64_t* __restrict__ keys, int M, int k,
                                                           uint32_t* __restrict__ sorted) {
  __shared__ uint32_t s_hist[1 << kSelBits];
  __shared__ uint64_t s_key[kSelMax];
  __shared__ uint32_t s_slot[kSelMax];
  __shared__ uint32_t s_wl[NT / 64], s_we[NT / 64];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint64_t* kt = keys + (size_t)t * M;
  // the key words through a buffer descriptor: slot q = tid + j NT is voffset 8 tid (+4: high word) and
  // the constant soffset 8 j NT, so the unrolled j loops share one address register (flat loads kept a
  // 64-bit address per j live across the passes and spilled at 49 keys per thread)
  const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void*)kt, 0, M * 8, 0x00020000);
  auto lo_word = [&](int j) { return __builtin_amdgcn_raw_buffer_load_b32(kr, tid * 8, j * NT * 8, 0); };
  auto hi_word = [&](int j) { return __builtin_amdgcn_raw_buffer_load_b32(kr, tid * 8 + 4, j * NT * 8, 0); };
  uint32_t xh[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int q = tid + j * NT;
    xh[j] = q < M ? hi_word(j) : 0u;
  }
  uint64_t prefix = 0, pmask = 0;
  uint32_t need = (uint32_t)k;  // rank (1-based) of T among the keys that match the prefix
  // digits aligned to the words: 11, 11, 10 bits of the high word, then 11, 11, 10 of the low word
  constexpr int kShift[6] = {53, 42, 32, 21, 10, 0}, kBits[6] = {11, 11, 10, 11, 11, 10};
  for (int pass = 0; pass < 6; ++pass) {
    const int bits = kBits[pass], shift = kShift[pass];
    const uint32_t dmask = (1u << bits) - 1u;
    const bool hiword = shift >= 32;  // this pass reads only high-word bits (prefix bits are high too)
    for (int i = tid; i < (1 << kSelBits); i += NT) s_hist[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int q = tid + j * NT;
      bool act = q < M;
      uint32_t dg = 0;
      if (hiword) {
        act = act && (xh[j] & (uint32_t)(pmask >> 32)) == (uint32_t)(prefix >> 32);
        dg = (xh[j] >> (shift - 32)) & dmask;
      } else {
        act = act && xh[j] == (uint32_t)(prefix >> 32);  // high word fixed by now: its ties only
        if (act) {
          const uint64_t x = ((uint64_t)xh[j] << 32) | lo_word(j);
          act = (x & pmask) == prefix;
          dg = (uint32_t)(x >> shift) & dmask;
        }
      }
      const uint64_t am = __ballot(act);
      if (am) {  // wave-uniform
        const int l0 = __ffsll((long long)am) - 1;
        const uint32_t d0 = (uint32_t)__shfl((int)dg, l0, 64);
        if (__ballot(act && dg != d0) == 0ull) {
          if (lane == l0) atomicAdd(&s_hist[d0], (uint32_t)__popcll(am));
        } else if (act) {
          atomicAdd(&s_hist[dg], 1u);
        }
      }
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: the digit whose cumulative count reaches need (kSelPer bins per lane)
      constexpr int kSelPer = (1 << kSelBits) / 64;
      uint32_t sum = 0;
      for (int j = 0; j < kSelPer; ++j) sum += s_hist[kSelPer * tid + j];
      uint32_t inc = sum;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
      }
      const uint32_t exc = inc - sum;
      if (exc < need && inc >= need) {
        uint32_t c = exc;
        int d = kSelPer * tid;
        for (int j = 0; j < kSelPer; ++j) {
          const uint32_t h = s_hist[kSelPer * tid + j];
          if (c + h >= need) {
            d = kSelPer * tid + j;
            break;
          }
          c += h;
        }
        s_need = need - c;
        s_prefix = prefix | ((uint64_t)d << shift);
      }
    }
    __syncthreads();
    need = s_need;
    prefix = s_prefix;
    pmask |= (uint64_t)dmask << shift;
    __syncthreads();
  }
  // keys < T: exactly k - need of them; keys == T: the first `need` in slot order (slots ascend with j
  // within a thread and with the thread within a chunk of NT slots)
  const uint32_t nless = (uint32_t)k - need;
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t th = (uint32_t)(prefix >> 32);
  uint32_t base_l = 0, base_e = 0;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int q = tid + j * NT;
    bool lt = q < M && xh[j] < th, eq = false;
    uint64_t x = (uint64_t)xh[j] << 32;
    if (q < M && xh[j] == th) {  // high-word tie: the full key decides
      x |= lo_word(j);
      lt = x < prefix;
      eq = x == prefix;
    } else if (lt) {
      x |= lo_word(j);
    }
    const uint64_t bl = __ballot(lt), be = __ballot(eq);
    if (lane == 0) {
      s_wl[wid] = (uint32_t)__popcll(bl);
      s_we[wid] = (uint32_t)__popcll(be);
    }
    __syncthreads();
    uint32_t ol = 0, oe = 0, tl = 0, te = 0;
    for (int w = 0; w < NT / 64; ++w) {
      if (w < wid) {
        ol += s_wl[w];
        oe += s_we[w];
      }
      tl += s_wl[w];
      te += s_we[w];
    }
    if (lt) {
      const uint32_t pos = base_l + ol + (uint32_t)__popcll(bl & below);
      s_key[pos] = x;
      s_slot[pos] = (uint32_t)q;
    }
    if (eq) {
      const uint32_t r = base_e + oe + (uint32_t)__popcll(be & below);
      if (r < need) {
        s_key[nless + r] = x;
        s_slot[nless + r] = (uint32_t)q;
      }
    }
    base_l += tl;
    base_e += te;
    __syncthreads();
  }
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = k + tid; i < P; i += NT) {
    s_key[i] = ~0ull;
    s_slot[i] = ~0u;
  }
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = tid; i < P; i += NT) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t ki = s_key[i], kj = s_key[j];
          const uint32_t si = s_slot[i], sj = s_slot[j];
          const bool gt = ki > kj || (ki == kj && si > sj);
          if (gt == ((i & size) == 0)) {
            s_key[i] = kj;
            s_key[j] = ki;
            s_slot[i] = sj;
            s_slot[j] = si;
          }
        }
      }
    }
  __syncthreads();
  for (int r = tid; r < k; r += NT) sorted[(size_t)t * M + r] = (uint32_t)((size_t)t * M) + s_slot[r];
}

// The first k (<= kSelMax) entries of each tile's stable key order by a tree of sorted runs, in one
// launch and with many CUs of a many-tile call busy (k_pm_select runs one workgroup per tile: 7 on 256
// CUs at the reference's 7 x 50,000).  Leaf g of tile t (grid.x) sorts the keys of slots
// [4096 g, 4096 g + 4096) by (key, slot) in LDS -- the stable order: slots are unique, so every pair
// is distinct -- and keeps the first k as its run.  Two sibling runs are merged by whichever of their
// two workgroups finishes second (a per-node ticket: the first leaves, so no workgroup waits on
// another), keeping the first k, and that workgroup climbs; the root writes
// sorted[t M + r] = t M + slot for r < k.  Merge: an element's rank in the merged run is its own
// index plus the count of the other run's smaller entries (binary search in LDS).  Runs live in
// run_key / run_slot at the first leaf of their node (k entries per leaf); the writer's stores are
// released (agent-scope fence, barrier) before its ticket, the second arrival acquires before reading.
// GCS_TOPK_SC1 (default): the write-through run hand-off of cdna_hip_programming.md Guideline 16.
// Hardware assumption (gfx950, not promised by the HIP / HSA memory model): agent-scope relaxed atomic
// stores of the run go to the shared L2 (sc1) and complete before the storing wave passes
// s_waitcnt vmcnt(0), so a relaxed ticket add after the workgroup barrier orders them for the second
// arrival, whose one agent-scope acquire drops its CU's stale lines before it reads the run.  Checked
// under repetition by tests/test_gpu_primitive_map.py::test_topk_tree_handoff_stress (24 views of seven
// dense 50,000-slot tiles against the oracle's stable top-k); GCS_TOPK_SC1=0 builds the acq_rel ticket.
#ifndef GCS_TOPK_SC1
#define GCS_TOPK_SC1 1
#endif
constexpr int kTopEpt = 4;                  // slots per thread in a leaf
constexpr int kTopChunk = kTopEpt * kPmRed;  // slots per leaf: 4,096 (13 leaves, 4 merge levels at 50,000)
constexpr int kTopMaxLevels = 8;             // up to 128 leaves per tile (M <= 524,288)
constexpr int kTopNodes = 64;                // tickets per level and tile
__device__ __forceinline__ bool topk_less(uint64_t ka, uint32_t sa, uint64_t kb, uint32_t sb) {
  return ka < kb || (ka == kb && sa < sb);
}
// entries of the node (lv, i)'s run: min(k, the node's slots)
__device__ __forceinline__ int topk_len(int M, int k, int lv, int i) {
  const long lo = (long)(i << lv) * kTopChunk, hi = min((long)M, (long)((i + 1) << lv) * kTopChunk);
  return (int)min((long)k, max(0L, hi - lo));
}
__global__ __launch_bounds__(kPmRed) void k_pm_topk(const uint64_t* __restrict__ keys, int M, int k, int G,
                                                     uint64_t* run_key, uint32_t* run_slot, uint32_t* tickets,
                                                     uint32_t* __restrict__ sorted, const uint32_t* __restrict__ skip) {
  if (skip && skip[blockIdx.y]) return;  // k_pm_topk_sparse wrote this tile's result
  // leaf: the chunk's keys / slots; merges: own run [0, k), sibling run [kSelMax, 2 kSelMax), merged
  // run [2 kSelMax, 3 kSelMax) (k <= kSelMax = 1,024)
  __shared__ uint64_t s_k[kTopChunk];
  __shared__ uint32_t s_s[kTopChunk];
  static_assert(3 * kSelMax <= kTopChunk, "merge buffers inside the leaf buffer");
  uint64_t* const s_ok = s_k + 2 * kSelMax;
  uint32_t* const s_os = s_s + 2 * kSelMax;
  __shared__ uint32_t s_go;
  const int t = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  uint64_t* rk = run_key + (size_t)t * G * k;
  uint32_t* rs = run_slot + (size_t)t * G * k;
  uint32_t* tk = tickets + (size_t)t * kTopMaxLevels * kTopNodes;
  {  // leaf: bitonic sort of the chunk (padding last: key ~0, slot ~0 above every real pair).  Each
     // thread holds 4 consecutive entries in registers: strides 1-2 are exchanges inside the thread,
     // strides 4-128 between lanes of one wave (shuffles, no barrier), and only strides 256-2048 go
     // through LDS (10 of the 78 stages; the all-LDS network took a barrier per stage).  (key, slot)
     // pairs are distinct, so any sorting network gives the same order.
    uint64_t rk4[kTopEpt];
    uint32_t rs4[kTopEpt];
#pragma unroll
    for (int e = 0; e < kTopEpt; ++e) {
      const int x = kTopEpt * tid + e, q = g * kTopChunk + x;
      rk4[e] = q < M ? keys[(size_t)t * M + q] : ~0ull;
      rs4[e] = q < M ? (uint32_t)q : ~0u;
    }
    const int lane = tid & 63;
    for (int size = 2; size <= kTopChunk; size <<= 1) {
      int stride = size >> 1;
      if (stride >= 4 * 64) {  // the LDS stages of this size, then back to registers
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kTopEpt; ++e) {
          s_k[kTopEpt * tid + e] = rk4[e];
          s_s[kTopEpt * tid + e] = rs4[e];
        }
        for (; stride >= 4 * 64; stride >>= 1) {
          __syncthreads();
#pragma unroll
          for (int e = 0; e < kTopEpt / 2; ++e) {  // the chunk's kTopChunk / 2 pairs, two per thread
            const int pr = tid + e * kPmRed;
            const int x = ((pr & ~(stride - 1)) << 1) | (pr & (stride - 1)), y = x | stride;
            const uint64_t kx = s_k[x], ky = s_k[y];
            const uint32_t sx = s_s[x], sy = s_s[y];
            if (topk_less(ky, sy, kx, sx) == ((x & size) == 0)) {
              s_k[x] = ky;
              s_k[y] = kx;
              s_s[x] = sy;
              s_s[y] = sx;
            }
          }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kTopEpt; ++e) {
          rk4[e] = s_k[kTopEpt * tid + e];
          rs4[e] = s_s[kTopEpt * tid + e];
        }
      }
      for (; stride >= kTopEpt; stride >>= 1) {  // partner lane = lane ^ (stride / 4), same e
        const int lx = stride / kTopEpt;
        const bool lower = (lane & lx) == 0;
#pragma unroll
        for (int e = 0; e < kTopEpt; ++e) {
          const int x = kTopEpt * tid + e;
          const uint64_t ok = (uint64_t)__shfl_xor((unsigned long long)rk4[e], lx, 64);
          const uint32_t os = (uint32_t)__shfl_xor((int)rs4[e], lx, 64);
          const bool asc = (x & size) == 0;
          const bool other_less = topk_less(ok, os, rk4[e], rs4[e]);
          // the lower index keeps the smaller entry when ascending, the larger otherwise
          if (other_less == (lower == asc)) {
            rk4[e] = ok;
            rs4[e] = os;
          }
        }
      }
      for (; stride > 0; stride >>= 1) {  // inside the thread: entries e and e ^ stride
#pragma unroll
        for (int e = 0; e < kTopEpt; ++e) {
          const int f = e ^ stride;
          if (f > e) {
            const int x = kTopEpt * tid + e;
            const bool asc = (x & size) == 0;
            if (topk_less(rk4[f], rs4[f], rk4[e], rs4[e]) == asc) {
              const uint64_t tk = rk4[e];
              const uint32_t ts = rs4[e];
              rk4[e] = rk4[f];
              rs4[e] = rs4[f];
              rk4[f] = tk;
              rs4[f] = ts;
            }
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kTopEpt; ++e) {
      s_k[kTopEpt * tid + e] = rk4[e];
      s_s[kTopEpt * tid + e] = rs4[e];
    }
    __syncthreads();
  }
  int lv = 0, i = g;
  int L = topk_len(M, k, 0, g);
  for (;;) {
    if ((1 << lv) >= G) {  // the root: every leaf of the tile is in this run
      for (int r = tid; r < L; r += kPmRed) sorted[(size_t)t * M + r] = (uint32_t)((size_t)t * M) + s_s[r];
      return;
    }
    const int sib = i ^ 1;
    if ((sib << lv) >= G) {  // no sibling at this level: the run moves up unchanged
      i >>= 1;
      ++lv;
      continue;
    }
    // publish this run, then take the node's ticket
    const size_t mine = (size_t)(i << lv) * k;
    uint32_t* ticket = tk + lv * kTopNodes + (i >> 1);
#if GCS_TOPK_SC1
    // The hand-off of cdna_hip_programming.md Guideline 16 (counter form): the run is stored
    // write-through (agent-scope relaxed atomic stores: sc1), every wave drains its stores before the
    // barrier, ONE lane adds to the ticket relaxed -- no release fence, whose L2 write-back the
    // acq_rel ticket paid once per workgroup and level -- and the second arrival's lane takes ONE
    // agent-scope acquire (the CU's stale lines dropped) before the workgroup's plain loads.
    for (int r = tid; r < L; r += kPmRed) {
      __hip_atomic_store(rk + mine + r, s_k[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rs + mine + r, s_s[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old != 0u) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_go = old;
    }
    __syncthreads();
#else
    for (int r = tid; r < L; r += kPmRed) {
      rk[mine + r] = s_k[r];
      rs[mine + r] = s_s[r];
    }
    // every wave's stores drained at the barrier, then ONE agent-scope release with the ticket (a
    // fence per thread wrote the L2 back once per wave: 0.75 ms per call), and the second arrival's
    // acquire on the same atomic before the workgroup reads the sibling's run
    __syncthreads();
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old != 0u) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      s_go = old;
    }
    __syncthreads();
#endif
    if (s_go == 0u) return;  // the sibling merges
    const int Ls = topk_len(M, k, lv, sib);
    const size_t other = (size_t)(sib << lv) * k;
    for (int r = tid; r < Ls; r += kPmRed) {
      s_k[kSelMax + r] = rk[other + r];
      s_s[kSelMax + r] = rs[other + r];
    }
    __syncthreads();
    const int Lo = topk_len(M, k, lv + 1, i >> 1);
    // ranks: own entry r -> r + #{sibling entries below it}; sibling entry r -> r + #{own entries below}
    for (int side = 0; side < 2; ++side) {
      const int La = side == 0 ? L : Ls, Lb = side == 0 ? Ls : L;
      const uint64_t* ak = s_k + (side == 0 ? 0 : kSelMax);
      const uint32_t* as = s_s + (side == 0 ? 0 : kSelMax);
      const uint64_t* bk = s_k + (side == 0 ? kSelMax : 0);
      const uint32_t* bs = s_s + (side == 0 ? kSelMax : 0);
      if (tid < La) {
        const uint64_t x = ak[tid];
        const uint32_t xs = as[tid];
        int lo = 0, hi = Lb;  // first b not below x
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (topk_less(bk[mid], bs[mid], x, xs)) lo = mid + 1; else hi = mid;
        }
        const int rank = tid + lo;
        if (rank < Lo) {
          s_ok[rank] = x;
          s_os[rank] = xs;
        }
      }
    }
    __syncthreads();
    for (int r = tid; r < Lo; r += kPmRed) {
      s_k[r] = s_ok[r];
      s_s[r] = s_os[r];
    }
    __syncthreads();
    L = Lo;
    i >>= 1;
    ++lv;
  }
}

// Sparse tiles first (GCSLAM_PM_TOPK_SPARSE=0: the tree for every tile).  A tile's slots split into
// the empty-slot group -- every slot whose key is the mode's empty-slot key E (mode 0: the key of
// score -1e30, mode 1: of retention -inf), whose stable order is slot order -- and the rest.  With at
// most kSpMax of the rest (a map tile of 50,000 slots holds a few hundred primitives), the stable
// order is [rest below E by (key, slot)] ++ [the E slots ascending] ++ [rest above E by (key, slot)]:
// its first k come from one LDS sort of the rest and the first clear bits of the tile's bitmap of
// non-E slots, which k_pm_keys writes (one ballot per half wave): the kernel reads 6 KB of bitmap
// and gathers the few keys it marks, never the 50,000.  One workgroup per tile; a tile with more
// than kSpMax writes skip[t] = 0 and the tree takes it (the tree's other tiles' workgroups return at
// once).  Same result as the tree: (key, slot) pairs are distinct.
constexpr int kSpMax = 2048;    // entries besides the empty slots
constexpr int kSpWords = 2048;  // slot bitmap words per tile: M <= 65,536
// Dense tiles (more than kSpMax others) in mode 1 (the eviction order) with at least k empty slots and
// no key below the empty-slot key E: the first k of the stable order are the first k empty slots in slot
// order (every other key is above E) -- read from the bitmap alone.  The tree took these tiles
// (50,000 keys each, ~54 us at 7 tiles of the reference size) for an answer the bitmap holds.
__global__ __launch_bounds__(kPmRed) void k_pm_topk_sparse(const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ other_bm, int M, int k,
                                                          int mode, uint32_t* __restrict__ skip,
                                                          uint32_t* __restrict__ sorted, uint32_t* __restrict__ below) {
  __shared__ uint64_t s_k[kSpMax];
  __shared__ uint32_t s_s[kSpMax];
  __shared__ uint32_t s_wo[kPmRed / 64], s_wz[kPmRed / 64];
  __shared__ uint32_t s_clo, s_below;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    s_clo = 0u;
    s_below = below[t];
    below[t] = 0u;  // re-armed for the next k_pm_keys
  }
  // the tile's words of k_pm_keys' bitmap (bit q of the tile = global bit t M + q, not word-aligned):
  // WPT consecutive tile words per thread, their set (other) and clear (empty) bits counted
  constexpr int WPT = kSpWords / kPmRed;
  const int nw = (M + 31) >> 5;
  const long b0 = (long)t * M;
  uint32_t ow[WPT];
  uint32_t no = 0u, nz = 0u;
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int w = WPT * tid + u;
    uint32_t x = 0u, valid = 0u;
    if (w < nw) {
      const long gb = b0 + 32L * w;
      const int sh = (int)(gb & 31);
      const uint32_t lo = other_bm[gb >> 5], hi = sh ? other_bm[(gb >> 5) + 1] : 0u;
      x = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
      const int nb = min(32, M - 32 * w);
      valid = nb == 32 ? ~0u : ((1u << nb) - 1u);
      x &= valid;
    }
    ow[u] = x;
    no += (uint32_t)__popc(x);
    nz += (uint32_t)__popc(~x & valid);
  }
  // exclusive block scans of both counts (slot order: the other entries land in slot order)
  uint32_t xo = no, xz = nz;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t yo = (uint32_t)__shfl_up((int)xo, off, 64), yz = (uint32_t)__shfl_up((int)xz, off, 64);
    if (lane >= off) {
      xo += yo;
      xz += yz;
    }
  }
  if (lane == 63) {
    s_wo[wid] = xo;
    s_wz[wid] = xz;
  }
  __syncthreads();
  uint32_t ro = xo - no, rz = xz - nz, n = 0u, nzt = 0u;
  for (int w = 0; w < kPmRed / 64; ++w) {
    if (w < wid) {
      ro += s_wo[w];
      rz += s_wz[w];
    }
    n += s_wo[w];
    nzt += s_wz[w];
  }
  const int kk0 = min(k, M);
  if (n > (uint32_t)kSpMax) {
    if (!(mode == 1 && s_below == 0u && nzt >= (uint32_t)kk0)) {  // the tree's
      if (tid == 0) skip[t] = 0u;
      return;
    }
    if (tid == 0) skip[t] = 1u;
    uint32_t* out = sorted + (size_t)t * M;
    const uint32_t tb = (uint32_t)((size_t)t * M);
    uint32_t rank = rz;
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int w = WPT * tid + u;
      uint32_t zb = 0u;
      if (w < nw) {
        const int nb = min(32, M - 32 * w);
        zb = ~ow[u] & (nb == 32 ? ~0u : ((1u << nb) - 1u));
      }
      while (zb != 0u && rank < (uint32_t)kk0) {
        const int bit = __ffs((int)zb) - 1;
        zb &= zb - 1u;
        out[rank] = tb + (uint32_t)(32 * w + bit);
        ++rank;
      }
      rank += (uint32_t)__popc(zb);
    }
    return;
  }
  if (tid == 0) skip[t] = 1u;
  // gather the other entries' keys into LDS in slot order: a word's marked keys are loaded together
  // (predicated), then stored (one round trip per word; the map's primitives fill the first slots of
  // a tile, so a few threads hold full words, and a load-store chain per bit cost them 32 each)
  const uint64_t* kt = keys + (size_t)t * M;
  {
    uint32_t r = ro;
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const uint32_t x = ow[u];
      if (x == 0u) continue;
      const int qb = 32 * (WPT * tid + u);
      uint64_t kv[32];
#pragma unroll
      for (int b = 0; b < 32; ++b) kv[b] = (x >> b) & 1u ? kt[qb + b] : 0ull;
#pragma unroll
      for (int b = 0; b < 32; ++b)
        if ((x >> b) & 1u) {
          s_k[r] = kv[b];
          s_s[r] = (uint32_t)(qb + b);
          ++r;
        }
    }
  }
  // bitonic sort of the n entries by (key, slot) in LDS (padding above every real pair)
  int P = 1;
  while (P < (int)n) P <<= 1;
  for (int i = (int)n + tid; i < P; i += kPmRed) {
    s_k[i] = ~0ull;
    s_s[i] = ~0u;
  }
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int pr = tid; pr < P / 2; pr += kPmRed) {
        const int x = ((pr & ~(stride - 1)) << 1) | (pr & (stride - 1)), y = x | stride;
        const uint64_t kx = s_k[x], ky = s_k[y];
        const uint32_t sx = s_s[x], sy = s_s[y];
        if (topk_less(ky, sy, kx, sx) == ((x & size) == 0)) {
          s_k[x] = ky;
          s_k[y] = kx;
          s_s[x] = sy;
          s_s[y] = sx;
        }
      }
    }
  __syncthreads();
  // c_lo = the entries below the empty-slot key E (a prefix of the sorted run: one boundary writer)
  const uint64_t E = ord_key(mode == 0 ? 1e30 : -INFINITY);  // k_pm_keys' empty-slot keys
  for (int i = tid; i < (int)n; i += kPmRed)
    if (s_k[i] < E && (i + 1 == (int)n || s_k[i + 1] >= E)) s_clo = (uint32_t)(i + 1);
  __syncthreads();
  const int clo = (int)s_clo, ne = M - (int)n, kk = min(k, M);
  uint32_t* out = sorted + (size_t)t * M;
  const uint32_t tb = (uint32_t)((size_t)t * M);
  for (int r = tid; r < (int)n; r += kPmRed) {
    const int pos = r < clo ? r : r + ne;
    if (pos < kk) out[pos] = tb + s_s[r];
  }
  // the empty slots at positions clo.. : the first `need` clear bits, in slot order
  const int need = kk > clo ? min(kk - clo, ne) : 0;
  uint32_t rank = rz;
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int w = WPT * tid + u;
    uint32_t zb = 0u;
    if (w < nw) {
      const int nb = min(32, M - 32 * w);
      zb = ~ow[u] & (nb == 32 ? ~0u : ((1u << nb) - 1u));
    }
    while (zb != 0u && rank < (uint32_t)need) {
      const int bit = __ffs((int)zb) - 1;
      zb &= zb - 1u;
      out[clo + (int)rank] = tb + (uint32_t)(32 * w + bit);
      ++rank;
    }
    rank += (uint32_t)__popc(zb);
  }
}

// second (stable) pass of the per-tile sort: key = the entry's tile position
__global__ __launch_bounds__(kPmThreads) void k_pm_segkeys(const uint32_t* vals, long total, int M, uint32_t* seg) {
  const long g = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (g < total) seg[g] = vals[g] / (uint32_t)M;
}

struct PmViewOut {
  double *pos, *cov, *dir, *kap, *w, *eta, *col;
  int64_t *ids, *lsup, *tid;
  uint8_t* valid;
  int32_t* slots;
};

__global__ __launch_bounds__(kPmThreads) void k_pm_view(PmStore st, const int32_t* tiles, const int64_t* tile_ids,
                                                        int n, int k, const uint32_t* sorted, double eps_lift,
                                                        double eps_mass, PmViewOut o) {
#pragma clang fp contract(off)
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= n * k) return;
  const int t = g / k, r = g % k;
  const int ti = tiles[t];
  const int q = ti >= 0 ? (int)(sorted[(size_t)t * st.M + r] % (uint32_t)st.M) : r;  // missing tile: all keys equal
  double L[9], th[3], es[3] = {0.0, 0.0, 0.0}, rgb[3] = {0.5, 0.5, 0.5}, w = 0.0;
  long long id = 0, last = 0;
  uint8_t v = 0;
  for (int c = 0; c < 9; ++c) L[c] = 0.0;
  for (int c = 0; c < 3; ++c) th[c] = 0.0;
  constexpr int ne = 3 * kNL;
  if (ti >= 0) {
    const size_t i = sidx(st, ti, q);
    for (int c = 0; c < 9; ++c) L[c] = st.lam[9 * i + c];
    for (int c = 0; c < 3; ++c) {
      th[c] = st.th[3 * i + c];
      rgb[c] = st.rgb[3 * i + c];
    }
    for (int b = 0; b < kNL; ++b)
      for (int c = 0; c < 3; ++c) {
        const double e = st.eta[(size_t)ne * i + 3 * b + c];
        es[c] = b == 0 ? e : es[c] + e;
        if (o.eta) o.eta[(size_t)ne * g + 3 * b + c] = e;
      }
    w = st.w[i];
    id = st.ids[i];
    last = st.lsup[i];
    v = st.valid[i];
  } else if (o.eta) {
    for (int c = 0; c < ne; ++c) o.eta[(size_t)ne * g + c] = 0.0;
  }
  double a[3][3], det;
  int perm[3];
  lu3(L, eps_lift, a, perm, det);
  double mu[3];
  lu3_solve(a, perm, th, mu);
  if (o.pos)
    for (int c = 0; c < 3; ++c) o.pos[3 * g + c] = mu[c];
  if (o.cov) {
    double S[9];
    lu3_inv(a, perm, S);
    for (int c = 0; c < 9; ++c) o.cov[9 * g + c] = S[c];
  }
  const double kap = sqrt((es[0] * es[0] + es[1] * es[1]) + es[2] * es[2]);
  if (o.dir)
    for (int c = 0; c < 3; ++c) o.dir[3 * g + c] = es[c] / (kap + eps_mass);
  if (o.kap) o.kap[g] = kap;
  if (o.w) o.w[g] = w;
  if (o.col)
    for (int c = 0; c < 3; ++c) o.col[3 * g + c] = rgb[c];
  if (o.ids) o.ids[g] = id;
  if (o.lsup) o.lsup[g] = last;
  if (o.valid) o.valid[g] = v ? 1 : 0;  // 0/1 bytes: the caller may view them as bool
  if (o.slots) o.slots[g] = q;
  if (o.tid) o.tid[g] = tile_ids[t];
}

struct PmRows {
  const double *lam, *th, *eta, *w, *resp, *col;
  const uint8_t* valid;
  const int32_t *src, *tpos, *slots;
  int n;
};

// one workgroup: tile by tile, the masked proposals land in the K lowest-retention slots
__global__ __launch_bounds__(kPmThreads) void k_pm_insert(PmStore st, const int32_t* tiles, int n, int K,
                                                          const uint32_t* sorted, PmRows r, double ts, long long seq,
                                                          long long next_id, int64_t* ids_out, int32_t* n_ins) {
  // one workgroup per listed tile (grid n): ids continue tile by tile, so tile t's first id is
  // next_id + the valid proposals of tiles 0 .. t-1 (counted here; at most n K flags)
  __shared__ int s_w[kPmThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int ne = 3 * kNL;
  const int t = blockIdx.x;
  long long base = next_id;
  {
    int c = 0;
    for (int row = threadIdx.x; row < t * K; row += kPmThreads) c += r.valid[row] ? 1 : 0;
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
    if (lane == 0) s_w[wid] = c;
    __syncthreads();
    for (int w = 0; w < kPmThreads / 64; ++w) base += s_w[w];
    __syncthreads();
  }
  {
    const int ti = tiles[t];
    int run = 0;
    for (int q0 = 0; q0 < K; q0 += kPmThreads) {
      const int q = q0 + threadIdx.x;
      const int row = t * K + q;
      const int d = q < K && r.valid[row] ? 1 : 0;
      int x = d;
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      __syncthreads();
      if (lane == 63) s_w[wid] = x;
      __syncthreads();
      int pre = run + x - d;
      for (int w = 0; w < wid; ++w) pre += s_w[w];
      int tot = 0;
      for (int w = 0; w < kPmThreads / 64; ++w) tot += s_w[w];
      if (q < K) {
        const long long id = d ? base + pre : -1;
        if (ids_out) ids_out[row] = id;
        if (d) {
          const size_t i = sidx(st, ti, (int)(sorted[(size_t)t * st.M + q] % (uint32_t)st.M));
          for (int c = 0; c < 9; ++c) st.lam[9 * i + c] = r.lam[9 * (size_t)row + c];
          for (int c = 0; c < 3; ++c) st.th[3 * i + c] = r.th[3 * (size_t)row + c];
          for (int c = 0; c < ne; ++c) st.eta[(size_t)ne * i + c] = r.eta[(size_t)ne * row + c];
          const double wn = r.w[row];
          const int s = r.src ? r.src[row] : 1;
          const double cam = wn * (s == 0 ? 1.0 : 0.0), lid = wn * (s == 1 ? 1.0 : 0.0);
          double cn[3] = {0.0, 0.0, 0.0};
          if (r.col)
            for (int c = 0; c < 3; ++c) cn[c] = r.col[3 * (size_t)row + c];
          for (int c = 0; c < 3; ++c) {
            const double rg = cam > 0.0 ? clip01(cn[c]) : 0.5;
            st.acc[3 * i + c] = cn[c] * cam;
            st.col[3 * i + c] = rg;
            st.rgb[3 * i + c] = rg;
          }
          st.w[i] = wn;
          st.ids[i] = id;
          st.cam[i] = cam;
          st.lid[i] = lid;
          st.den[i] = cam;
          st.ts[i] = ts;
          st.cts[i] = ts;
          st.lsup[i] = seq;
          st.lupd[i] = seq;
          st.valid[i] = 1;
        }
      }
      run += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) n_ins[t] = run;
  }
}

// fuse: key = (tile position, slot) for the rows that contribute (valid, tile listed)
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_keys(PmRows r, int n_tiles, int M, uint32_t* keys,
                                                             uint32_t* vals, uint32_t* err) {
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= r.n) return;
  const int tp = r.tpos[g], q = r.slots[g];
  const bool ok = q >= 0 && q < M;
  if (!ok) err[0] = 1u;
  const bool v = (r.valid ? r.valid[g] != 0 : true) && tp >= 0 && tp < n_tiles && ok;
  keys[g] = v ? (uint32_t)tp * (uint32_t)M + (uint32_t)q : kNoKey;
  vals[g] = (uint32_t)g;
}

// one lane per key run (sorted stable: rows in input order): d = sum r x from 0, then slot += d
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_apply(PmStore st, const int32_t* tiles, PmRows r,
                                                              const uint32_t* keys, const uint32_t* vals,
                                                              long long seq) {
#pragma clang fp contract(off)
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= r.n) return;
  const uint32_t key = keys[g];
  if (key == kNoKey || (g > 0 && keys[g - 1] == key)) return;
  constexpr int ne = 3 * kNL;
  double dL[9], dth[3], de[3 * kNL], dw = 0.0, drs = 0.0, dcam = 0.0, dlid = 0.0, dacc[3] = {0.0, 0.0, 0.0}, dden = 0.0;
  for (int c = 0; c < 9; ++c) dL[c] = 0.0;
  for (int c = 0; c < 3; ++c) dth[c] = 0.0;
  for (int c = 0; c < ne; ++c) de[c] = 0.0;
  for (int p = g; p < r.n && keys[p] == key; ++p) {
    const size_t row = vals[p];
    const double rr = r.resp[row] * 1.0;  // resp * valid (valid here)
    for (int c = 0; c < 9; ++c) dL[c] = dL[c] + rr * r.lam[9 * row + c];
    for (int c = 0; c < 3; ++c) dth[c] = dth[c] + rr * r.th[3 * row + c];
    for (int c = 0; c < ne; ++c) de[c] = de[c] + rr * r.eta[(size_t)ne * row + c];
    const double rw = rr * r.w[row];
    dw = dw + rw;
    drs = drs + rr;
    if (r.src) {
      const int s = r.src[row];
      const double wc = rw * (s == 0 ? 1.0 : 0.0);
      dcam = dcam + wc;
      dlid = dlid + rw * (s == 1 ? 1.0 : 0.0);
      if (r.col) {
        for (int c = 0; c < 3; ++c) dacc[c] = dacc[c] + clip01(r.col[3 * row + c]) * wc;
        dden = dden + wc;
      }
    }
  }
  const int t = (int)(key / (uint32_t)st.M), q = (int)(key % (uint32_t)st.M);
  const size_t i = sidx(st, tiles[t], q);
  for (int c = 0; c < 9; ++c) st.lam[9 * i + c] = st.lam[9 * i + c] + dL[c];
  for (int c = 0; c < 3; ++c) {
    st.th[3 * i + c] = st.th[3 * i + c] + dth[c];
    st.acc[3 * i + c] = st.acc[3 * i + c] + dacc[c];
  }
  for (int c = 0; c < ne; ++c) st.eta[(size_t)ne * i + c] = st.eta[(size_t)ne * i + c] + de[c];
  st.w[i] = st.w[i] + dw;
  st.cam[i] = st.cam[i] + dcam;
  st.lid[i] = st.lid[i] + dlid;
  st.den[i] = st.den[i] + dden;
  if (drs > 0.0) {
    st.lsup[i] = seq;
    st.lupd[i] = seq;
  }
}

// every listed tile: rgb = where(cam > 0, clip(accum / max(denom, eps)), gray), colors = rgb (:1097-1105)
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_rgb(PmStore st, const int32_t* tiles, int n, double eps) {
#pragma clang fp contract(off)
  const long g = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= (long)n * st.M) return;
  const size_t i = sidx(st, tiles[g / st.M], (int)(g % st.M));
  const double den = fmax(st.den[i], eps);
  const bool cam = st.cam[i] > 0.0;
  for (int c = 0; c < 3; ++c) {
    const double v = cam ? clip01(st.acc[3 * i + c] / den) : 0.5;
    st.rgb[3 * i + c] = v;
    st.col[3 * i + c] = v;
  }
}

// timestamps.at[unique(target_slots)].set(ts) in every listed tile (all rows' slots, :1112) and
// the unique-slot flags for n_fused
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_ts(PmStore st, const int32_t* tiles, int n, PmRows r,
                                                           double ts, uint32_t* mark) {
  const long g = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= (long)n * r.n) return;
  const int t = (int)(g / r.n), row = (int)(g % r.n);
  const int q = r.slots[row];
  if (q < 0 || q >= st.M) return;
  st.ts[sidx(st, tiles[t], q)] = ts;
  if (t == 0) mark[q] = 1u;
}

// Step 12b's per-block fuse calls in one pass: key = ((tile position x M + slot) x nb + block) for
// the contributing rows, so a (tile, slot) group's rows sort by block and, within a block, by row.
// Also timestamps.at[unique(target_slots)].set(ts) in every listed tile (:1112; k_pm_fuse_ts's
// writes: no kernel of the fuse reads ts, so they move here).
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_keys_blocks(PmStore st, const int32_t* tiles, double ts,
                                                                    PmRows r, int n_tiles, int M, int nb, int rpb,
                                                                    uint32_t* keys, uint32_t* vals, uint8_t* mark,
                                                                    uint32_t* err, uint32_t nokey) {
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= r.n) return;
  const int tp = r.tpos[g], q = r.slots[g], b = g / rpb;
  const bool ok = q >= 0 && q < M;
  if (!ok) err[0] = 1u;
  else mark[(size_t)b * M + q] = 1;  // every row's slot counts for n_fused (np.unique(target_slots))
  if (ok)
    for (int t = 0; t < n_tiles; ++t) st.ts[sidx(st, tiles[t], q)] = ts;
  const bool v = (r.valid ? r.valid[g] != 0 : true) && tp >= 0 && tp < n_tiles && ok;
  keys[g] = v ? ((uint32_t)tp * (uint32_t)M + (uint32_t)q) * (uint32_t)nb + (uint32_t)b : nokey;
  vals[g] = (uint32_t)g;
}

// The fuse's (key, row) sort for up to kSsWideMax rows in two launches (GCS_FUSE_SMALLSORT; rocPRIM's
// radix sort took five launches at these sizes -- a block sort and four merge passes, ~33 us plus their
// host dispatch).  Each pair is one u64 (key << 32 | row), so the pairs are distinct and their order is
// the stable key order.  k_ss_block: 1,024-pair runs sorted in LDS (bitonic); k_ss_merge: every pair's
// final position = its rank in its run + the pairs below it in every other run (a binary search of each
// run, the runs staged in LDS sixteen at a time: one group up to kSsMax rows -- the reference's 1,536 x 8
// fuse rows --, four groups up to kSsWideMax), then the scatter.
#ifndef GCS_FUSE_SMALLSORT
#define GCS_FUSE_SMALLSORT 1
#endif
constexpr int kSsRun = 1024;
constexpr int kSsMax = 16 * kSsRun;  // 128 KB of runs in k_ss_merge's LDS: one group
constexpr int kSsWideMax = 4 * kSsMax;  // 65,536 rows: four groups
__global__ __launch_bounds__(512) void k_ss_block(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                 int n, uint64_t* __restrict__ runs) {
  __shared__ uint64_t s[kSsRun];
  const int t = threadIdx.x, base = blockIdx.x * kSsRun;
  for (int i = t; i < kSsRun; i += 512) {
    const int g = base + i;
    s[i] = g < n ? ((uint64_t)keys[g] << 32) | (uint64_t)vals[g] : ~0ull;
  }
  for (int size = 2; size <= kSsRun; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      // strides below 64: a wave's pairs lie in its own 128 entries (wave-ordered LDS, no block barrier)
      if (stride >= 64 || size == 2) {
        __syncthreads();
      } else {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      }
      const int x = ((t & ~(stride - 1)) << 1) | (t & (stride - 1)), y = x | stride;
      const uint64_t a = s[x], b = s[y];
      if ((b < a) == ((x & size) == 0)) {
        s[x] = b;
        s[y] = a;
      }
    }
  __syncthreads();
  for (int i = t; i < kSsRun; i += 512) runs[base + i] = s[i];
}
__global__ __launch_bounds__(kSsRun) void k_ss_merge(const uint64_t* __restrict__ runs, int n, int nrun,
                                                     uint32_t* __restrict__ keys_s, uint32_t* __restrict__ vals_s) {
  constexpr int kG = kSsMax / kSsRun;  // runs per LDS group
  __shared__ uint64_t s[kSsMax];
  const int t = threadIdx.x;
  const int g = blockIdx.x * kSsRun + t;
  const int j = blockIdx.x;  // this block's run
  const uint64_t x = runs[g];  // (the grid is nrun blocks: g < nrun kSsRun)
  int pos = t;
  for (int r0 = 0; r0 < nrun; r0 += kG) {
    if (r0 > 0) __syncthreads();  // the previous group's searches are done with s
    {  // every run's loads in flight before the LDS stores (one round trip, not one per run)
      uint64_t v[kG];
#pragma unroll
      for (int i = 0; i < kG; ++i) v[i] = r0 + i < nrun ? runs[(r0 + i) * kSsRun + t] : 0ull;
#pragma unroll
      for (int i = 0; i < kG; ++i)
        if (r0 + i < nrun) s[i * kSsRun + t] = v[i];
    }
    __syncthreads();
    // the pairs of every other run below x: fixed-step lower bounds, the runs' searches side by side
    int lo[kG];
#pragma unroll
    for (int i = 0; i < kG; ++i) lo[i] = 0;
#pragma unroll
    for (int step = kSsRun / 2; step >= 1; step >>= 1)
#pragma unroll
      for (int i = 0; i < kG; ++i)
        if (r0 + i < nrun && s[i * kSsRun + lo[i] + step - 1] < x) lo[i] += step;
#pragma unroll
    for (int i = 0; i < kG; ++i)
      if (r0 + i < nrun && r0 + i != j) pos += lo[i] + (lo[i] == kSsRun - 1 && s[i * kSsRun + kSsRun - 1] < x ? 1 : 0);
  }
  if (x == ~0ull) return;  // padding (after every real pair of the last run)
  keys_s[pos] = (uint32_t)(x >> 32);
  vals_s[pos] = (uint32_t)x;
}

// Long runs of one (tile, slot, block) key -- many measurements associated to the same primitive, as
// in a sparse map -- were one lane's serial walk (the live path's map update spent 0.5 ms in it).  A run
// longer than kFuseChunk (32) rows is cut into chunks: the run's first chunk ends at the first position
// b with b % kFuseChunk == 0 and b - kFuseChunk at or after the run start, later chunks at every such
// b; one lane per chunk sums its rows in row order into P (field-major, kFT fields) and its length
// into Lc, and the group's lane adds the chunk sums in order.  Runs of at most kFuseChunk rows are
// never cut: their sums are bitwise the per-row walk's.  (Deterministic either way.)
constexpr int kFuseChunk = 32;
constexpr int kFT = 28;  // L 9 | theta 3 | eta 9 | r w | r | camera w | lidar w | rgb accumulation 3
__device__ __forceinline__ bool fuse_long_start(const uint32_t* keys, int n, int pos, uint32_t key) {
  if (pos == 0 || keys[pos - 1] != key) return pos + kFuseChunk < n && keys[pos + kFuseChunk] == key;
  return pos % kFuseChunk == 0 && pos >= kFuseChunk && keys[pos - kFuseChunk] == key;
}
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_chunks(PmRows r, const uint32_t* keys, const uint32_t* vals,
                                                               double* P, int* Lc, uint32_t nokey) {
#pragma clang fp contract(off)
  const int pos = blockIdx.x * kPmThreads + threadIdx.x;
  if (pos >= r.n) return;
  const uint32_t key = keys[pos];
  if (key == nokey || !fuse_long_start(keys, r.n, pos, key)) return;
  constexpr int ne = 3 * kNL;
  static_assert(9 + 3 + ne + 4 + 3 == kFT, "fuse chunk layout");
  double dL[9], dth[3], de[ne], dw = 0.0, drs = 0.0, dcam = 0.0, dlid = 0.0, dacc[3] = {0.0, 0.0, 0.0};
  for (int c = 0; c < 9; ++c) dL[c] = 0.0;
  for (int c = 0; c < 3; ++c) dth[c] = 0.0;
  for (int c = 0; c < ne; ++c) de[c] = 0.0;
  // the chunk's end first (contiguous key reads), then the rows with a known trip count, so that
  // several rows' loads are in flight at once (the sum itself stays in row order)
  int end = pos + 1;
  while (end < r.n && keys[end] == key && !(end % kFuseChunk == 0 && keys[end - kFuseChunk] == key)) ++end;
#pragma unroll 2
  for (int q = pos; q < end; ++q) {
    const size_t row = vals[q];
    const double rr = r.resp[row] * 1.0;
    for (int c = 0; c < 9; ++c) dL[c] = dL[c] + rr * r.lam[9 * row + c];
    for (int c = 0; c < 3; ++c) dth[c] = dth[c] + rr * r.th[3 * row + c];
    for (int c = 0; c < ne; ++c) de[c] = de[c] + rr * r.eta[(size_t)ne * row + c];
    const double rw = rr * r.w[row];
    dw = dw + rw;
    drs = drs + rr;
    if (r.src) {
      const int sv = r.src[row];
      const double wc = rw * (sv == 0 ? 1.0 : 0.0);
      dcam = dcam + wc;
      dlid = dlid + rw * (sv == 1 ? 1.0 : 0.0);
      if (r.col)
        for (int c = 0; c < 3; ++c) dacc[c] = dacc[c] + clip01(r.col[3 * row + c]) * wc;
    }
  }
  const size_t n = (size_t)r.n;
  for (int c = 0; c < 9; ++c) P[c * n + pos] = dL[c];
  for (int c = 0; c < 3; ++c) P[(9 + c) * n + pos] = dth[c];
  for (int c = 0; c < ne; ++c) P[(12 + c) * n + pos] = de[c];
  P[21 * n + pos] = dw;
  P[22 * n + pos] = drs;
  P[23 * n + pos] = dcam;
  P[24 * n + pos] = dlid;
  for (int c = 0; c < 3; ++c) P[(25 + c) * n + pos] = dacc[c];
  Lc[pos] = end - pos;
}

// GCS_FUSE_RUNS (default): a long run is summed by one wave instead of chunk by chunk -- lane l takes
// rows start + l, + 64, ... in order, the lanes meet in a fixed xor tree -- and stored as one chunk of
// the run's length (k_pm_fuse_apply_blocks then adds one sum per long run).  The chunk walk was a
// serial chain of dependent row loads per lane (up to 63 rows): 40-50 us per map update on scans
// whose sparse map draws hundreds of associations to one primitive.  Deterministic either way; runs of
// at most kFuseChunk rows are untouched (the per-row walk's sums).
#ifndef GCS_FUSE_RUNS
#define GCS_FUSE_RUNS 1
#endif
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_runs(PmRows r, const uint32_t* keys, const uint32_t* vals,
                                                             double* P, int* Lc, uint32_t nokey) {
#pragma clang fp contract(off)
  __shared__ int s_start[kPmThreads];
  __shared__ int s_wn[kPmThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int pos = blockIdx.x * kPmThreads + t;
  bool st = false;
  if (pos < r.n) {
    const uint32_t key = keys[pos];
    st = key != nokey && (pos == 0 || keys[pos - 1] != key) && pos + kFuseChunk < r.n && keys[pos + kFuseChunk] == key;
  }
  // the block's long-run starts in position order
  const unsigned long long m = __ballot(st);
  if (lane == 0) s_wn[wid] = __popcll(m);
  __syncthreads();
  int base = 0, total = 0;
  for (int w = 0; w < kPmThreads / 64; ++w) {
    if (w < wid) base += s_wn[w];
    total += s_wn[w];
  }
  if (st) s_start[base + __popcll(m & ((1ull << lane) - 1ull))] = pos;
  __syncthreads();
  constexpr int ne = 3 * kNL;
  static_assert(9 + 3 + ne + 4 + 3 == kFT, "fuse chunk layout");
  const size_t n = (size_t)r.n;
  for (int k = wid; k < total; k += kPmThreads / 64) {  // one wave per long run
    const int s = s_start[k];
    const uint32_t key = keys[s];
    int e = s + kFuseChunk;  // the run's end: the first position past it (64 probes per step)
    for (;;) {
      const int p = e + lane;
      const unsigned long long out = __ballot(!(p < r.n && keys[p] == key));
      if (out) {
        e += __ffsll((long long)out) - 1;
        break;
      }
      e += 64;
    }
    double f[kFT];
#pragma unroll
    for (int c = 0; c < kFT; ++c) f[c] = 0.0;
    for (int q = s + lane; q < e; q += 64) {
      const size_t row = vals[q];
      const double rr = r.resp[row] * 1.0;
#pragma unroll
      for (int c = 0; c < 9; ++c) f[c] = f[c] + rr * r.lam[9 * row + c];
#pragma unroll
      for (int c = 0; c < 3; ++c) f[9 + c] = f[9 + c] + rr * r.th[3 * row + c];
#pragma unroll
      for (int c = 0; c < ne; ++c) f[12 + c] = f[12 + c] + rr * r.eta[(size_t)ne * row + c];
      const double rw = rr * r.w[row];
      f[21] = f[21] + rw;
      f[22] = f[22] + rr;
      if (r.src) {
        const int sv = r.src[row];
        const double wc = rw * (sv == 0 ? 1.0 : 0.0);
        f[23] = f[23] + wc;
        f[24] = f[24] + rw * (sv == 1 ? 1.0 : 0.0);
        if (r.col)
#pragma unroll
          for (int c = 0; c < 3; ++c) f[25 + c] = f[25 + c] + clip01(r.col[3 * row + c]) * wc;
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int c = 0; c < kFT; ++c) f[c] = f[c] + __shfl_xor(f[c], off, 64);
    if (lane < kFT) {  // lane c stores field c (every lane holds the whole sum)
      double v = f[0];
#pragma unroll
      for (int c = 1; c < kFT; ++c) v = lane == c ? f[c] : v;
      P[(size_t)lane * n + s] = v;
    }
    if (lane == 0) Lc[s] = e - s;
  }
}

// one lane per (tile, slot) group: for each block in order, d = the block's rows summed in row order
// (a long run: its chunk sums in order, k_pm_fuse_chunks), then slot += d -- the reference's
// block-by-block fuse calls (pipeline.py:1272-1327)
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_apply_blocks(PmStore st, const int32_t* tiles, PmRows r,
                                                                     const uint32_t* keys, const uint32_t* vals,
                                                                     int nb, long long seq, const double* P,
                                                                     const int* Lc, uint32_t nokey) {
#pragma clang fp contract(off)
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= r.n) return;
  const uint32_t key = keys[g];
  if (key == nokey) return;
  const uint32_t grp = key / (uint32_t)nb;
  if (g > 0 && keys[g - 1] != nokey && keys[g - 1] / (uint32_t)nb == grp) return;
  constexpr int ne = 3 * kNL;
  const int t = (int)(grp / (uint32_t)st.M), q = (int)(grp % (uint32_t)st.M);
  const size_t i = sidx(st, tiles[t], q);
  // the slot's accumulators first: their loads overlap the rows' (the adds below keep their order)
  double sL[9], sth[3], sacc[3], se[ne], sw = st.w[i], scam = st.cam[i], slid = st.lid[i], sden = st.den[i];
  for (int c = 0; c < 9; ++c) sL[c] = st.lam[9 * i + c];
  for (int c = 0; c < 3; ++c) {
    sth[c] = st.th[3 * i + c];
    sacc[c] = st.acc[3 * i + c];
  }
  for (int c = 0; c < ne; ++c) se[c] = st.eta[(size_t)ne * i + c];
  bool sup = false;
  int pos = g;
  while (pos < r.n && keys[pos] != nokey && keys[pos] / (uint32_t)nb == grp) {
    const uint32_t kb = keys[pos];
    double dL[9], dth[3], de[ne], dw = 0.0, drs = 0.0, dcam = 0.0, dlid = 0.0, dacc[3] = {0.0, 0.0, 0.0}, dden = 0.0;
    for (int c = 0; c < 9; ++c) dL[c] = 0.0;
    for (int c = 0; c < 3; ++c) dth[c] = 0.0;
    for (int c = 0; c < ne; ++c) de[c] = 0.0;
    if (P && fuse_long_start(keys, r.n, pos, kb)) {  // a long run: its chunk sums, in order
      const size_t n = (size_t)r.n;
      bool first = true;
      while (pos < r.n && keys[pos] == kb) {
        const int len = Lc[pos];
        if (first) {
          for (int c = 0; c < 9; ++c) dL[c] = P[c * n + pos];
          for (int c = 0; c < 3; ++c) dth[c] = P[(9 + c) * n + pos];
          for (int c = 0; c < ne; ++c) de[c] = P[(12 + c) * n + pos];
          dw = P[21 * n + pos];
          drs = P[22 * n + pos];
          if (r.src) {
            dcam = P[23 * n + pos];
            dlid = P[24 * n + pos];
            if (r.col) {
              for (int c = 0; c < 3; ++c) dacc[c] = P[(25 + c) * n + pos];
              dden = dcam;
            }
          }
          first = false;
        } else {
          for (int c = 0; c < 9; ++c) dL[c] = dL[c] + P[c * n + pos];
          for (int c = 0; c < 3; ++c) dth[c] = dth[c] + P[(9 + c) * n + pos];
          for (int c = 0; c < ne; ++c) de[c] = de[c] + P[(12 + c) * n + pos];
          dw = dw + P[21 * n + pos];
          drs = drs + P[22 * n + pos];
          if (r.src) {
            const double wc = P[23 * n + pos];
            dcam = dcam + wc;
            dlid = dlid + P[24 * n + pos];
            if (r.col) {
              for (int c = 0; c < 3; ++c) dacc[c] = dacc[c] + P[(25 + c) * n + pos];
              dden = dden + wc;
            }
          }
        }
        pos += len;
      }
    }
    for (; pos < r.n && keys[pos] == kb; ++pos) {
      const size_t row = vals[pos];
      const double rr = r.resp[row] * 1.0;
      for (int c = 0; c < 9; ++c) dL[c] = dL[c] + rr * r.lam[9 * row + c];
      for (int c = 0; c < 3; ++c) dth[c] = dth[c] + rr * r.th[3 * row + c];
      for (int c = 0; c < ne; ++c) de[c] = de[c] + rr * r.eta[(size_t)ne * row + c];
      const double rw = rr * r.w[row];
      dw = dw + rw;
      drs = drs + rr;
      if (r.src) {
        const int sv = r.src[row];
        const double wc = rw * (sv == 0 ? 1.0 : 0.0);
        dcam = dcam + wc;
        dlid = dlid + rw * (sv == 1 ? 1.0 : 0.0);
        if (r.col) {
          for (int c = 0; c < 3; ++c) dacc[c] = dacc[c] + clip01(r.col[3 * row + c]) * wc;
          dden = dden + wc;
        }
      }
    }
    // (one block's run: added to the slot in block order, as the per-block fuse steps do)
    for (int c = 0; c < 9; ++c) sL[c] = sL[c] + dL[c];
    for (int c = 0; c < 3; ++c) {
      sth[c] = sth[c] + dth[c];
      sacc[c] = sacc[c] + dacc[c];
    }
    for (int c = 0; c < ne; ++c) se[c] = se[c] + de[c];
    sw = sw + dw;
    scam = scam + dcam;
    slid = slid + dlid;
    sden = sden + dden;
    sup = sup || drs > 0.0;
  }
  for (int c = 0; c < 9; ++c) st.lam[9 * i + c] = sL[c];
  for (int c = 0; c < 3; ++c) {
    st.th[3 * i + c] = sth[c];
    st.acc[3 * i + c] = sacc[c];
  }
  for (int c = 0; c < ne; ++c) st.eta[(size_t)ne * i + c] = se[c];
  st.w[i] = sw;
  st.cam[i] = scam;
  st.lid[i] = slid;
  st.den[i] = sden;
  if (sup) {
    st.lsup[i] = seq;
    st.lupd[i] = seq;
  }
}

// unique slots per block (grid: blocks of slots x nb): integer atomics into device counters
// Each mark is read by one lane, which clears it: the marks are all zero again for the next call
// (zeroed once at allocation; no per-call fill).
// ticket (may be null): the last block to finish publishes the nb counters to dst (the mapped buffer)
// and re-arms them and the ticket -- each block's count add happens before its ticket add, which is a
// release at agent scope (one lane per block), and the last block acquires at agent scope before it
// reads the counts back as agent-scope atomic loads; this was a launch of its own (k_pm_publish_u32,
// ~5 us of step 12b)
__global__ __launch_bounds__(kPmThreads) void k_pm_count_marks_blocks(uint8_t* mark, int M, uint32_t* cnt,
                                                                      uint32_t* ticket, int nb, uint32_t* dst) {
  __shared__ double lds[kPmThreads / 64];
  __shared__ int s_last;
  const int b = blockIdx.y;
  double c = 0.0;
  for (int q = blockIdx.x * kPmThreads + threadIdx.x; q < M; q += gridDim.x * kPmThreads) {
    uint8_t& mk = mark[(size_t)b * M + q];
    c += mk ? 1.0 : 0.0;
    if (mk) mk = 0;
  }
  c = block_sum_d<kPmThreads>(c, lds);
  if (threadIdx.x == 0 && c > 0.0) atomicAdd(cnt + b, (uint32_t)c);
  if (!ticket) return;
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    s_last = tk == gridDim.x * gridDim.y - 1u ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  for (int i = threadIdx.x; i < nb; i += kPmThreads) {
    dst[i] = __hip_atomic_load(cnt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// unique target slots: per-block counts of the marks, added with an integer atomic (exact in any order)
__global__ __launch_bounds__(kPmThreads) void k_pm_count_marks(const uint32_t* mark, int M, uint32_t* n_unique) {
  __shared__ double lds[kPmThreads / 64];
  const int q = blockIdx.x * kPmThreads + threadIdx.x;
  double c = q < M && mark[q] ? 1.0 : 0.0;
  c = block_sum_d<kPmThreads>(c, lds);
  if (threadIdx.x == 0 && c > 0.0) atomicAdd(n_unique, (uint32_t)c);
}

// grid (tiles, blocks per tile): block b of tile t covers slots b*kPmRed + j*gridDim.y*kPmRed
__device__ __forceinline__ int part_row() { return blockIdx.x * gridDim.y + blockIdx.y; }

// valid counts (partials: one per block)
__global__ __launch_bounds__(kPmRed) void k_pm_count(PmStore st, const int32_t* tiles, double* part) {
  __shared__ double lds[kPmRed / 64];
  const int ti = tiles[blockIdx.x];
  double c = 0.0;
  for (int q = blockIdx.y * kPmRed + threadIdx.x; q < st.M; q += gridDim.y * kPmRed)
    c += st.valid[sidx(st, ti, q)] ? 1.0 : 0.0;
  c = block_sum_d<kPmRed>(c, lds);
  if (threadIdx.x == 0) part[part_row()] = c;
}

// cull (:1217-1250): below = valid & w < thr -> invalid; culled count, mass dropped, sum of all weights,
// valid count after (one workgroup per tile, fixed-order sums)
// forget != 0: the forgetting pass of step 12b rides along (w := gamma w after the cull read it,
// :1443-1447 -- the same product k_pm_forget writes, one pass over the tile instead of two)
__global__ __launch_bounds__(kPmRed) void k_pm_cull(PmStore st, const int32_t* tiles, double thr, double* part,
                                                    int forget, double gamma) {
  __shared__ double lds[kPmRed / 64];
  const int ti = tiles[blockIdx.x];
  double nb = 0.0, md = 0.0, ws = 0.0, nv = 0.0;
  for (int q = blockIdx.y * kPmRed + threadIdx.x; q < st.M; q += gridDim.y * kPmRed) {
    const size_t i = sidx(st, ti, q);
    const double w = st.w[i];
    const bool v = st.valid[i] != 0;
    const bool b = v && w < thr;
    nb += b ? 1.0 : 0.0;
    md += w * (b ? 1.0 : 0.0);
    ws += w;
    nv += (v && !b) ? 1.0 : 0.0;
    if (b) st.valid[i] = 0;
    if (forget) st.w[i] = gamma * w;
  }
  nb = block_sum_d<kPmRed>(nb, lds);
  md = block_sum_d<kPmRed>(md, lds);
  ws = block_sum_d<kPmRed>(ws, lds);
  nv = block_sum_d<kPmRed>(nv, lds);
  if (threadIdx.x == 0) {
    double* o = part + 4 * part_row();
    o[0] = nb;
    o[1] = md;
    o[2] = ws;
    o[3] = nv;
  }
}

__global__ __launch_bounds__(kPmThreads) void k_pm_forget(PmStore st, const int32_t* tiles, int n, double gamma) {
  const long g = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= (long)n * st.M) return;
  const size_t i = sidx(st, tiles[g / st.M], (int)(g % st.M));
  st.w[i] = gamma * st.w[i];
}

// recency inflate (:1425-1463): decay = clip(exp(-lam dt), min_scale, 1) on valid slots; Lambda, theta
// scaled; per tile [sum (1 - decay) valid, sum (1/decay - 1) valid, n_valid]
__global__ __launch_bounds__(kPmRed) void k_pm_recency(PmStore st, const int32_t* tiles, long long seq, double lam,
                                                       double min_scale, double* out) {
#pragma clang fp contract(off)
  __shared__ double lds[kPmRed / 64];
  const int ti = tiles[blockIdx.x];
  double dn = 0.0, inf = 0.0, nv = 0.0;
  for (int q = blockIdx.y * kPmRed + threadIdx.x; q < st.M; q += gridDim.y * kPmRed) {
    const size_t i = sidx(st, ti, q);
    // an empty slot's factor is 1 and its terms are zero (x * 1.0 == x): only valid slots are read
    // and written (the map is sparse: the reference sizes' 50,000-slot tiles hold a few thousand)
    if (st.valid[i] == 0) continue;
    const long long dt = max(0ll, seq - st.lsup[i]);
    const double d = fmin(fmax(exp(-lam * (double)dt), min_scale), 1.0);
    for (int c = 0; c < 9; ++c) st.lam[9 * i + c] = st.lam[9 * i + c] * d;
    for (int c = 0; c < 3; ++c) st.th[3 * i + c] = st.th[3 * i + c] * d;
    nv += 1.0;
    dn += (1.0 - d) * 1.0;
    inf += ((1.0 / d) - 1.0) * 1.0;
  }
  dn = block_sum_d<kPmRed>(dn, lds);
  inf = block_sum_d<kPmRed>(inf, lds);
  nv = block_sum_d<kPmRed>(nv, lds);
  if (threadIdx.x == 0) {
    out[3 * part_row()] = dn;
    out[3 * part_row() + 1] = inf;
    out[3 * part_row() + 2] = nv;
  }
}

// ---------------------------------------------------------------- merge-reduce
__global__ __launch_bounds__(kPmThreads) void k_pm_merge_prep(PmStore st, int ti, double eps_lift, double* mu,
                                                              double* Sig, double* det) {
  const int q = blockIdx.x * kPmThreads + threadIdx.x;
  if (q >= st.M) return;
  const size_t i = sidx(st, ti, q);
  double a[3][3], d;
  int perm[3];
  lu3(st.lam + 9 * i, eps_lift, a, perm, d);
  lu3_solve(a, perm, st.th + 3 * i, mu + 3 * q);
  double S[9];
  lu3_inv(a, perm, S);
  for (int c = 0; c < 9; ++c) Sig[9 * q + c] = S[c];
  double b[3][3], dS;
  int pb[3];
  lu3(S, 0.0, b, pb, dS);
  det[q] = dS;
}

// pair p of triu_indices(M, 1), row-major
__device__ __forceinline__ void pair_ij(long p, int M, int& i, int& j) {
  const double m2 = 2.0 * M - 1.0;
  int ii = (int)floor((m2 - sqrt(m2 * m2 - 8.0 * (double)p)) * 0.5);
  ii = max(0, min(ii, M - 2));
  auto start = [M](long r) { return r * (2L * M - r - 1) / 2; };
  while (ii > 0 && start(ii) > p) --ii;
  while (ii < M - 2 && start(ii + 1) <= p) ++ii;
  i = ii;
  j = (int)(p - start(ii)) + ii + 1;
}

__global__ __launch_bounds__(kPmThreads) void k_pm_merge_dist(PmStore st, int ti, long P, double eps_lift,
                                                              const double* mu, const double* Sig, const double* det,
                                                              double* dist) {
#pragma clang fp contract(off)
  const long p = (long)blockIdx.x * kPmThreads + threadIdx.x;
  if (p >= P) return;
  int i, j;
  pair_ij(p, st.M, i, j);
  if (!(st.valid[sidx(st, ti, i)] && st.valid[sidx(st, ti, j)])) {
    dist[p] = INFINITY;
    return;
  }
  double S[9];
  for (int c = 0; c < 9; ++c) S[c] = 0.5 * (Sig[9 * i + c] + Sig[9 * j + c]);
  double a[3][3], dS;
  int perm[3];
  lu3(S, 0.0, a, perm, dS);
  double b[3][3], dd;
  int pb[3];
  lu3(S, eps_lift, b, pb, dd);
  double Si[9];
  lu3_inv(b, pb, Si);
  const double dm[3] = {mu[3 * i] - mu[3 * j], mu[3 * i + 1] - mu[3 * j + 1], mu[3 * i + 2] - mu[3 * j + 2]};
  double row[3];
  for (int c = 0; c < 3; ++c) row[c] = (dm[0] * Si[c] + dm[1] * Si[3 + c]) + dm[2] * Si[6 + c];
  const double quad = 0.125 * ((row[0] * dm[0] + row[1] * dm[1]) + row[2] * dm[2]);
  const double lt = 0.5 * log(dS / sqrt(det[i] * det[j] + 1e-24));
  dist[p] = quad + lt;
}

struct MinKey {
  double d;
  long p;
};
__device__ __forceinline__ bool key_less(double d1, long p1, double d2, long p2) {
  return d1 < d2 || (d1 == d2 && p1 < p2);
}

// one round: block argmin of (distance, pair) over the eligible pairs -> partials
__global__ __launch_bounds__(kPmThreads) void k_pm_merge_min(PmStore st, long P, const double* dist, double thr,
                                                             const uint8_t* used, double* pd, long long* pp) {
  __shared__ double sd[kPmThreads];
  __shared__ long long sp[kPmThreads];
  double bd = INFINITY;
  long bp = -1;
  for (long p = (long)blockIdx.x * kPmThreads + threadIdx.x; p < P; p += (long)gridDim.x * kPmThreads) {
    const double d = dist[p];
    if (!(isfinite(d) && d < thr)) continue;
    int i, j;
    pair_ij(p, st.M, i, j);
    if (used[i] || used[j]) continue;
    if (bp < 0 || key_less(d, p, bd, bp)) {
      bd = d;
      bp = p;
    }
  }
  sd[threadIdx.x] = bd;
  sp[threadIdx.x] = bp;
  __syncthreads();
  for (int s = kPmThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const long p2 = sp[threadIdx.x + s];
      if (p2 >= 0 && (sp[threadIdx.x] < 0 || key_less(sd[threadIdx.x + s], p2, sd[threadIdx.x], sp[threadIdx.x]))) {
        sd[threadIdx.x] = sd[threadIdx.x + s];
        sp[threadIdx.x] = p2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    pd[blockIdx.x] = sd[0];
    pp[blockIdx.x] = sp[0];
  }
}

__global__ void k_pm_merge_pick(int M, const double* pd, const long long* pp, int nblk, uint8_t* used, int32_t* sel,
                                int32_t* n_sel) {
  if (threadIdx.x != 0) return;
  double bd = INFINITY;
  long bp = -1;
  for (int b = 0; b < nblk; ++b)
    if (pp[b] >= 0 && (bp < 0 || key_less(pd[b], pp[b], bd, bp))) {
      bd = pd[b];
      bp = pp[b];
    }
  if (bp < 0) return;
  int i, j;
  pair_ij(bp, M, i, j);
  used[i] = used[j] = 1;
  const int k = n_sel[0];
  sel[2 * k] = i;
  sel[2 * k + 1] = j;
  n_sel[0] = k + 1;
}

__global__ void k_pm_merge_apply(PmStore st, int ti, const int32_t* sel, const int32_t* n_sel, const double* mu,
                                 const double* Sig, double eps_psd) {
#pragma clang fp contract(off)
  const int k = threadIdx.x;
  if (k >= n_sel[0]) return;
  const int qi = sel[2 * k], qj = sel[2 * k + 1];
  const size_t i = sidx(st, ti, qi), j = sidx(st, ti, qj);
  const double w1 = st.w[i], w2 = st.w[j], ws = w1 + w2;
  if (!(ws > 0.0)) return;
  double mm[3], d1[3], d2[3];
  for (int c = 0; c < 3; ++c) mm[c] = (w1 * mu[3 * qi + c] + w2 * mu[3 * qj + c]) / ws;
  for (int c = 0; c < 3; ++c) {
    d1[c] = mu[3 * qi + c] - mm[c];
    d2[c] = mu[3 * qj + c] - mm[c];
  }
  double Sm[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      Sm[3 * r + c] = (w1 * (Sig[9 * qi + 3 * r + c] + d1[r] * d1[c]) + w2 * (Sig[9 * qj + 3 * r + c] + d2[r] * d2[c])) /
                          ws + (r == c ? eps_psd : 0.0);
  double a[3][3], dt;
  int perm[3];
  lu3(Sm, 0.0, a, perm, dt);
  double Lm[9];
  lu3_inv(a, perm, Lm);
  for (int c = 0; c < 9; ++c) st.lam[9 * i + c] = Lm[c];
  for (int r = 0; r < 3; ++r) st.th[3 * i + r] = (Lm[3 * r] * mm[0] + Lm[3 * r + 1] * mm[1]) + Lm[3 * r + 2] * mm[2];
  constexpr int ne = 3 * kNL;
  for (int c = 0; c < ne; ++c)
    st.eta[(size_t)ne * i + c] = (w1 * st.eta[(size_t)ne * i + c] + w2 * st.eta[(size_t)ne * j + c]) / ws;
  const double cam = st.cam[i] + st.cam[j];
  const double den = st.den[i] + st.den[j];
  for (int c = 0; c < 3; ++c) {
    const double acc = st.acc[3 * i + c] + st.acc[3 * j + c];
    const double rg = cam > 0.0 ? clip01(acc / fmax(den, eps_psd)) : 0.5;
    st.acc[3 * i + c] = acc;
    st.col[3 * i + c] = rg;
    st.rgb[3 * i + c] = rg;
  }
  st.cam[i] = cam;
  st.lid[i] = st.lid[i] + st.lid[j];
  st.den[i] = den;
  st.w[i] = ws;
  st.ts[i] = fmax(st.ts[i], st.ts[j]);
  st.cts[i] = fmin(st.cts[i], st.cts[j]);
  st.lsup[i] = max(st.lsup[i], st.lsup[j]);
  st.lupd[i] = max(st.lupd[i], st.lupd[j]);
  st.w[j] = 0.0;
  st.valid[j] = 0;
}

constexpr int kMergeBlocks = 512;

// ---------------------------------------------------------------- step 12b (pipeline.py:1244-1447)
struct PmMeas {
  const double *lam, *th, *eta, *w, *col;
  const uint8_t* valid;
  const int32_t* src;
  int n;
  const double* resp;
  const int64_t *ctile, *cslot;
  const double* rmass;
  int k;
};

struct PmWorld {
  double R[9], t[3], eps_lift;
};

// Lambda_w = (R Lambda) R^T, mu_w = R (Lambda + eps I)^-1 theta + t, theta_w = Lambda_w mu_w, eta_w = R eta
__device__ __forceinline__ void world_row(const PmWorld& W, const double* L, const double* th, const double* eta, int nl, double* Lw,
                          double* thw, double* ew, double* muw) {
#pragma clang fp contract(off)
  double RL[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) RL[3 * r + c] = (W.R[3 * r] * L[c] + W.R[3 * r + 1] * L[3 + c]) + W.R[3 * r + 2] * L[6 + c];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      Lw[3 * r + c] = (RL[3 * r] * W.R[3 * c] + RL[3 * r + 1] * W.R[3 * c + 1]) + RL[3 * r + 2] * W.R[3 * c + 2];
  double a[3][3], det, mb[3];
  int perm[3];
  lu3(L, W.eps_lift, a, perm, det);
  lu3_solve(a, perm, th, mb);
  for (int r = 0; r < 3; ++r) muw[r] = ((W.R[3 * r] * mb[0] + W.R[3 * r + 1] * mb[1]) + W.R[3 * r + 2] * mb[2]) + W.t[r];
  if (thw)
    for (int r = 0; r < 3; ++r) thw[r] = (Lw[3 * r] * muw[0] + Lw[3 * r + 1] * muw[1]) + Lw[3 * r + 2] * muw[2];
  if (ew)
    for (int b = 0; b < nl; ++b)
      for (int r = 0; r < 3; ++r)
        ew[3 * b + r] = (W.R[3 * r] * eta[3 * b] + W.R[3 * r + 1] * eta[3 * b + 1]) + W.R[3 * r + 2] * eta[3 * b + 2];
}

struct PmRowBuf {
  double *lam, *th, *eta, *w, *resp, *col, *fm;
  uint8_t* valid;
  int32_t *src, *tpos, *slots;
  double* w_host;  // k_pm_proposals: the proposal weights also into the mapped buffer (may be null)
};

// step 12b's tile list and active ids as kernel arguments (no host-to-device copy)
constexpr int kPmArgTiles = 64;
struct PmTileArgs {
  int n;
  int32_t tiles[kPmArgTiles];
  int64_t ids[kPmArgTiles];
};
__global__ void k_pm_stage_tiles(PmTileArgs a, int32_t* tiles, int64_t* ids) {
  const int i = threadIdx.x;
  if (i < a.n) {
    tiles[i] = a.tiles[i];
    ids[i] = a.ids[i];
  }
}

// per association block b and listed tile t: the sum of fm over the block's rows with tpos == t (the
// fused_mass_total terms, pipeline.py:1306-1308), a fixed-order tree per (b, t), into mapped memory
// grid (blocks, tiles): one workgroup per (association block, tile) -- the tiles' sums used to run
// one after another in the block's workgroup (n passes and n reductions in sequence)
__global__ __launch_bounds__(kPmThreads) void k_pm_fm_sums(const double* fm, const int32_t* tpos, int bk, int n,
                                                           double* out) {
  __shared__ double lds[kPmThreads / 64];
  const int b = blockIdx.x, t = blockIdx.y;
  double s = 0.0;
  for (int q = threadIdx.x; q < bk; q += kPmThreads) {
    const size_t g = (size_t)b * bk + q;
    s += tpos[g] == t ? fm[g] : 0.0;
  }
  s = block_sum_d<kPmThreads>(s, lds);
  if (threadIdx.x == 0) out[b * n + t] = s;
}

// block_associations_for_fuse (primitive_association.py:561-588) + the world transform, rows in
// (block, measurement, candidate) order; fm = w r [valid and tile active] (fused mass terms)
__global__ __launch_bounds__(kPmThreads) void k_pm_fuse_rows(PmMeas m, PmWorld W, int nl, int block, int nrows,
                                                             const int64_t* act_ids, int n_act, PmRowBuf o) {
  const int g = blockIdx.x * kPmThreads + threadIdx.x;
  if (g >= nrows) return;
  const int row = g / m.k, k = g % m.k;  // row = b * block + i
  const int mi = min(row, m.n - 1);
  const bool vr = row < m.n && m.valid[mi] != 0;
  const int64_t tid = m.ctile[(size_t)mi * m.k + k];
  int tp = -1;
  for (int q = 0; q < n_act; ++q)
    if (act_ids[q] == tid) {
      tp = q;
      break;
    }
  const double r = m.resp[(size_t)mi * m.k + k] * (vr ? 1.0 : 0.0);
  double Lw[9], thw[3], ew[3 * kNL], muw[3];
  world_row(W, m.lam + 9 * (size_t)mi, m.th + 3 * (size_t)mi, m.eta + (size_t)3 * kNL * mi, kNL, Lw, thw, ew, muw);
  for (int c = 0; c < 9; ++c) o.lam[9 * (size_t)g + c] = Lw[c];
  for (int c = 0; c < 3; ++c) {
    o.th[3 * (size_t)g + c] = thw[c];
    o.col[3 * (size_t)g + c] = m.col ? m.col[3 * (size_t)mi + c] : 0.0;
  }
  for (int c = 0; c < 3 * kNL; ++c) o.eta[(size_t)3 * kNL * g + c] = ew[c];
  const double w = m.w[mi];
  o.w[g] = w;
  o.resp[g] = r;
  o.valid[g] = vr ? 1 : 0;
  o.src[g] = m.src ? m.src[mi] : 1;
  o.tpos[g] = tp;
  o.slots[g] = (int32_t)m.cslot[(size_t)mi * m.k + k];
  o.fm[g] = (vr && tp >= 0) ? (w * r) * 1.0 : 0.0;
  (void)block;
}

// Novelty proposals per active tile (pipeline.py:1331-1375): one 1024-thread workgroup per tile;
// the stable argsort of -score_t is a rank count over (key, index); rows in (tile, rank) order.
constexpr int kPropThreads = 1024;
constexpr int kPropLds = 2048;     // measurement rows a map update handles (scores and ranks in LDS)
constexpr int kPropMaxIns = 1024;  // k_insert_tile bound
__global__ __launch_bounds__(kPropThreads) void k_pm_proposals(PmMeas m, PmWorld W, int nl, double eps_mass,
                                                               double h_tile, const int64_t* act_ids, int kins,
                                                               double* score_buf, int64_t* tile_buf, PmRowBuf o) {
#pragma clang fp contract(off)
  __shared__ double lds[kPropThreads / 64];
  __shared__ double s_sc[kPropLds];
  __shared__ int s_in[kPropLds], s_pre[kPropLds], s_slot[kPropMaxIns];
  __shared__ double s_key[kPropLds];  // the compacted rows' keys -score, in index order
  __shared__ int s_wsum[kPropThreads / 64];
  __shared__ int s_any;
  const int t = blockIdx.x;
  const int64_t tid = act_ids[t];
  double* sc = score_buf + (size_t)t * m.n;
  double nv = 0.0;
  for (int i = threadIdx.x; i < m.n; i += kPropThreads) nv += m.valid[i] ? 1.0 : 0.0;
  nv = block_sum_d<kPropThreads>(nv, lds);
  const double asum = fmax(nv, eps_mass);
  for (int i = threadIdx.x; i < m.n; i += kPropThreads) {  // the measurement's tile at z_t (tiling.py:126-145)
    double Lw[9], muw[3];
    world_row(W, m.lam + 9 * (size_t)i, m.th + 3 * (size_t)i, nullptr, 0, Lw, nullptr, nullptr, muw);
    const double h = fmax(h_tile, 1e-12);
    const double s2 = muw[0] * 0.5 + muw[1] * (1.7320508075688772 * 0.5);
    const long long c1 = (long long)floor(muw[0] / h), c2 = (long long)floor(s2 / h), cz = (long long)floor(muw[2] / h);
    const long long M21 = (1LL << 21) - 1, B21 = 1LL << 20;
    const int64_t mt = (((c1 + B21) & M21) << 42) | (((c2 + B21) & M21) << 21) | ((cz + B21) & M21);
    if (t == 0) tile_buf[i] = mt;
    const double vf = m.valid[i] ? 1.0 : 0.0;
    const double a = vf / asum;
    const double nov = fmax(a - m.rmass[i], 0.0);
    const double score = nov * m.w[i] - (1.0 - vf) * 1e6;
    sc[i] = mt == tid ? score : -1e30;
    s_sc[i] = sc[i];
  }
  __syncthreads();
  const double* scr = s_sc;
  // rank of each measurement under (-score_t ascending, index); ranks < kins are the proposals.  The
  // tile's measurements (score_t > -1e29) are compacted in index order and ranked among themselves;
  // every other row has the key 1e30, above all of them, so its rank is c + (its index among them).
  int* slot_of = s_slot;
  int run = 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int c0 = 0; c0 < m.n; c0 += kPropThreads) {
    const int i = c0 + threadIdx.x;
    const int f = i < m.n && scr[i] > -1e29 ? 1 : 0;
    int x = f;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    __syncthreads();
    if (lane == 63) s_wsum[wid] = x;
    __syncthreads();
    int pre = run + x - f;
    for (int w = 0; w < wid; ++w) pre += s_wsum[w];
    int tot = 0;
    for (int w = 0; w < kPropThreads / 64; ++w) tot += s_wsum[w];
    if (f) s_in[pre] = i;
    s_pre[i < m.n ? i : 0] = i < m.n ? pre : 0;  // in-tile rows before i
    run += tot;
  }
  __syncthreads();
  const int c = run;
  // the compacted keys in their own array (s_in is in index order, so the index tie-break is the
  // position's)
  for (int a = threadIdx.x; a < c; a += kPropThreads) s_key[a] = -scr[s_in[a]];
  __syncthreads();
  // one wave per row: its lanes count the smaller keys over strided slices of the list and add the
  // counts (integers: exact in any order), so every row costs c / 64 steps -- a lane per row with an
  // early exit left the top-ranked rows scanning the whole list while the rest of the block waited
  for (int a = wid; a < c; a += kPropThreads / 64) {
    const double ka = s_key[a];
    int cnt = 0;
    for (int b = lane; b < c; b += 64) {
      const double kb = s_key[b];
      cnt += (kb < ka || (kb == ka && b < a)) ? 1 : 0;
    }
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0 && cnt < kins) slot_of[cnt] = s_in[a];
  }
  for (int i = threadIdx.x; i < m.n; i += kPropThreads) {
    if (scr[i] > -1e29) continue;
    const int rank = c + (i - s_pre[i]);
    if (rank < kins) slot_of[rank] = i;
  }
  if (threadIdx.x == 0) s_any = 0;
  __syncthreads();
  for (int q = threadIdx.x; q < kins; q += kPropThreads) {
    const int i = slot_of[q];
    if (q < m.n && sc[i] > -1e20) s_any = 1;  // in_tile[ins] & (score_t[ins] > -1e20) (plain store: one value)
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kins; q += kPropThreads) {
    const size_t g = (size_t)t * kins + q;
    const int i = q < m.n ? slot_of[q] : 0;
    const bool in_tile = q < m.n && sc[i] > -1e29;  // score_t == -1e30 exactly where out of tile
    const bool vn = s_any ? (in_tile && sc[i] > -1e20) : true;
    double Lw[9], thw[3], ew[3 * kNL], muw[3];
    world_row(W, m.lam + 9 * (size_t)i, m.th + 3 * (size_t)i, m.eta + (size_t)3 * kNL * i, kNL, Lw, thw, ew, muw);
    for (int c = 0; c < 9; ++c) o.lam[9 * g + c] = Lw[c];
    for (int c = 0; c < 3; ++c) {
      o.th[3 * g + c] = thw[c];
      o.col[3 * g + c] = m.col ? m.col[3 * (size_t)i + c] : 0.0;
    }
    for (int c = 0; c < 3 * kNL; ++c) o.eta[(size_t)3 * kNL * g + c] = ew[c];
    const double vf = m.valid[i] ? 1.0 : 0.0;
    const double nov = fmax(vf / asum - m.rmass[i], 0.0);
    o.w[g] = in_tile ? nov * m.w[i] : 0.0;
    if (o.w_host) o.w_host[g] = o.w[g];
    o.valid[g] = vn ? 1 : 0;
    o.src[g] = m.src ? m.src[i] : 1;
  }
}

}  // namespace
}  // namespace gcs

using namespace gcs;

struct gcs_pmap {
  int device = 0, M = 0, T = 0, nl = 3, max_merge = 0;
  hipStream_t own = nullptr, stream = nullptr;
  PmStore st{};
  void* fields[GCS_PM_NFIELDS] = {};
  // sort scratch (view / insert: T tiles x M slots)
  uint64_t *keys = nullptr, *keys_s = nullptr;
  uint32_t *vals = nullptr, *vals_s = nullptr;
  uint32_t* seg = nullptr;  // tile positions of the key-sorted entries
  int32_t* d_tiles = nullptr;
  int64_t* d_tids = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  // fuse scratch (grown on demand)
  uint32_t *fk = nullptr, *fk_s = nullptr, *fv = nullptr, *fv_s = nullptr;
  void* ftemp = nullptr;
  size_t ftemp_bytes = 0;
  int frows = 0;
  double* fterm = nullptr;  // step 12b: chunk sums of long fuse runs (k_pm_fuse_chunks), grown
  int* flen = nullptr;
  size_t fterm_n = 0;
  uint32_t* mark = nullptr;  // fuse: slots seen (n_fused)
  uint32_t* dcnt = nullptr;  // fuse: unique-slot counter (device memory: atomics stay off the mapped buffer)
  uint8_t* bmark = nullptr;   // step 12b: slots seen per association block (grown)
  size_t bmark_bytes = 0;
  uint32_t* bcnt = nullptr;   // step 12b: unique slots per block (kMaxFuseBlocks)
  uint32_t* bticket = nullptr;  // step 12b: k_pm_count_marks_blocks' arrival ticket
  // step-12b scratch (grown on demand)
  void* ub = nullptr;
  size_t ub_bytes = 0;
  // merge scratch
  double *mmu = nullptr, *msig = nullptr, *mdet = nullptr, *mdist = nullptr, *mpd = nullptr;
  long long* mpp = nullptr;
  uint8_t* mused = nullptr;
  int32_t *msel = nullptr, *mnsel = nullptr;
  // k_pm_topk: per-tile runs (grown) and the merge tickets (max_tiles x levels x nodes, zeroed once;
  // each merging workgroup re-arms its ticket)
  uint64_t* run_key = nullptr;
  uint32_t* run_slot = nullptr;
  size_t run_cap = 0;
  uint32_t* tickets = nullptr;
  uint32_t* topk_skip = nullptr;  // k_pm_topk_sparse -> k_pm_topk: the tiles it finished (max_tiles)
  uint32_t* other_bm = nullptr;   // k_pm_keys -> k_pm_topk_sparse: non-empty-key bitmap (max_tiles x M bits)
  uint32_t* below = nullptr;      // k_pm_keys -> k_pm_topk_sparse: per tile, keys under the empty-slot key
  // small host-mapped results
  char* h_small = nullptr;
  char* d_small = nullptr;
  std::string err;
  // step 12b queued by gcs::live::pmap_update_launch, read by pmap_update_collect
  struct {
    bool on = false;
    int n = 0, nb = 0, kins = 0, nbt = 0;
    int64_t next_id = 0;
    std::vector<int32_t> tiles;
    gcs_pmap_update_config cfg{};
  } pend;
};

namespace {
constexpr size_t kSmall = 4 << 20;
constexpr size_t kWiOff = 1 << 20;  // step 12b: proposal weights (n x k_insert_tile doubles)
constexpr size_t kFmOff = 2 << 20;  // step 12b: fused mass per (association block, tile)
constexpr size_t kRecOff = 3 << 20; // recency inflation partials (kept apart from step 12b's cull partials)
constexpr size_t kPartOff = 1 << 16;  // per-(tile, block) reduction partials in the mapped buffer
constexpr int kMaxBlocksPerTile = 64;
constexpr int kMaxFuseBlocks = 256;  // association blocks of one map update
int blocks_per_tile(int M) { return std::max(1, std::min(kMaxBlocksPerTile, (M + kPmRed - 1) / kPmRed)); }
const int kFieldWidth[GCS_PM_NFIELDS] = {9, 3, -1, 1, 1, 1, 3, 1, 1, 3, 1, 3, 1, 1, 1, 1};
const int kFieldBytes[GCS_PM_NFIELDS] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 1};

int pm_fail(gcs_pmap* p, int rc, const std::string& m) {
  p->err = m;
  return rc;
}
#define PMCHK(p, call)                                                                                   \
  do {                                                                                                   \
    hipError_t e_ = (call);                                                                              \
    if (e_ != hipSuccess) return pm_fail(p, GCS_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

size_t field_elems(const gcs_pmap* p, int f) {
  const int w = kFieldWidth[f] < 0 ? 3 * p->nl : kFieldWidth[f];
  return (size_t)p->M * w;
}

int check_tiles(gcs_pmap* p, const int32_t* tiles, int n, bool allow_missing) {
  if (n < 0 || n > p->T) return pm_fail(p, GCS_ERR_ARG, "tile list longer than max_tiles");
  if (n > 0 && !tiles) return pm_fail(p, GCS_ERR_ARG, "null tile list");
  std::vector<char> seen(p->T, 0);
  for (int i = 0; i < n; ++i) {
    if (tiles[i] < 0 && allow_missing) continue;
    if (tiles[i] < 0 || tiles[i] >= p->T) return pm_fail(p, GCS_ERR_ARG, "tile storage index out of range");
    if (!allow_missing && seen[tiles[i]]) return pm_fail(p, GCS_ERR_ARG, "tile listed twice");
    seen[tiles[i]] = 1;
  }
  return GCS_OK;
}

int upload_tiles(gcs_pmap* p, const int32_t* tiles, int n) {
  if (n > 0) PMCHK(p, hipMemcpyAsync(p->d_tiles, tiles, n * sizeof(int32_t), hipMemcpyHostToDevice, p->stream));
  return GCS_OK;
}

// stable per-tile sort of the slot keys (mode 0 view, 1 eviction): one radix sort of every listed
// tile's (key, tile position x M + slot), then a stable radix sort on the tile position -- per tile the
// key order with ties by slot (LSD composition).  Result (tile position x M + slot) in vals.
int sort_tiles(gcs_pmap* p, int n, int mode, long long seq, double lam, int k) {
  const long total = (long)n * p->M;
  const unsigned gb = (unsigned)((total + kPmThreads - 1) / kPmThreads);
  static const bool sparse = [] {
    const char* e = getenv("GCSLAM_PM_TOPK_SPARSE");
    return !(e && e[0] == '0');
  }();
  // only the first k of each tile are read: a per-tile select + LDS sort replaces the full radix sort
  // (GCSLAM_PM_FULLSORT=1 keeps the full sort, for A/B)
  static const bool full = [] {
    const char* e = getenv("GCSLAM_PM_FULLSORT");
    return e && e[0] == '1';
  }();
  // high key words in registers up to 8 per thread (M <= 8,192; 52 per thread spills at 1024 threads)
  static const bool glob = [] {
    const char* e = getenv("GCSLAM_PM_SELECT_GLOBAL");  // A/B: the global-memory passes
    return e && e[0] == '1';
  }();
  // GCSLAM_PM_SELECT: "radix" (one workgroup, keys read from memory each pass) for A/B; default: the
  // register select up to 8 keys per thread (M <= 8,192), the tree of sorted runs (k_pm_topk) above.
  // Measured at 7 x 50,000 (profiles/r03/pmap): tree 61-73 us, radix ~120 us, and the register select
  // at 98 keys per thread (512 threads, buffer loads, no spill) 186 us -- its LDS histogram atomics
  // on the keys' low-entropy top bits serialise.
  static const int sel = [] {
    const char* e = getenv("GCSLAM_PM_SELECT");
    return e && strcmp(e, "radix") == 0 ? 2 : 0;
  }();
  const bool part = k >= 1 && k <= kSelMax && !full;
  const int G = (p->M + kTopChunk - 1) / kTopChunk;
  const bool reg8 = p->M <= 8 * kPmRed;
  const bool use_tree = part && !glob && sel == 0 && !reg8 && G > 1 && G <= (1 << (kTopMaxLevels - 1));
  // the sparse / dense-shortcut pass runs exactly when k_pm_keys writes its bitmap and counts
  const bool sp = use_tree && sparse && p->M > 8 * kPmRed && p->M <= 32 * kSpWords;
  hipLaunchKernelGGL(k_pm_keys, dim3(gb), dim3(kPmThreads), 0, p->stream, p->st, (const int32_t*)p->d_tiles, n, mode,
                     seq, lam, p->keys, p->vals, sp ? p->other_bm : nullptr, p->below);
  if (part) {
    const uint64_t* kk = (const uint64_t*)p->keys;
    if (use_tree) {
      const size_t need = (size_t)n * G * k;
      if (need > p->run_cap) {
        if (p->run_key) PMCHK(p, hipFree(p->run_key));
        if (p->run_slot) PMCHK(p, hipFree(p->run_slot));
        p->run_key = nullptr;
        p->run_slot = nullptr;
        PMCHK(p, hipMalloc(&p->run_key, need * 8));
        PMCHK(p, hipMalloc(&p->run_slot, need * 4));
        p->run_cap = need;
      }
      if (sp)  // sparse tiles (most map tiles) and empty-rich dense ones: their result directly; the tree the others
        hipLaunchKernelGGL(k_pm_topk_sparse, dim3(n), dim3(kPmRed), 0, p->stream, kk, (const uint32_t*)p->other_bm,
                           p->M, k, mode, p->topk_skip, p->vals, p->below);
      hipLaunchKernelGGL(k_pm_topk, dim3(G, n), dim3(kPmRed), 0, p->stream, kk, p->M, k, G, p->run_key, p->run_slot,
                         p->tickets, p->vals, sp ? (const uint32_t*)p->topk_skip : nullptr);
    } else if (!glob && sel != 2 && reg8)
      hipLaunchKernelGGL((k_pm_select_reg<8, kPmRed>), dim3(n), dim3(kPmRed), 0, p->stream, kk, p->M, k, p->vals);
    else
      hipLaunchKernelGGL(k_pm_select, dim3(n), dim3(kPmRed), 0, p->stream, kk, p->M, k, p->vals);
    PMCHK(p, hipGetLastError());
    return GCS_OK;
  }
  size_t tb = p->temp_bytes;
  PMCHK(p, rocprim::radix_sort_pairs(p->temp, tb, p->keys, p->keys_s, p->vals, p->vals_s, (unsigned)total, 0u, 64u,
                                     p->stream));
  if (n > 1) {
    unsigned bits = 1;
    while ((1u << bits) < (unsigned)n) ++bits;
    hipLaunchKernelGGL(k_pm_segkeys, dim3(gb), dim3(kPmThreads), 0, p->stream, (const uint32_t*)p->vals_s, total, p->M,
                       (uint32_t*)p->keys);
    tb = p->temp_bytes;
    PMCHK(p, rocprim::radix_sort_pairs(p->temp, tb, (uint32_t*)p->keys, p->seg, p->vals_s, p->vals, (unsigned)total, 0u,
                                       bits, p->stream));
  } else {
    PMCHK(p, hipMemcpyAsync(p->vals, p->vals_s, total * 4, hipMemcpyDeviceToDevice, p->stream));
  }
  return GCS_OK;
}

// valid counts of the n listed tiles (host, after a sync)
int count_tiles(gcs_pmap* p, const int32_t* d_tiles, int n, int32_t* count) {
  const int nbt = blocks_per_tile(p->M);
  hipLaunchKernelGGL(k_pm_count, dim3(n, nbt), dim3(kPmRed), 0, p->stream, p->st, d_tiles, (double*)(p->d_small + kPartOff));
  PMCHK(p, hipGetLastError());
  PMCHK(p, hipStreamSynchronize(p->stream));
  const double* h = (const double*)(p->h_small + kPartOff);
  for (int t = 0; t < n; ++t) {
    double c = 0.0;
    for (int b = 0; b < nbt; ++b) c += h[t * nbt + b];
    count[t] = (int32_t)c;
  }
  return GCS_OK;
}

PmRows rows_of(const gcs_pmap_rows* r) {
  PmRows o{};
  o.lam = r->Lambdas;
  o.th = r->thetas;
  o.eta = r->etas;
  o.w = r->weights;
  o.resp = r->responsibilities;
  o.col = r->colors;
  o.valid = r->valid;
  o.src = r->sources;
  o.tpos = r->tile_pos;
  o.slots = r->slots;
  o.n = r->n;
  return o;
}
}  // namespace

extern "C" {

int gcs_pmap_create(int32_t m_tile, int32_t max_tiles, int32_t n_lobes, int32_t max_merge, int32_t device,
                    gcs_pmap** out) {
  if (!out || m_tile < 1 || max_tiles < 1 || n_lobes != kNL || max_merge < 0) return GCS_ERR_ARG;
  if ((long)m_tile * max_tiles >= (1L << 31)) return GCS_ERR_ARG;
  if ((size_t)max_tiles * kMaxBlocksPerTile * 4 * sizeof(double) > kSmall - kPartOff) return GCS_ERR_ARG;
  gcs_pmap* p = new gcs_pmap();
  p->device = device;
  p->M = m_tile;
  p->T = max_tiles;
  p->nl = n_lobes;
  p->max_merge = std::min(max_merge, m_tile);
  auto bad = [&](hipError_t e) { return e != hipSuccess; };
  auto fail = [&]() {
    gcs_pmap_destroy(p);
    return GCS_ERR_HIP;
  };
  if (bad(hipSetDevice(device)) || bad(hipStreamCreateWithFlags(&p->own, hipStreamNonBlocking))) return fail();
  p->stream = p->own;
  for (int f = 0; f < GCS_PM_NFIELDS; ++f)
    if (bad(hipMalloc(&p->fields[f], field_elems(p, f) * kFieldBytes[f] * (size_t)max_tiles))) return fail();
  PmStore& s = p->st;
  s.lam = (double*)p->fields[GCS_PM_LAMBDAS];
  s.th = (double*)p->fields[GCS_PM_THETAS];
  s.eta = (double*)p->fields[GCS_PM_ETAS];
  s.w = (double*)p->fields[GCS_PM_WEIGHTS];
  s.ts = (double*)p->fields[GCS_PM_TIMESTAMPS];
  s.cts = (double*)p->fields[GCS_PM_CREATED];
  s.col = (double*)p->fields[GCS_PM_COLORS];
  s.cam = (double*)p->fields[GCS_PM_CAM_MASS];
  s.lid = (double*)p->fields[GCS_PM_LIDAR_MASS];
  s.acc = (double*)p->fields[GCS_PM_RGB_ACCUM];
  s.den = (double*)p->fields[GCS_PM_RGB_DENOM];
  s.rgb = (double*)p->fields[GCS_PM_RGB];
  s.lsup = (int64_t*)p->fields[GCS_PM_LAST_SUPPORTED];
  s.lupd = (int64_t*)p->fields[GCS_PM_LAST_UPDATE];
  s.ids = (int64_t*)p->fields[GCS_PM_IDS];
  s.valid = (uint8_t*)p->fields[GCS_PM_VALID];
  s.M = m_tile;
  s.nl = n_lobes;
  const size_t tot = (size_t)m_tile * max_tiles;
  if (bad(hipMalloc(&p->keys, tot * 8)) || bad(hipMalloc(&p->keys_s, tot * 8)) || bad(hipMalloc(&p->vals, tot * 4)) ||
      bad(hipMalloc(&p->vals_s, tot * 4)) || bad(hipMalloc(&p->seg, tot * 4)) ||
      bad(hipMalloc(&p->d_tiles, max_tiles * 4)) || bad(hipMalloc(&p->d_tids, max_tiles * 8)) ||
      bad(hipMalloc(&p->mark, (size_t)m_tile * 4)) || bad(hipMalloc(&p->dcnt, 4)) ||
      bad(hipMalloc(&p->bcnt, kMaxFuseBlocks * 4)) ||
      bad(hipMemset(p->bcnt, 0, kMaxFuseBlocks * 4)) ||  // once: the last counting block re-zeroes
      bad(hipMalloc(&p->bticket, 4)) || bad(hipMemset(p->bticket, 0, 4)) ||
      bad(hipMalloc(&p->tickets, (size_t)max_tiles * kTopMaxLevels * kTopNodes * 4)) ||
      bad(hipMemset(p->tickets, 0, (size_t)max_tiles * kTopMaxLevels * kTopNodes * 4)) ||
      bad(hipMalloc(&p->topk_skip, (size_t)max_tiles * 4)) || bad(hipMalloc(&p->below, (size_t)max_tiles * 4)) ||
      bad(hipMemset(p->below, 0, (size_t)max_tiles * 4)) ||
      bad(hipMalloc(&p->other_bm, ((size_t)max_tiles * m_tile / 32 + 4) * 4)) ||
      bad(hipMemset(p->other_bm, 0, ((size_t)max_tiles * m_tile / 32 + 4) * 4)) ||
      bad(hipStreamSynchronize(nullptr)) ||  // (null-stream clears: done before p->stream's kernels)
      bad(hipHostMalloc((void**)&p->h_small, kSmall, hipHostMallocMapped)) ||
      bad(hipHostGetDevicePointer((void**)&p->d_small, p->h_small, 0)))
    return fail();
  size_t tb = 0, tb2 = 0;
  if (bad(rocprim::radix_sort_pairs(nullptr, tb, p->keys, p->keys_s, p->vals, p->vals_s, (unsigned)tot, 0u, 64u,
                                    p->stream)) ||
      bad(rocprim::radix_sort_pairs(nullptr, tb2, (uint32_t*)p->keys, p->seg, p->vals_s, p->vals, (unsigned)tot, 0u,
                                    16u, p->stream)) ||
      bad(hipMalloc(&p->temp, std::max<size_t>(std::max(tb, tb2), 16))))
    return fail();
  p->temp_bytes = std::max<size_t>(std::max(tb, tb2), 16);
  if (p->max_merge >= 2) {
    const long P = (long)p->max_merge * (p->max_merge - 1) / 2;
    if (bad(hipMalloc(&p->mmu, (size_t)p->max_merge * 3 * 8)) || bad(hipMalloc(&p->msig, (size_t)p->max_merge * 9 * 8)) ||
        bad(hipMalloc(&p->mdet, (size_t)p->max_merge * 8)) || bad(hipMalloc(&p->mdist, (size_t)P * 8)) ||
        bad(hipMalloc(&p->mpd, kMergeBlocks * 8)) || bad(hipMalloc(&p->mpp, kMergeBlocks * 8)) ||
        bad(hipMalloc(&p->mused, p->max_merge)) || bad(hipMalloc(&p->msel, 2 * 1024 * 4)) ||
        bad(hipMalloc(&p->mnsel, 4)))
      return fail();
  }
  for (int t = 0; t < max_tiles; ++t)
    hipLaunchKernelGGL(k_pm_clear, dim3((m_tile + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream, p->st, t);
  if (bad(hipStreamSynchronize(p->stream))) return fail();
  *out = p;
  return GCS_OK;
}

int gcs_pmap_destroy(gcs_pmap* p) {
  if (!p) return GCS_ERR_ARG;
  (void)hipSetDevice(p->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  for (void* f : p->fields)
    if (f) (void)hipFree(f);
  void* bufs[] = {p->keys, p->keys_s, p->vals, p->vals_s, p->seg, p->d_tiles, p->d_tids, p->temp, p->fk, p->fk_s,
                  p->fv, p->fv_s, p->ftemp, p->mark, p->dcnt, p->bmark, p->bcnt, p->bticket, p->mmu, p->msig, p->mdet, p->mdist, p->mpd, p->mpp, p->mused,
                  p->msel, p->mnsel, p->ub, p->run_key, p->run_slot, p->tickets, p->fterm, p->flen, p->topk_skip, p->other_bm, p->below};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (p->h_small) (void)hipHostFree(p->h_small);
  if (p->own) (void)hipStreamDestroy(p->own);
  delete p;
  return GCS_OK;
}

const char* gcs_pmap_last_error(const gcs_pmap* p) { return p ? p->err.c_str() : "null map"; }

int gcs_pmap_set_stream(gcs_pmap* p, void* stream) {
  if (!p) return GCS_ERR_ARG;
  hipStream_t ns = stream ? (hipStream_t)stream : p->own;
  if (ns == p->stream) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  PMCHK(p, hipStreamSynchronize(p->stream));
  p->stream = ns;
  return GCS_OK;
}

int gcs_pmap_clear_tile(gcs_pmap* p, int32_t tile) {
  if (int rc = gcs::live::pmap_clear_tile_launch(p, tile)) return rc;
  PMCHK(p, hipStreamSynchronize(p->stream));
  return GCS_OK;
}

int gcs_pmap_read(gcs_pmap* p, int32_t tile, int32_t field, void* host) {
  if (!p || !host || field < 0 || field >= GCS_PM_NFIELDS) return GCS_ERR_ARG;
  if (tile < 0 || tile >= p->T) return pm_fail(p, GCS_ERR_ARG, "tile storage index out of range");
  PMCHK(p, hipSetDevice(p->device));
  const size_t b = field_elems(p, field) * kFieldBytes[field];
  PMCHK(p, hipMemcpyAsync(host, (char*)p->fields[field] + b * tile, b, hipMemcpyDeviceToHost, p->stream));
  PMCHK(p, hipStreamSynchronize(p->stream));
  return GCS_OK;
}

int gcs_pmap_write(gcs_pmap* p, int32_t tile, int32_t field, const void* host) {
  if (!p || !host || field < 0 || field >= GCS_PM_NFIELDS) return GCS_ERR_ARG;
  if (tile < 0 || tile >= p->T) return pm_fail(p, GCS_ERR_ARG, "tile storage index out of range");
  PMCHK(p, hipSetDevice(p->device));
  const size_t b = field_elems(p, field) * kFieldBytes[field];
  PMCHK(p, hipMemcpyAsync((char*)p->fields[field] + b * tile, host, b, hipMemcpyHostToDevice, p->stream));
  PMCHK(p, hipStreamSynchronize(p->stream));
  return GCS_OK;
}

// device-to-device copy of whole tiles (every field), on dst's stream: a hypothesis that must not
// update the node's map works on copies of the tiles its scan touches (same tile size and lobes)
int gcs_pmap_copy_tiles(gcs_pmap* dst, const int32_t* dst_tiles, const gcs_pmap* src, const int32_t* src_tiles,
                        int32_t n) {
  if (!dst || !src || n < 0 || (n > 0 && (!dst_tiles || !src_tiles))) return GCS_ERR_ARG;
  if (dst->M != src->M || dst->nl != src->nl || dst->device != src->device)
    return pm_fail(dst, GCS_ERR_ARG, "copy_tiles: maps of different tile size, lobe count or device");
  for (int i = 0; i < n; ++i)
    if (dst_tiles[i] < 0 || dst_tiles[i] >= dst->T || src_tiles[i] < 0 || src_tiles[i] >= src->T)
      return pm_fail(dst, GCS_ERR_ARG, "tile storage index out of range");
  PMCHK(dst, hipSetDevice(dst->device));
  if (src->stream != dst->stream) PMCHK(dst, hipStreamSynchronize(src->stream));  // src's pending updates
  for (int i = 0; i < n; ++i)
    for (int f = 0; f < GCS_PM_NFIELDS; ++f) {
      const size_t b = field_elems(dst, f) * kFieldBytes[f];
      PMCHK(dst, hipMemcpyAsync((char*)dst->fields[f] + b * dst_tiles[i], (const char*)src->fields[f] + b * src_tiles[i],
                                b, hipMemcpyDeviceToDevice, dst->stream));
    }
  PMCHK(dst, hipStreamSynchronize(dst->stream));
  return GCS_OK;
}

int gcs_pmap_extract_view(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, int32_t m_view,
                          double eps_lift, double eps_mass, gcs_pmap_view* o) {
  if (int rc = gcs::live::pmap_view_launch(p, tiles, tile_ids, n, m_view, eps_lift, eps_mass, o)) return rc;
  if (n > 0) PMCHK(p, hipStreamSynchronize(p->stream));
  return GCS_OK;
}
}  // extern "C"

namespace gcs {
namespace live {
int pmap_bind_stream(gcs_pmap* p, void* s) {
  if ((hipStream_t)s == p->stream) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  PMCHK(p, hipStreamSynchronize(p->stream));
  p->stream = (hipStream_t)s;
  return GCS_OK;
}

int pmap_clear_tile_launch(gcs_pmap* p, int32_t tile) {
  if (!p) return GCS_ERR_ARG;
  if (tile < 0 || tile >= p->T) return pm_fail(p, GCS_ERR_ARG, "tile storage index out of range");
  PMCHK(p, hipSetDevice(p->device));
  hipLaunchKernelGGL(k_pm_clear, dim3((p->M + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream, p->st,
                     tile);
  PMCHK(p, hipGetLastError());
  return GCS_OK;
}

int pmap_copy_staged_ids(gcs_pmap* p, int64_t* dst, int32_t n) {
  if (n > 0) PMCHK(p, hipMemcpyAsync(dst, p->d_tids, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToDevice, p->stream));
  return GCS_OK;
}

int pmap_view_launch(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, int32_t m_view,
                     double eps_lift, double eps_mass, gcs_pmap_view* o) {
  if (!p || !o || !tile_ids) return GCS_ERR_ARG;
  if (m_view <= 0) return pm_fail(p, GCS_ERR_ARG, "extract_atlas_map_view: m_tile_view must be > 0");
  if (m_view > p->M) return pm_fail(p, GCS_ERR_ARG, "m_tile_view exceeds the tile size");
  if (int rc = check_tiles(p, tiles, n, true)) return rc;
  if (n == 0) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  if (n <= kPmArgTiles) {  // the tile list and ids as kernel arguments (no host-to-device copies)
    PmTileArgs ta{};
    ta.n = n;
    for (int t = 0; t < n; ++t) {
      ta.tiles[t] = tiles[t];
      ta.ids[t] = tile_ids[t];
    }
    hipLaunchKernelGGL(k_pm_stage_tiles, dim3(1), dim3(kPmArgTiles), 0, p->stream, ta, p->d_tiles, p->d_tids);
  } else {
    if (int rc = upload_tiles(p, tiles, n)) return rc;
    PMCHK(p, hipMemcpyAsync(p->d_tids, tile_ids, n * sizeof(int64_t), hipMemcpyHostToDevice, p->stream));
  }
  if (int rc = sort_tiles(p, n, 0, 0, 0.0, m_view)) return rc;
  PmViewOut v{o->positions, o->covariances, o->directions, o->kappas, o->weights, o->etas, o->colors,
              o->primitive_ids, o->last_supported_scan_seq, o->candidate_tile_ids, o->valid_mask,
              o->candidate_slots};
  hipLaunchKernelGGL(k_pm_view, dim3((n * m_view + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream,
                     p->st, (const int32_t*)p->d_tiles, (const int64_t*)p->d_tids, n, m_view,
                     (const uint32_t*)p->vals, eps_lift, eps_mass, v);
  PMCHK(p, hipGetLastError());
  return GCS_OK;
}
}  // namespace live
}  // namespace gcs

extern "C" {

int gcs_pmap_insert_masked(gcs_pmap* p, const int32_t* tiles, int32_t n, int32_t K, const gcs_pmap_rows* rows,
                           double timestamp, int64_t scan_seq, double lam, int64_t next_global_id, int64_t* new_ids,
                           int32_t* n_inserted, int32_t* count) {
  if (!p || !rows || !n_inserted || !count) return GCS_ERR_ARG;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  if (K < 0 || K > p->M) return pm_fail(p, GCS_ERR_ARG, "K proposals exceed the tile size");
  if (rows->n != n * K) return pm_fail(p, GCS_ERR_ARG, "rows.n must be n_tiles x K");
  if (n * K > 0 && (!rows->Lambdas || !rows->thetas || !rows->etas || !rows->weights || !rows->valid))
    return pm_fail(p, GCS_ERR_ARG, "null proposal array");
  if (n == 0) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  if (int rc = upload_tiles(p, tiles, n)) return rc;
  int32_t* d_ins = (int32_t*)p->d_small;
  if (K > 0) {
    if (int rc = sort_tiles(p, n, 1, scan_seq, lam, K)) return rc;
    hipLaunchKernelGGL(k_pm_insert, dim3(n), dim3(kPmThreads), 0, p->stream, p->st, (const int32_t*)p->d_tiles, n, K,
                       (const uint32_t*)p->vals, rows_of(rows), timestamp, (long long)scan_seq,
                       (long long)next_global_id, new_ids, d_ins);
  } else {
    PMCHK(p, hipMemsetAsync(d_ins, 0, n * sizeof(int32_t), p->stream));
  }
  if (int rc = count_tiles(p, (const int32_t*)p->d_tiles, n, count)) return rc;
  memcpy(n_inserted, p->h_small, n * sizeof(int32_t));
  return GCS_OK;
}

namespace {
int fuse_impl(gcs_pmap* p, const int32_t* tiles, int32_t n, const gcs_pmap_rows* rows, double timestamp,
              int64_t scan_seq, double eps_mass, int32_t* n_fused, bool rebuild_rgb);
}
int gcs_pmap_fuse(gcs_pmap* p, const int32_t* tiles, int32_t n, const gcs_pmap_rows* rows, double timestamp,
                  int64_t scan_seq, double eps_mass, int32_t* n_fused) {
  return fuse_impl(p, tiles, n, rows, timestamp, scan_seq, eps_mass, n_fused, true);
}
}  // extern "C"

namespace {
// rebuild_rgb = false: a later call on the same tiles rebuilds it (rgb is a function of the slot's
// accumulators alone, so only the last rebuild of a sequence is observable)
int fuse_impl(gcs_pmap* p, const int32_t* tiles, int32_t n, const gcs_pmap_rows* rows, double timestamp,
              int64_t scan_seq, double eps_mass, int32_t* n_fused, bool rebuild_rgb) {
  if (!p || !rows || !n_fused) return GCS_ERR_ARG;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  const int R = rows->n;
  if (R < 0) return GCS_ERR_ARG;
  *n_fused = 0;
  if (R == 0 || n == 0) return GCS_OK;  // K == 0: the reference's exact no-op
  if (!rows->Lambdas || !rows->thetas || !rows->etas || !rows->weights || !rows->responsibilities ||
      !rows->tile_pos || !rows->slots)
    return pm_fail(p, GCS_ERR_ARG, "null contribution array");
  PMCHK(p, hipSetDevice(p->device));
  if (R > p->frows) {
    for (void* b : {(void*)p->fk, (void*)p->fk_s, (void*)p->fv, (void*)p->fv_s, p->ftemp})
      if (b) (void)hipFree(b);
    p->fk = p->fk_s = p->fv = p->fv_s = nullptr;
    p->ftemp = nullptr;
    const int cap = std::max(R, 16384);
    PMCHK(p, hipMalloc(&p->fk, cap * 4));
    PMCHK(p, hipMalloc(&p->fk_s, cap * 4));
    PMCHK(p, hipMalloc(&p->fv, cap * 4));
    PMCHK(p, hipMalloc(&p->fv_s, cap * 4));
    size_t tb = 0;
    PMCHK(p, rocprim::radix_sort_pairs(nullptr, tb, p->fk, p->fk_s, p->fv, p->fv_s, (unsigned)cap, 0u, 32u, p->stream));
    p->ftemp_bytes = std::max<size_t>(tb, 16);
    PMCHK(p, hipMalloc(&p->ftemp, p->ftemp_bytes));
    p->frows = cap;
  }
  if (int rc = upload_tiles(p, tiles, n)) return rc;
  uint32_t* d_err = (uint32_t*)(p->d_small + 8192);
  uint32_t* d_nf = p->dcnt;
  *(uint32_t*)(p->h_small + 8192) = 0u;
  PMCHK(p, hipMemsetAsync(p->dcnt, 0, 4, p->stream));
  const PmRows r = rows_of(rows);
  const int rb = (R + kPmThreads - 1) / kPmThreads;
  hipLaunchKernelGGL(k_pm_fuse_keys, dim3(rb), dim3(kPmThreads), 0, p->stream, r, n, p->M, p->fk, p->fv, d_err);
  size_t tb = p->ftemp_bytes;
  PMCHK(p, rocprim::radix_sort_pairs(p->ftemp, tb, p->fk, p->fk_s, p->fv, p->fv_s, (unsigned)R, 0u, 32u, p->stream));
  hipLaunchKernelGGL(k_pm_fuse_apply, dim3(rb), dim3(kPmThreads), 0, p->stream, p->st, (const int32_t*)p->d_tiles, r,
                     (const uint32_t*)p->fk_s, (const uint32_t*)p->fv_s, (long long)scan_seq);
  const long tm = (long)n * p->M;
  if (rebuild_rgb)
    hipLaunchKernelGGL(k_pm_fuse_rgb, dim3((unsigned)((tm + kPmThreads - 1) / kPmThreads)), dim3(kPmThreads), 0,
                       p->stream, p->st, (const int32_t*)p->d_tiles, n, eps_mass);
  PMCHK(p, hipMemsetAsync(p->mark, 0, (size_t)p->M * 4, p->stream));
  const long tr = (long)n * R;
  hipLaunchKernelGGL(k_pm_fuse_ts, dim3((unsigned)((tr + kPmThreads - 1) / kPmThreads)), dim3(kPmThreads), 0,
                     p->stream, p->st, (const int32_t*)p->d_tiles, n, r, timestamp, p->mark);
  hipLaunchKernelGGL(k_pm_count_marks, dim3((p->M + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream,
                     (const uint32_t*)p->mark, p->M, d_nf);
  PMCHK(p, hipMemcpyAsync(p->h_small + 8200, p->dcnt, 4, hipMemcpyDeviceToHost, p->stream));
  PMCHK(p, hipGetLastError());
  PMCHK(p, hipStreamSynchronize(p->stream));
  if (*(uint32_t*)(p->h_small + 8192)) return pm_fail(p, GCS_ERR_ARG, "target slot out of range (rows skipped)");
  *n_fused = (int32_t)*(uint32_t*)(p->h_small + 8200);
  return GCS_OK;
}

// Step 12b's fuse: nb association blocks of rpb rows each (rows block-major), every listed tile
// (already uploaded to d_tiles), in one sort + one apply (no host syncs between the blocks);
// nf (host, nb): each block's unique target slots.  One sync at the end.
// nf == nullptr: no sync -- the counts go to the mapped buffer (h_small + 9216) and the caller
// checks the slot-range flag (h_small + 8192) after its own sync
int fuse_blocks(gcs_pmap* p, int32_t n, const gcs_pmap_rows* rows, int nb, int rpb, double timestamp, int64_t scan_seq,
                double eps_mass, int32_t* nf) {
  const int R = rows->n;
  if (nb > kMaxFuseBlocks) return pm_fail(p, GCS_ERR_ARG, "map update: more than 256 association blocks");
  if ((double)n * p->M * nb >= 4294967295.0) return pm_fail(p, GCS_ERR_ARG, "map update: fuse key space");
  if (R > p->frows) {
    for (void* b : {(void*)p->fk, (void*)p->fk_s, (void*)p->fv, (void*)p->fv_s, p->ftemp})
      if (b) (void)hipFree(b);
    p->fk = p->fk_s = p->fv = p->fv_s = nullptr;
    p->ftemp = nullptr;
    const int cap = std::max(R, 16384);
    PMCHK(p, hipMalloc(&p->fk, cap * 4));
    PMCHK(p, hipMalloc(&p->fk_s, cap * 4));
    PMCHK(p, hipMalloc(&p->fv, cap * 4));
    PMCHK(p, hipMalloc(&p->fv_s, cap * 4));
    size_t tb = 0;
    PMCHK(p, rocprim::radix_sort_pairs(nullptr, tb, p->fk, p->fk_s, p->fv, p->fv_s, (unsigned)cap, 0u, 32u, p->stream));
    // (also k_ss_block's runs: up to kSsWideMax rows)
    p->ftemp_bytes = std::max<size_t>(tb, (size_t)std::min(((cap + kSsRun - 1) / kSsRun) * kSsRun, kSsWideMax) * 8);
    PMCHK(p, hipMalloc(&p->ftemp, p->ftemp_bytes));
    p->frows = cap;
  }
  const size_t mb = (size_t)nb * p->M;
  if (mb > p->bmark_bytes) {
    if (p->bmark) PMCHK(p, hipFree(p->bmark));
    p->bmark = nullptr;
    PMCHK(p, hipMalloc(&p->bmark, mb));
    PMCHK(p, hipMemsetAsync(p->bmark, 0, mb, p->stream));  // once: k_pm_count_marks_blocks re-zeroes
    p->bmark_bytes = mb;
  }
  uint32_t* d_err = (uint32_t*)(p->d_small + 8192);
  *(uint32_t*)(p->h_small + 8192) = 0u;
  const PmRows r = rows_of(rows);
  const int rb = (R + kPmThreads - 1) / kPmThreads;
  // GCSLAM_FUSE_SORT_BITS=1: keys below n M nb, the skipped rows' key 2^bits - 1 above them, sorted on
  // the low bits only -- one onesweep pass fewer on the device, but measured ~35 us more host time per
  // map update in the radix sort's dispatch (live path, profiles/r05/live): off by default
  static const bool sig_bits = [] {
    const char* e = getenv("GCSLAM_FUSE_SORT_BITS");
    return e && atoi(e) != 0;
  }();
  unsigned bits = 32;
  if (sig_bits) {
    bits = 1;
    while (bits < 32 && ((double)(1ull << bits)) < (double)n * p->M * nb + 1.0) ++bits;
  }
  const uint32_t nokey = bits >= 32 ? kNoKey : (uint32_t)((1ull << bits) - 1ull);
  hipLaunchKernelGGL(k_pm_fuse_keys_blocks, dim3(rb), dim3(kPmThreads), 0, p->stream, p->st,
                     (const int32_t*)p->d_tiles, timestamp, r, n, p->M, nb, rpb, p->fk, p->fv, p->bmark, d_err, nokey);
  static const bool small_sort = [] {
    const char* e = getenv("GCSLAM_FUSE_SMALLSORT");
    return GCS_FUSE_SMALLSORT && !(e && e[0] == '0');
  }();
  if (small_sort && R <= kSsWideMax && p->ftemp_bytes >= (size_t)((R + kSsRun - 1) / kSsRun) * kSsRun * 8) {
    const int nrun = (R + kSsRun - 1) / kSsRun;
    hipLaunchKernelGGL(k_ss_block, dim3(nrun), dim3(512), 0, p->stream, (const uint32_t*)p->fk, (const uint32_t*)p->fv, R,
                       (uint64_t*)p->ftemp);
    hipLaunchKernelGGL(k_ss_merge, dim3(nrun), dim3(kSsRun), 0, p->stream, (const uint64_t*)p->ftemp, R, nrun, p->fk_s,
                       p->fv_s);
  } else {
    size_t tb = p->ftemp_bytes;
    PMCHK(p, rocprim::radix_sort_pairs(p->ftemp, tb, p->fk, p->fk_s, p->fv, p->fv_s, (unsigned)R, 0u, bits, p->stream));
  }
  if ((size_t)R * kFT > p->fterm_n) {
    if (p->fterm) PMCHK(p, hipFree(p->fterm));
    if (p->flen) PMCHK(p, hipFree(p->flen));
    p->fterm = nullptr;
    p->flen = nullptr;
    p->fterm_n = (size_t)std::max(R, 16384) * kFT;
    PMCHK(p, hipMalloc(&p->fterm, p->fterm_n * sizeof(double)));
    PMCHK(p, hipMalloc(&p->flen, (p->fterm_n / kFT) * sizeof(int)));
  }
  if (GCS_FUSE_RUNS)
    hipLaunchKernelGGL(k_pm_fuse_runs, dim3(rb), dim3(kPmThreads), 0, p->stream, r, (const uint32_t*)p->fk_s,
                       (const uint32_t*)p->fv_s, p->fterm, p->flen, nokey);
  else
    hipLaunchKernelGGL(k_pm_fuse_chunks, dim3(rb), dim3(kPmThreads), 0, p->stream, r, (const uint32_t*)p->fk_s,
                       (const uint32_t*)p->fv_s, p->fterm, p->flen, nokey);
  hipLaunchKernelGGL(k_pm_fuse_apply_blocks, dim3(rb), dim3(kPmThreads), 0, p->stream, p->st, (const int32_t*)p->d_tiles,
                     r, (const uint32_t*)p->fk_s, (const uint32_t*)p->fv_s, nb, (long long)scan_seq,
                     (const double*)p->fterm, (const int*)p->flen, nokey);
  const long tm = (long)n * p->M;
  hipLaunchKernelGGL(k_pm_fuse_rgb, dim3((unsigned)((tm + kPmThreads - 1) / kPmThreads)), dim3(kPmThreads), 0,
                     p->stream, p->st, (const int32_t*)p->d_tiles, n, eps_mass);
  hipLaunchKernelGGL(k_pm_count_marks_blocks, dim3(std::min(32, (p->M + kPmThreads - 1) / kPmThreads), nb),
                     dim3(kPmThreads), 0, p->stream, p->bmark, p->M, p->bcnt, p->bticket, nb,
                     (uint32_t*)(p->d_small + 9216));
  PMCHK(p, hipGetLastError());
  if (!nf) return GCS_OK;
  PMCHK(p, hipStreamSynchronize(p->stream));
  if (*(uint32_t*)(p->h_small + 8192)) return pm_fail(p, GCS_ERR_ARG, "target slot out of range (rows skipped)");
  for (int b = 0; b < nb; ++b) nf[b] = (int32_t)((const uint32_t*)(p->h_small + 9216))[b];
  return GCS_OK;
}
}  // namespace

extern "C" {

int gcs_pmap_cull(gcs_pmap* p, const int32_t* tiles, int32_t n, double thr, int32_t* n_culled, double* mass_dropped,
                  double* weight_sum, int32_t* count) {
  if (!p || !n_culled || !mass_dropped || !weight_sum || !count) return GCS_ERR_ARG;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  if (n == 0) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  if (int rc = upload_tiles(p, tiles, n)) return rc;
  const int nbt = blocks_per_tile(p->M);
  hipLaunchKernelGGL(k_pm_cull, dim3(n, nbt), dim3(kPmRed), 0, p->stream, p->st, (const int32_t*)p->d_tiles, thr,
                     (double*)(p->d_small + kPartOff), 0, 1.0);
  PMCHK(p, hipGetLastError());
  PMCHK(p, hipStreamSynchronize(p->stream));
  const double* h = (const double*)(p->h_small + kPartOff);
  for (int t = 0; t < n; ++t) {  // block partials folded in block order
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = 0; b < nbt; ++b)
      for (int k = 0; k < 4; ++k) a[k] += h[4 * (t * nbt + b) + k];
    n_culled[t] = (int32_t)a[0];
    mass_dropped[t] = a[1];
    weight_sum[t] = a[2];
    count[t] = (int32_t)a[3];
  }
  return GCS_OK;
}

int gcs_pmap_forget(gcs_pmap* p, const int32_t* tiles, int32_t n, double gamma) {
  if (!p) return GCS_ERR_ARG;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  if (n == 0) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  if (int rc = upload_tiles(p, tiles, n)) return rc;
  const long tm = (long)n * p->M;
  hipLaunchKernelGGL(k_pm_forget, dim3((unsigned)((tm + kPmThreads - 1) / kPmThreads)), dim3(kPmThreads), 0,
                     p->stream, p->st, (const int32_t*)p->d_tiles, n, gamma);
  PMCHK(p, hipGetLastError());
  PMCHK(p, hipStreamSynchronize(p->stream));
  return GCS_OK;
}

int gcs_pmap_recency_inflate(gcs_pmap* p, const int32_t* tiles, int32_t n, int64_t scan_seq, double lam,
                             double min_scale, double* stats) {
  if (!p || !stats) return GCS_ERR_ARG;
  if (int rc = gcs::live::pmap_recency_launch(p, tiles, n, scan_seq, lam, min_scale)) return rc;
  if (n > 0) PMCHK(p, hipStreamSynchronize(p->stream));
  gcs::live::pmap_recency_collect(p, n, stats);
  return GCS_OK;
}
}  // extern "C"

namespace gcs {
namespace live {
int pmap_recency_launch(gcs_pmap* p, const int32_t* tiles, int32_t n, int64_t scan_seq, double lam,
                        double min_scale) {
  if (!p) return GCS_ERR_ARG;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  if (n == 0) return GCS_OK;
  const int nbt = blocks_per_tile(p->M);
  if ((size_t)n * nbt * 3 * sizeof(double) > kSmall - kRecOff)
    return pm_fail(p, GCS_ERR_ARG, "recency inflation: partials exceed the mapped buffer");
  PMCHK(p, hipSetDevice(p->device));
  if (int rc = upload_tiles(p, tiles, n)) return rc;
  hipLaunchKernelGGL(k_pm_recency, dim3(n, nbt), dim3(kPmRed), 0, p->stream, p->st, (const int32_t*)p->d_tiles,
                     (long long)scan_seq, lam, min_scale, (double*)(p->d_small + kRecOff));
  PMCHK(p, hipGetLastError());
  return GCS_OK;
}

void pmap_recency_collect(gcs_pmap* p, int32_t n, double* stats) {
  stats[0] = stats[1] = stats[2] = 0.0;
  const int nbt = blocks_per_tile(p->M);
  const double* h = (const double*)(p->h_small + kRecOff);
  for (int t = 0; t < n; ++t) {  // per tile (block partials in order), then the reference's sums over tiles
    double a[3] = {0.0, 0.0, 0.0};
    for (int b = 0; b < nbt; ++b)
      for (int k = 0; k < 3; ++k) a[k] += h[3 * (t * nbt + b) + k];
    for (int k = 0; k < 3; ++k) stats[k] += a[k];
  }
}
}  // namespace live
}  // namespace gcs

extern "C" {

int gcs_pmap_merge_reduce(gcs_pmap* p, int32_t tile, double thr, int32_t max_pairs, double eps_psd, double eps_lift,
                          int32_t* n_merged, int32_t* pairs, int32_t* count) {
  if (!p || !n_merged || !count || (max_pairs > 0 && !pairs)) return GCS_ERR_ARG;
  if (tile < 0 || tile >= p->T) return pm_fail(p, GCS_ERR_ARG, "tile storage index out of range");
  if (p->M > p->max_merge) return pm_fail(p, GCS_ERR_ARG, "tile larger than the context's max_merge");
  if (max_pairs > 1024) return pm_fail(p, GCS_ERR_ARG, "max_pairs above 1024");
  *n_merged = 0;
  PMCHK(p, hipSetDevice(p->device));
  const int32_t tl[1] = {tile};
  if (int rc = upload_tiles(p, tl, 1)) return rc;
  const int M = p->M;
  const long P = (long)M * (M - 1) / 2;
  if (max_pairs > 0 && P > 0) {
    hipLaunchKernelGGL(k_pm_merge_prep, dim3((M + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream,
                       p->st, tile, eps_lift, p->mmu, p->msig, p->mdet);
    hipLaunchKernelGGL(k_pm_merge_dist, dim3((unsigned)((P + kPmThreads - 1) / kPmThreads)), dim3(kPmThreads), 0,
                       p->stream, p->st, tile, P, eps_lift, (const double*)p->mmu, (const double*)p->msig,
                       (const double*)p->mdet, p->mdist);
    PMCHK(p, hipMemsetAsync(p->mused, 0, M, p->stream));
    PMCHK(p, hipMemsetAsync(p->mnsel, 0, 4, p->stream));
    const int nb = (int)std::min<long>(kMergeBlocks, (P + kPmThreads - 1) / kPmThreads);
    for (int k = 0; k < max_pairs; ++k) {
      hipLaunchKernelGGL(k_pm_merge_min, dim3(nb), dim3(kPmThreads), 0, p->stream, p->st, P, (const double*)p->mdist,
                         thr, (const uint8_t*)p->mused, p->mpd, p->mpp);
      hipLaunchKernelGGL(k_pm_merge_pick, dim3(1), dim3(64), 0, p->stream, M, (const double*)p->mpd,
                         (const long long*)p->mpp, nb, p->mused, p->msel, p->mnsel);
    }
    hipLaunchKernelGGL(k_pm_merge_apply, dim3(1), dim3(1024), 0, p->stream, p->st, tile, (const int32_t*)p->msel,
                       (const int32_t*)p->mnsel, (const double*)p->mmu, (const double*)p->msig, eps_psd);
    PMCHK(p, hipMemcpyAsync(n_merged, p->mnsel, 4, hipMemcpyDeviceToHost, p->stream));
    PMCHK(p, hipMemcpyAsync(pairs, p->msel, 2 * max_pairs * 4, hipMemcpyDeviceToHost, p->stream));
  }
  return count_tiles(p, (const int32_t*)p->d_tiles, 1, count);
}

int gcs_pmap_map_update(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, const double* z_t6,
                        double timestamp, int64_t scan_seq, int64_t* next_global_id,
                        const gcs_pmap_update_config* cfg, const gcs_pmap_update_inputs* in,
                        gcs_pmap_update_stats* st, int32_t* counts) {
  if (!p || !next_global_id || !st || !counts) return GCS_ERR_ARG;
  memset(st, 0, sizeof(*st));
  if (int rc = gcs::live::pmap_update_launch(p, tiles, tile_ids, n, z_t6, timestamp, scan_seq, *next_global_id, cfg,
                                             in))
    return rc;
  return gcs::live::pmap_update_collect(p, next_global_id, st, counts);
}
}  // extern "C"

namespace gcs {
namespace live {
int pmap_update_launch(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, const double* z_t6,
                       double timestamp, int64_t scan_seq, int64_t next_global_id, const gcs_pmap_update_config* cfg,
                       const gcs_pmap_update_inputs* in) {
  if (!p || !z_t6 || !cfg || !in || !tile_ids) return GCS_ERR_ARG;
  p->pend.on = false;
  if (int rc = check_tiles(p, tiles, n, false)) return rc;
  if (in->n_total < 1 || in->k_assoc < 1 || !in->Lambdas || !in->thetas || !in->etas || !in->weights || !in->valid ||
      !in->responsibilities || !in->candidate_tile_ids || !in->candidate_slots || !in->row_masses)
    return pm_fail(p, GCS_ERR_ARG, "map update: missing measurement or association array");
  if (cfg->block_size < 1 || cfg->k_insert_tile < 0 || cfg->k_insert_tile > kPropMaxIns || in->n_lobes != p->nl)
    return pm_fail(p, GCS_ERR_ARG, "map update: bad block size, insert budget (<= 1024) or lobe count");
  if (in->n_total > kPropLds) return pm_fail(p, GCS_ERR_ARG, "map update: more than 2048 measurement rows");
  p->pend.n = n;
  p->pend.next_id = next_global_id;
  p->pend.cfg = *cfg;
  p->pend.tiles.assign(tiles, tiles + n);
  if (n == 0) {
    p->pend.on = true;
    return GCS_OK;
  }
  PMCHK(p, hipSetDevice(p->device));
  PmWorld W{};
  so3_exp(z_t6 + 3, W.R);
  for (int k = 0; k < 3; ++k) W.t[k] = z_t6[k];
  W.eps_lift = cfg->eps_lift;
  PmMeas m{in->Lambdas, in->thetas, in->etas, in->weights, in->colors, in->valid, in->sources, in->n_total,
           in->responsibilities, in->candidate_tile_ids, in->candidate_slots, in->row_masses, in->k_assoc};
  const int N = in->n_total, K = in->k_assoc, B = cfg->block_size, nl = p->nl;
  const int nb = (N + B - 1) / B;
  const int nrows = nb * B * K;
  const int kins = std::min(cfg->k_insert_tile, N);
  const int nprop = n * kins;
  const int R = std::max(nrows, nprop);
  // row buffers: lam 9, th 3, eta 3 nl, w, resp, col 3, fm (f64); valid (u8); src, tpos, slots (i32)
  const size_t f64s = (size_t)R * (9 + 3 + 3 * nl + 1 + 1 + 3 + 1);
  const size_t need = f64s * 8 + (size_t)R * (1 + 12) + (size_t)n * N * 8 + (size_t)n * kins * 4 + (size_t)N * 8 +
                      n * 8 + 256;
  if (need > p->ub_bytes) {
    if (p->ub) PMCHK(p, hipFree(p->ub));
    p->ub = nullptr;
    PMCHK(p, hipMalloc(&p->ub, need));
    p->ub_bytes = need;
  }
  double* f = (double*)p->ub;
  PmRowBuf o{};
  o.lam = f; f += (size_t)R * 9;
  o.th = f; f += (size_t)R * 3;
  o.eta = f; f += (size_t)R * 3 * nl;
  o.w = f; f += R;
  o.resp = f; f += R;
  o.col = f; f += (size_t)R * 3;
  o.fm = f; f += R;
  double* score = f; f += (size_t)n * N;
  int32_t* slot_of = (int32_t*)f;  // behind the scores (k_pm_proposals' layout)
  int64_t* mtile = (int64_t*)((char*)slot_of + (((size_t)n * kins * 4 + 7) & ~(size_t)7));
  int64_t* act = mtile + N;
  char* c8 = (char*)(act + n);
  o.valid = (uint8_t*)c8;
  int32_t* i32 = (int32_t*)(c8 + (((size_t)R + 7) & ~(size_t)7));
  o.src = i32; i32 += R;
  o.tpos = i32; i32 += R;
  o.slots = i32;
  (void)slot_of;
  // one device pass, one sync: every count and mass term the stats need goes to the mapped buffer
  // and is read after the single stream synchronize at the end (the per-operator entry points keep
  // their own syncs)
  if (n <= kPmArgTiles) {
    PmTileArgs ta{};
    ta.n = n;
    for (int t = 0; t < n; ++t) {
      ta.tiles[t] = tiles[t];
      ta.ids[t] = tile_ids[t];
    }
    hipLaunchKernelGGL(k_pm_stage_tiles, dim3(1), dim3(kPmArgTiles), 0, p->stream, ta, p->d_tiles, act);
  } else {
    PMCHK(p, hipMemcpyAsync(act, tile_ids, n * sizeof(int64_t), hipMemcpyHostToDevice, p->stream));
    if (int rc = upload_tiles(p, tiles, n)) return rc;
  }
  // fuse: per association block, every active tile (pipeline.py:1265-1327)
  hipLaunchKernelGGL(k_pm_fuse_rows, dim3((nrows + kPmThreads - 1) / kPmThreads), dim3(kPmThreads), 0, p->stream, m, W,
                     nl, B, nrows, (const int64_t*)act, n, o);
  PMCHK(p, hipGetLastError());
  if ((size_t)nb * n * 8 > kRecOff - kFmOff || (size_t)nprop * 8 > kFmOff - kWiOff)
    return pm_fail(p, GCS_ERR_ARG, "map update: stats exceed the mapped buffer");
  if (n > 0)
    hipLaunchKernelGGL(k_pm_fm_sums, dim3(nb, n), dim3(kPmThreads), 0, p->stream, (const double*)o.fm,
                       (const int32_t*)o.tpos, B * K, n, (double*)(p->d_small + kFmOff));
  gcs_pmap_rows ra{};
  ra.Lambdas = o.lam;
  ra.thetas = o.th;
  ra.etas = o.eta;
  ra.weights = o.w;
  ra.responsibilities = o.resp;
  ra.valid = o.valid;
  ra.colors = o.col;
  ra.sources = o.src;
  ra.tile_pos = o.tpos;
  ra.slots = o.slots;
  ra.n = nrows;
  if (int rc = fuse_blocks(p, n, &ra, nb, B * K, timestamp, scan_seq, cfg->eps_mass, nullptr)) return rc;
  // novelty insertion per active tile (pipeline.py:1331-1392): proposals, the eviction order (select of
  // the lowest retention keys) and the writes; ids continue tile by tile from next_global_id
  int32_t* d_ins = (int32_t*)p->d_small;
  if (kins > 0) {
    PmRowBuf ob = o;
    ob.w_host = (double*)(p->d_small + kWiOff);
    hipLaunchKernelGGL(k_pm_proposals, dim3(n), dim3(kPropThreads), 0, p->stream, m, W, nl, cfg->eps_mass, cfg->h_tile,
                       (const int64_t*)act, kins, score, mtile, ob);
    PMCHK(p, hipGetLastError());
    gcs_pmap_rows rp{};
    rp.Lambdas = o.lam;
    rp.thetas = o.th;
    rp.etas = o.eta;
    rp.weights = o.w;
    rp.valid = o.valid;
    rp.colors = o.col;
    rp.sources = o.src;
    rp.n = nprop;
    if (int rc = sort_tiles(p, n, 1, scan_seq, cfg->recency_decay_lambda, kins)) return rc;
    hipLaunchKernelGGL(k_pm_insert, dim3(n), dim3(kPmThreads), 0, p->stream, p->st, (const int32_t*)p->d_tiles, n, kins,
                       (const uint32_t*)p->vals, rows_of(&rp), timestamp, (long long)scan_seq,
                       (long long)next_global_id, (int64_t*)nullptr, d_ins);
    PMCHK(p, hipGetLastError());
  }
  // per tile: cull (its partials carry the valid count after it) and forget in one pass
  // (pipeline.py:1413-1447)
  const int nbt = blocks_per_tile(p->M);
  hipLaunchKernelGGL(k_pm_cull, dim3(n, nbt), dim3(kPmRed), 0, p->stream, p->st, (const int32_t*)p->d_tiles,
                     cfg->cull_threshold, (double*)(p->d_small + kPartOff), 1, cfg->forgetting_factor);
  PMCHK(p, hipGetLastError());
  p->pend.nb = nb;
  p->pend.kins = kins;
  p->pend.nbt = nbt;
  p->pend.on = true;
  return GCS_OK;
}

int pmap_update_collect(gcs_pmap* p, int64_t* next_global_id, gcs_pmap_update_stats* st, int32_t* counts) {
  if (!p || !next_global_id || !st || !counts) return GCS_ERR_ARG;
  memset(st, 0, sizeof(*st));
  if (!p->pend.on) return pm_fail(p, GCS_ERR_STATE, "map update: nothing queued");
  p->pend.on = false;
  const int n = p->pend.n, nb = p->pend.nb, kins = p->pend.kins, nbt = p->pend.nbt;
  const gcs_pmap_update_config* cfg = &p->pend.cfg;
  const int32_t* tiles = p->pend.tiles.data();
  *next_global_id = p->pend.next_id;
  if (n == 0) return GCS_OK;
  PMCHK(p, hipSetDevice(p->device));
  PMCHK(p, hipStreamSynchronize(p->stream));
  if (*(uint32_t*)(p->h_small + 8192)) return pm_fail(p, GCS_ERR_ARG, "target slot out of range (rows skipped)");
  {
    const uint32_t* nfb = (const uint32_t*)(p->h_small + 9216);
    const double* fms = (const double*)(p->h_small + kFmOff);
    for (int b = 0; b < nb; ++b) {
      st->fused_count += n * (int32_t)nfb[b];
      for (int t = 0; t < n; ++t) st->fused_mass_total += fms[b * n + t];  // per (block, tile) sums
    }
  }
  if (kins > 0) {
    const int32_t* ni = (const int32_t*)p->h_small;
    const double* wi = (const double*)(p->h_small + kWiOff);
    for (int t = 0; t < n; ++t) {
      st->insert_count_total += ni[t];
      *next_global_id += ni[t];
      std::vector<double> ws(wi + (size_t)t * kins, wi + (size_t)(t + 1) * kins);
      double sm = 0.0;
      for (double x : ws) sm += x;
      st->insert_mass_total += sm;
      std::sort(ws.begin(), ws.end());
      const int i95 = std::min((int)(0.95 * (double)kins), kins - 1);
      st->insert_mass_p95 = std::max(st->insert_mass_p95, ws[i95]);
    }
  }
  std::vector<int32_t> nc(n);
  std::vector<double> md(n);
  {
    const double* h = (const double*)(p->h_small + kPartOff);
    for (int t = 0; t < n; ++t) {  // block partials folded in block order (gcs_pmap_cull)
      double a[4] = {0.0, 0.0, 0.0, 0.0};
      for (int b = 0; b < nbt; ++b)
        for (int k = 0; k < 4; ++k) a[k] += h[4 * (t * nbt + b) + k];
      nc[t] = (int32_t)a[0];
      md[t] = a[1];
      counts[t] = (int32_t)a[3];
    }
  }
  for (int t = 0; t < n; ++t) {
    st->evicted_count += nc[t];
    st->evicted_mass_total += nc[t] ? md[t] : 0.0;
  }
  const bool capped = cfg->merge_max_tile_size > 0 && p->M > cfg->merge_max_tile_size;
  if (!capped && cfg->k_merge_pairs > 0 && p->M >= 2) {
    if (p->M > p->max_merge) return pm_fail(p, GCS_ERR_ARG, "map update: merge needs max_merge >= m_tile");
    std::vector<int32_t> pairs(2 * (size_t)cfg->k_merge_pairs);
    for (int t = 0; t < n; ++t) {
      if (counts[t] < 2) continue;
      int32_t nm = 0;
      if (int rc = gcs_pmap_merge_reduce(p, tiles[t], cfg->merge_threshold, cfg->k_merge_pairs, cfg->eps_psd,
                                         cfg->eps_lift, &nm, pairs.data(), &counts[t]))
        return rc;
      st->merged_count += nm;
    }
  }
  return GCS_OK;
}
}  // namespace live
}  // namespace gcs
