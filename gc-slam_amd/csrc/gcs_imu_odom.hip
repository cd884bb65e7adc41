// Step 9's IMU / odometry evidence family on the device: the reference's
// _compute_imu_odom_branch (FS/backend/pipeline.py:442-566, 595-776) with its eleven factors
// (imu_evidence.py:276-589, imu_gyro_evidence.py:38-163, imu_preintegration_factor.py:46-180,
// odom_evidence.py:39-154, odom_twist_evidence.py:58-430, planar_prior.py:55-195) as one workgroup:
//   * the window statistics -- dt_int (the sorted in-window stamps' positive gaps), dt_imu, omega_avg
//     (pipeline.py:262-313, 522-548) -- as block reductions and a bitonic sort in LDS;
//   * the scan-to-scan preintegration as gcs_preint_scan.h's parallel scans (k_preint's form);
//   * the IMU vMF factor's per-sample transport consistency, its two medians (bitonic sorts) and the
//     reliability-weighted sums (fixed-order block sums);
//   * lane 0 then runs the shared assembly (gcs_imu_odom_core.h imu_odom_assemble) -- the very code
//     the host branch runs -- into device memory, and every lane copies the result to a pinned host
//     record stamped with a sequence number and a checksum (the scan mirror's protocol, gcs_layout.h).
// The host form (gcs_evidence.cpp) stays the default; GCSLAM_DEVICE_IMU_ODOM=1 / GCS_DEBUG_DEVICE_IMU_ODOM
// selects this one, on its own stream beside the bin path's kernels.
#include <hip/hip_runtime.h>

#include <math.h>

#include "gcs_imu_odom_core.h"
#include "gcs_kernels.h"
#include "gcs_layout.h"
#include "gcs_preint_scan.h"

// timing probes (not parity builds; `make variant VSRC=gcs_imu_odom.hip VDEF=-DGCS_IO_PROBE=n`): 1 skips
// the three sorts, 2 the preintegration scan, 4 the vMF per-sample terms (bit mask)
#ifndef GCS_IO_PROBE
#define GCS_IO_PROBE 0
#endif

namespace gcs {
namespace {

constexpr int kIoThreads = preint::kPreintThreads;  // 512
constexpr int kIoWaves = kIoThreads / 64;
static_assert(kImuOdomMaxM <= 2 * kIoThreads, "the sorts hold two keys per lane");
static_assert(kIoThreads == 512, "io_sort's network: 1,024 positions");

// block reductions in a fixed order: a xor tree per wave, then the waves in order (every lane gets it)
__device__ __forceinline__ double io_block_sum(double v, double* s) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) s[wid] = v;
  __syncthreads();
  double r = s[0];
  for (int w = 1; w < kIoWaves; ++w) r += s[w];
  return r;
}
__device__ __forceinline__ double io_block_min(double v, double* s) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane == 0) s[wid] = v;
  __syncthreads();
  double r = s[0];
  for (int w = 1; w < kIoWaves; ++w) r = fmin(r, s[w]);
  return r;
}
__device__ __forceinline__ double io_block_max(double v, double* s) { return -io_block_min(-v, s); }

// ascending bitonic sort of the first np2 (a power of two, block-uniform) of the 2 kIoThreads keys in k
// (LDS; pad with +inf): lane t holds positions 2t and 2t + 1, so a stride-1 exchange stays in the lane,
// strides 2-64 are shuffles inside the wave (a wave holds 128 consecutive positions) and only strides of
// 128-512 go through LDS.  A network over np2 positions leaves the positions past np2 in place (a
// partner of such a position lies past np2 too), so a window of m samples costs log2(np2) (log2(np2) +
// 1) / 2 stages: 15 at the reference's ~20-sample windows instead of 55.
constexpr int kIoKeys = 2 * kIoThreads;
__device__ void io_sort(double* k, int np2) {
  const int t = (int)threadIdx.x;
  __syncthreads();
  double v[2] = {k[2 * t], k[2 * t + 1]};
  for (int size = 2; size <= np2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      double o[2];
      if (stride >= 128) {  // across waves
        __syncthreads();
        k[2 * t] = v[0];
        k[2 * t + 1] = v[1];
        __syncthreads();
        o[0] = k[(2 * t) ^ stride];
        o[1] = k[(2 * t + 1) ^ stride];
      } else if (stride == 1) {
        o[0] = v[1];
        o[1] = v[0];
      } else {
        o[0] = __shfl_xor(v[0], stride >> 1, 64);
        o[1] = __shfl_xor(v[1], stride >> 1, 64);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = 2 * t + j;
        const bool up = (p & size) == 0, low = (p & stride) == 0;
        // the lower position of an ascending pair keeps the smaller key, and so on
        const bool keep_small = low == up;
        v[j] = keep_small ? (o[j] < v[j] ? o[j] : v[j]) : (o[j] > v[j] ? o[j] : v[j]);
      }
    }
  __syncthreads();
  k[2 * t] = v[0];
  k[2 * t + 1] = v[1];
  __syncthreads();
}

__device__ __forceinline__ int io_pow2(int n) {
  int p = 2;
  while (p < n) p <<= 1;
  return p;
}

// numpy median of the first n sorted keys: the middle one, or the mean of the two middle ones
__device__ __forceinline__ double io_median(const double* k, int n) {
  const int h = n / 2;
  return (n % 2) ? k[h] : 0.5 * (k[h - 1] + k[h]);
}

__global__ __launch_bounds__(kIoThreads) void k_imu_odom(ImuOdomDevArgs a) {
  __shared__ double s_key[2 * kIoThreads];
  __shared__ double s_e[2 * kIoThreads];
  __shared__ double s_red[kIoWaves];
  __shared__ int s_cnt[kIoWaves + 1];
  __shared__ double s_pre[9];
  const int tid = (int)threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m = a.m;
  const double* stamps = a.win;
  const double* gyro = a.win + m;
  const double* accel = a.win + 4 * m;
  const double* w_int = a.win + 7 * m;
  const double* sm = a.win + 8 * m;  // the small inputs (ImuOdomDevArgs layout)
  const double* pose0 = sm + kIoPose0;
  const double* mu_inc = sm + kIoMuInc;
  const double* gb = mu_inc + 9;
  const double* ab = mu_inc + 12;
  const double* grav = sm + kIoGravity;
  const double t0 = a.t_last_scan, t1 = a.t_scan;
  // ---- dt_imu and omega_avg (pipeline.py:522-548): the valid stamps (> 0)
  double tmin = INFINITY, tmax = -INFINITY, ws = 0.0;
  int nv = 0;
  for (int i = tid; i < m; i += kIoThreads)
    if (stamps[i] > 0.0) {
      ++nv;
      tmin = fmin(tmin, stamps[i]);
      tmax = fmax(tmax, stamps[i]);
      ws += w_int[i];
    }
  tmin = io_block_min(tmin, s_red);
  tmax = io_block_max(tmax, s_red);
  const double wsum = io_block_sum(ws, s_red);
  const int n_valid = (int)io_block_sum((double)nv, s_red);
  double dt_imu = n_valid >= 2 ? (tmax - tmin) / (double)(n_valid - 1 > 1 ? n_valid - 1 : 1) : 0.0;
  dt_imu = dt_imu > 1e-12 ? dt_imu : 1e-12;
  const double inv = 1.0 / (wsum + kEpsMass);
  double om[3] = {0.0, 0.0, 0.0};
  for (int i = tid; i < m; i += kIoThreads)
    if (stamps[i] > 0.0) {
      const double wn = w_int[i] * inv;
      for (int k = 0; k < 3; ++k) om[k] += wn * (gyro[3 * i + k] - gb[k]);
    }
  for (int k = 0; k < 3; ++k) om[k] = io_block_sum(om[k], s_red);
  // ---- dt_int (pipeline.py:262-313): the in-window stamps in order, sorted, their positive gaps summed
  const double eps = 1e-9;
  int n_in = 0;
  {
    int base = 0;
    for (int c0 = 0; c0 < m; c0 += kIoThreads) {  // order-preserving compaction into s_key
      const int i = c0 + tid;
      const bool in = i < m && stamps[i] > t0 - eps && stamps[i] <= t1 + eps && stamps[i] > 0.0;
      const unsigned long long bal = __ballot(in);
      const int before = __popcll(bal & ((1ull << lane) - 1ull));
      __syncthreads();
      if (lane == 0) s_cnt[wid] = __popcll(bal);
      __syncthreads();
      int off = base;
      for (int w = 0; w < wid; ++w) off += s_cnt[w];
      if (in) s_key[off + before] = stamps[i];
      int tot = 0;
      for (int w = 0; w < kIoWaves; ++w) tot += s_cnt[w];
      base += tot;
    }
    n_in = base;
  }
  // IMU stamps arrive in order: the sort runs only when a pair of the in-window stamps is not (the
  // reference sorts unconditionally; the sorted keys are the same)
  bool unsorted = false;
  __syncthreads();
  for (int i = 1 + tid; i < n_in; i += kIoThreads) unsorted = unsorted || s_key[i] < s_key[i - 1];
  if (__syncthreads_or(unsorted) && !(GCS_IO_PROBE & 1)) {
    for (int i = n_in + tid; i < kIoKeys; i += kIoThreads) s_key[i] = INFINITY;
    io_sort(s_key, io_pow2(n_in));
  }
  double gaps = 0.0;
  for (int i = 1 + tid; i < n_in; i += kIoThreads) {
    const double g = s_key[i] - s_key[i - 1];
    gaps += g > 0.0 ? g : 0.0;
  }
  gaps = io_block_sum(gaps, s_red);
  double dt_int = 0.0;
  if (n_in >= 2) {
    const double span = t1 - t0;
    dt_int = gaps < span ? gaps : span;
    dt_int = dt_int > 0.0 ? dt_int : 0.0;
  }
  // ---- the scan-to-scan preintegration (pipeline.py:442-453; imu_preintegration.py:47-147)
  double Pc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, vc[3] = {0, 0, 0}, pc[3] = {0, 0, 0}, ess = 0.0;
  if (!(GCS_IO_PROBE & 2))
    preint::window_carry(stamps, gyro, accel, m, [=](int i, double) { return w_int[i]; }, pose0 + 3, gb, ab, grav,
                         Pc, vc, pc, ess);
  if (tid == 0) {
    double R0[9], Re[9], dR[9];
    so3_exp(pose0 + 3, R0);
    preint::mat3_mul_inplace(R0, Pc, Re);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dR[3 * i + j] = R0[i] * Re[j] + R0[3 + i] * Re[3 + j] + R0[6 + i] * Re[6 + j];
    for (int i = 0; i < 3; ++i) s_pre[i] = R0[i] * pc[0] + R0[3 + i] * pc[1] + R0[6 + i] * pc[2];  // dp (body)
    for (int i = 0; i < 3; ++i) s_pre[6 + i] = R0[i] * vc[0] + R0[3 + i] * vc[1] + R0[6 + i] * vc[2];  // dv
    so3_log(dR, s_pre + 3);  // drot
  }
  // ---- the IMU vMF factor's per-sample statistics (imu_evidence.py:276-399)
  for (int i = tid; i < m && !(GCS_IO_PROBE & 4); i += kIoThreads) {  // transport consistency e_i (central differences)
    double df[3], ai[3], c[3];
    for (int k = 0; k < 3; ++k) {
      ai[k] = accel[3 * i + k] - ab[k];
      if (i == 0) df[k] = ((accel[3 + k] - ab[k]) - ai[k]) / (dt_imu + kEpsMass);
      else if (i == m - 1) df[k] = (ai[k] - (accel[3 * (i - 1) + k] - ab[k])) / (dt_imu + kEpsMass);
      else df[k] = ((accel[3 * (i + 1) + k] - ab[k]) - (accel[3 * (i - 1) + k] - ab[k])) / (2 * dt_imu + kEpsMass);
    }
    cross3(gyro + 3 * i, ai, c);
    const double ex = df[0] + c[0], ey = df[1] + c[1], ez = df[2] + c[2];
    s_e[i] = sqrt(ex * ex + ey * ey + ez * ez);
  }
  __syncthreads();
  for (int i = tid; i < kIoKeys; i += kIoThreads) s_key[i] = i < m ? s_e[i] : INFINITY;
  if (!(GCS_IO_PROBE & 1)) io_sort(s_key, io_pow2(m));
  const double med = io_median(s_key, m);
  __syncthreads();
  for (int i = tid; i < kIoKeys; i += kIoThreads) s_key[i] = i < m ? fabs(s_e[i] - med) : INFINITY;
  if (!(GCS_IO_PROBE & 1)) io_sort(s_key, io_pow2(m));
  host::ImuVmfStats v{};
  v.sigma = io_median(s_key, m) / 0.6745 + kEpsMass;
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // rel, w, w_int, S[3]
  for (int i = tid; i < m; i += kIoThreads) {
    const double q = s_e[i] / v.sigma;
    const double rel = exp(-0.5 * (q * q));
    const double w = w_int[i] * rel;
    acc[0] += rel;
    acc[1] += w;
    acc[2] += w_int[i];
    double ai[3];
    for (int k = 0; k < 3; ++k) ai[k] = accel[3 * i + k] - ab[k];
    const double n = sqrt(ai[0] * ai[0] + ai[1] * ai[1] + ai[2] * ai[2]);
    for (int k = 0; k < 3; ++k) acc[3 + k] += w * (ai[k] / (n + kEpsMass));
  }
  v.rel_sum = io_block_sum(acc[0], s_red);
  v.ess_w = io_block_sum(acc[1], s_red);
  v.ess_raw = io_block_sum(acc[2], s_red);
  for (int k = 0; k < 3; ++k) v.S[k] = io_block_sum(acc[3 + k], s_red);
  // ---- the statistics for the assembly kernel (one wave, its registers free of this kernel's sorts)
  if (tid == 0) {
    double* st = a.out + kIoOutWords;
    st[0] = v.S[0]; st[1] = v.S[1]; st[2] = v.S[2];
    st[3] = v.ess_w; st[4] = v.ess_raw; st[5] = v.rel_sum; st[6] = v.sigma;
    st[7] = dt_imu; st[8] = dt_int; st[9] = om[0]; st[10] = om[1]; st[11] = om[2];
    for (int k = 0; k < 9; ++k) st[12 + k] = s_pre[k];
  }
}

// The eleven factors and their sum (the host branch's code, gcs_imu_odom_core.h) into device memory:
// the four waves' lane 0 run the six factor parts -- the 6x6 odometry factor alone, the others in pairs
// (the parts read only the inputs; their results meet in LDS) --, then lane 0 adds them in the
// pipeline's order; the first wave then copies the record to the pinned host record, stamped.  One wave
// per SIMD: a part's fixed-size algebra (the 6x6 Jacobi) keeps its arrays in up to 512 registers.
constexpr int kIoAsmWaves = 4;
__global__ __launch_bounds__(64 * kIoAsmWaves) void k_imu_odom_assemble(ImuOdomDevArgs a) {
  __shared__ host::ImuOdomParts s_p;
  const int tid = (int)threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int m = a.m;
  const double* sm = a.win + 8 * m;
  const double* mu_inc = sm + kIoMuInc;
  host::ImuOdomOut* out = reinterpret_cast<host::ImuOdomOut*>(a.out);
  double* extra = a.out + kIoOutWords - 5;
  const double* st = a.out + kIoOutWords;
  host::ImuVmfStats v{};
  double om[3], pre[9];
  host::ImuOdomInputs in{};
  if (lane == 0) {
    v.S[0] = st[0]; v.S[1] = st[1]; v.S[2] = st[2];
    v.ess_w = st[3]; v.ess_raw = st[4]; v.rel_sum = st[5]; v.sigma = st[6];
    om[0] = st[9]; om[1] = st[10]; om[2] = st[11];
    for (int k = 0; k < 9; ++k) pre[k] = st[12 + k];
    in.m = m;
    in.stamps = a.win; in.gyro = a.win + m; in.accel = a.win + 4 * m; in.w_int = a.win + 7 * m;
    in.dt_imu = st[7]; in.dt_int = st[8]; in.dt_sec = a.dt_sec;
    in.omega_avg = om;
    in.dp_int = pre; in.drot_int = pre + 3; in.dv_int = pre + 6;
    in.pose0 = sm + kIoPose0; in.pose_pred = sm + kIoPosePred; in.mu_prev = sm + kIoMuPrev; in.mu_inc = mu_inc;
    in.accel_bias = mu_inc + 12;
    in.gravity = sm + kIoGravity;
    in.Sigma_g = sm + kIoSigmaG; in.Sigma_a = sm + kIoSigmaA;
    in.odom_pose = sm + kIoOdomPose; in.odom_cov = sm + kIoOdomCov; in.odom_twist = sm + kIoOdomTwist;
    in.odom_twist_cov = sm + kIoOdomTwistCov;
    in.planar_z_ref = a.planar_z_ref; in.planar_z_sigma = a.planar_z_sigma; in.planar_vz_sigma = a.planar_vz_sigma;
  }
  if (tid == 0) host::io_init(*out);
  __syncthreads();
  if (lane == 0) {  // parts {0}, {1, 4}, {2, 3}, {5}
    constexpr int kFirst[kIoAsmWaves] = {0, 1, 2, 5}, kSecond[kIoAsmWaves] = {-1, 4, 3, -1};
    host::io_part(kFirst[wid], in, v, s_p, *out);
    if (kSecond[wid] >= 0) host::io_part(kSecond[wid], in, v, s_p, *out);
  }
  __syncthreads();
  if (tid == 0) {
    host::io_sum(in, s_p, *out);
    extra[0] = in.dt_int; extra[1] = in.dt_imu; extra[2] = om[0]; extra[3] = om[1]; extra[4] = om[2];
  }
  __syncthreads();
  // ---- the stamped copy to the pinned host record: kIoOutWords words, sequence, checksum
  if (!a.host || wid != 0) return;
  uint64_t* hw = reinterpret_cast<uint64_t*>(a.host);
  const uint64_t* dw = reinterpret_cast<const uint64_t*>(a.out);
  unsigned long long h = 0;
  for (int i = tid; i < kIoOutWords; i += 64) {
    const uint64_t w = dw[i];
    hw[i] = w;
    h += mirror_word_hash(w, (uint32_t)i);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) h += __shfl_xor(h, o, 64);
  __threadfence_system();
  if (tid == 0) {
    const uint64_t seq = *a.dseq + 1u;
    *a.dseq = seq;
    const uint64_t sum = mirror_word_hash(seq, (uint32_t)kIoOutWords) + h;
    hw[kIoOutWords + 1] = sum;
    hw[kIoOutWords] = seq;
  }
}

}  // namespace

hipError_t launch_imu_odom(const ImuOdomDevArgs& a, hipStream_t s) {
  if (a.m < 2 || a.m > kImuOdomMaxM) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_imu_odom, dim3(1), dim3(kIoThreads), 0, s, a);
  hipLaunchKernelGGL(k_imu_odom_assemble, dim3(1), dim3(64 * kIoAsmWaves), 0, s, a);
  return hipGetLastError();
}

}  // namespace gcs
