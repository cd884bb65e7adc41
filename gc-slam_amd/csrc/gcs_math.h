// Host/device f64 math shared by the HIP kernels and the host 22-D tail.
// Lie maps restate fl_ws/src/fl_slam_poc/fl_slam_poc/common/geometry/se3_jax.py;
// the PSD projection restates domain_projection_psd_core (common/primitives.py:80-123)
// with a 3x3 cyclic Jacobi eigensolver instead of LAPACK syevd.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "gcs_sh_tables.h"

// instrumented build only (make prof): device counters of the 3x3 PSD paths
#ifdef GCS_PHASE_PROF
__device__ unsigned long long g_psd_count[4];  // non-zero inputs, deflation path, non-finite
#ifdef __HIP_DEVICE_COMPILE__
#define GCS_PSD_COUNT(k) atomicAdd(&g_psd_count[k], 1ull)
#endif
#endif
#ifndef GCS_PSD_COUNT
#define GCS_PSD_COUNT(k)
#endif

#define GCS_HD __host__ __device__ __forceinline__

namespace gcs {

constexpr double kEpsPsd = 1e-12;     // constants.py:70
constexpr double kEpsLift = 1e-9;     // constants.py:71
constexpr double kEpsMass = 1e-12;    // constants.py:72
constexpr double kEpsR = 1e-6;        // constants.py:73
constexpr double kKappaR0 = 0.8;      // constants.py:95
constexpr double kKappaTau = 0.03;    // constants.py:96
constexpr double kF64Eps = 2.220446049250313e-16;
constexpr double kSmallAngle = 1e-7;  // se3_jax.py:29
constexpr double kWeightFloor = 1e-12;  // constants.py:256
constexpr double kTimeWarpSigmaFrac = 0.1;  // constants.py:143

// Canonical dot (x*x' + y*y') + z*z' with no fused multiply-add: the op order the
// oracle uses, so nearest-bin / kNN decisions are bit-identical (DESIGN.md "indices").
GCS_HD double dot3_exact(double ax, double ay, double az, double bx, double by, double bz) {
#pragma clang fp contract(off)
  double xx = ax * bx;
  double yy = ay * by;
  double zz = az * bz;
  double s = xx + yy;
  return s + zz;
}

// Ray direction of a deskewed point from the LiDAR origin (pipeline.py:589-593): (p - o) / (|p - o| +
// eps).  One expression for every kernel that forms it -- the point kernel, and the bin kernel's staging
// that re-derives it from the 32-B record (gcs_layout.h PointRec32) -- so they agree bit for bit.
GCS_HD void ray_dir(double px, double py, double pz, const double* o, double* d) {
#pragma clang fp contract(off)
  double rx = px - o[0], ry = py - o[1], rz = pz - o[2];
  double nrm = sqrt(dot3_exact(rx, ry, rz, rx, ry, rz));
  double den = nrm + kEpsMass;
  d[0] = rx / den; d[1] = ry / den; d[2] = rz / den;
}

// 1 / d for a positive normal d.  Device: v_rcp_f64 and two Newton steps (within an ulp of the IEEE
// quotient, 5 instructions against the ~10 of the division's scale / fmas / fixup sequence); host: the
// division.  The bin kernels' per-bin finalize takes its reciprocals here (the tolerances of the
// quantities involved are >= 1e-12 relative).
GCS_HD double rcp_fast(double d) {
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  return fma(fma(-d, r, 1.0), r, r);
#else
  return 1.0 / d;
#endif
}

GCS_HD double sigmoid(double x) {
  // numerically symmetric logistic; above 40, exp(-x) < 2^-57 and 1 / (1 + exp(-x)) rounds to
  // exactly 1.0, which is returned without the exp (bitwise the same value)
  if (x > 40.0) return 1.0;
  if (x >= 0.0) {
    double e = exp(-x);
    return 1.0 / (1.0 + e);
  }
  double e = exp(x);
  return e / (1.0 + e);
}

// smooth_window_weights, imu_preintegration.py:20-43
GCS_HD double smooth_window(double t, double start, double end, double sigma) {
  double sig = sigma > 1e-6 ? sigma : 1e-6;
  const double a = (t - start) / sig, b = (end - t) / sig;
  // exp underflows to exactly 0 below -745.2, so a factor is exactly 0 there and w is the floor
  // (padded IMU samples, stamp 0): the same value without the two exps
  if (a < -746.0 || b < -746.0) return kWeightFloor;
  double w = sigmoid(a) * sigmoid(b);
  return w * (1.0 - kWeightFloor) + kWeightFloor;
}

// kappa_from_resultant_batch, kappa.py:130-169
GCS_HD double kappa_from_rbar(double rbar) {
  double R = rbar < 0.0 ? 0.0 : rbar;
  R = R > 1.0 - kEpsR ? 1.0 - kEpsR : R;
  double R2 = R * R;
  double k_low = (R * (3.0 - R2)) * rcp_fast(1.0 - R2 + kEpsR);
  double om = 1.0 - R2;
  double k_high = -log(om > kEpsR ? om : kEpsR);
  double s = sigmoid((R - kKappaR0) / kKappaTau);
  return (1.0 - s) * k_low + s * k_high;
}

// --------------------------------------------------------------------------- 3x3 helpers
// Symmetric 3x3 stored as a[9] row-major.
GCS_HD void mat3_mul(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

GCS_HD void skew3(const double* v, double* K) {
  K[0] = 0.0; K[1] = -v[2]; K[2] = v[1];
  K[3] = v[2]; K[4] = 0.0; K[5] = -v[0];
  K[6] = -v[1]; K[7] = v[0]; K[8] = 0.0;
}

// so3_exp, se3_jax.py:260-300
GCS_HD void so3_exp(const double* w, double* R) {
  double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double theta = sqrt(theta_sq);
  double K[9], K2[9];
  skew3(w, K);
  mat3_mul(K, K, K2);
  bool small = theta < kSmallAngle;
  double st = small ? 1.0 : theta;
  double st2 = theta_sq < kSmallAngle * kSmallAngle ? 1.0 : theta_sq;
  double a = small ? 1.0 : sin(st) / st;
  double b = small ? 0.5 : (1.0 - cos(st)) / st2;
  for (int i = 0; i < 9; ++i) R[i] = a * K[i] + b * K2[i];
  R[0] += 1.0; R[4] += 1.0; R[8] += 1.0;
}

// so3_log, se3_jax.py:303-365 (softmax near-pi axis mixture)
GCS_HD void so3_log(const double* R, double* w) {
  double ct = 0.5 * (R[0] + R[4] + R[8] - 1.0);
  ct = ct < -1.0 ? -1.0 : (ct > 1.0 ? 1.0 : ct);
  double theta = acos(ct);
  double vx = 0.5 * (R[7] - R[5]), vy = 0.5 * (R[2] - R[6]), vz = 0.5 * (R[3] - R[1]);
  if (theta < kSmallAngle) { w[0] = vx; w[1] = vy; w[2] = vz; return; }
  const double pi = 3.141592653589793;
  if (fabs(theta - pi) < 1e-7) {
    double d0 = 50.0 * (R[0] + 1.0), d1 = 50.0 * (R[4] + 1.0), d2 = 50.0 * (R[8] + 1.0);
    double m = d0 > d1 ? d0 : d1; m = m > d2 ? m : d2;
    double e0 = exp(d0 - m), e1 = exp(d1 - m), e2 = exp(d2 - m), es = e0 + e1 + e2;
    e0 /= es; e1 /= es; e2 /= es;
    double ax = e0 * (R[0] + 1.0) + e1 * R[1] + e2 * R[2];
    double ay = e0 * R[3] + e1 * (R[4] + 1.0) + e2 * R[5];
    double az = e0 * R[6] + e1 * R[7] + e2 * (R[8] + 1.0);
    double n = sqrt(ax * ax + ay * ay + az * az);
    n = n < kSmallAngle ? 1.0 : n;
    w[0] = ax / n * theta; w[1] = ay / n * theta; w[2] = az / n * theta;
    return;
  }
  double s = sin(theta);
  s = fabs(s) < kSmallAngle ? 1.0 : s;
  double f = theta / (2.0 * s);
  w[0] = f * (2.0 * vx); w[1] = f * (2.0 * vy); w[2] = f * (2.0 * vz);
}

// B(theta), C(theta) of se3_exp / se3_V, se3_jax.py:488-500
GCS_HD void se3_BC(double theta_sq, double* B, double* C, double* sin_c, double* cos_c) {
  double theta = sqrt(theta_sq);
  bool small = theta < kSmallAngle;
  double st = small ? 1.0 : theta;
  double st2 = theta_sq < kSmallAngle * kSmallAngle ? 1.0 : theta_sq;
  double sn = sin(st), cs = cos(st);
  *B = small ? 0.5 - theta_sq / 24.0 : (1.0 - cs) / st2;
  *C = small ? 1.0 / 6.0 - theta_sq / 120.0 : (st - sn) / (st2 * st);
  *sin_c = small ? 1.0 : sn / st;
  *cos_c = small ? 0.5 : (1.0 - cs) / st2;
}

// se3_exp (se3_jax.py:474-504): out = [V rho, phi]
GCS_HD void se3_exp(const double* xi, double* out) {
  const double* phi = xi + 3;
  double theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  double B, C, a, b;
  se3_BC(theta_sq, &B, &C, &a, &b);
  double K[9], K2[9];
  skew3(phi, K);
  mat3_mul(K, K, K2);
  for (int i = 0; i < 3; ++i) {
    double acc = xi[i];
    for (int j = 0; j < 3; ++j) acc += (B * K[3 * i + j] + C * K2[3 * i + j]) * xi[j];
    out[i] = acc;
  }
  out[3] = phi[0]; out[4] = phi[1]; out[5] = phi[2];
}

// se3_log, se3_jax.py:210-245 (with _se3_V_inv, :169-207)
GCS_HD void se3_log_hd(const double* T, double* out) {
  double R[9], phi[3];
  so3_exp(T + 3, R);
  so3_log(R, phi);
  double theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  double theta = sqrt(theta_sq);
  bool small = theta < kSmallAngle;
  double st = small ? 1.0 : theta;
  double st2 = theta_sq < kSmallAngle * kSmallAngle ? 1.0 : theta_sq;
  double denom = 2.0 * st * sin(st) + 1e-12;
  double D = small ? 1.0 / 12.0 + theta_sq / 720.0 : (1.0 / st2) - (1.0 + cos(st)) / denom;
  double K[9], K2[9];
  skew3(phi, K);
  mat3_mul(K, K, K2);
  for (int i = 0; i < 3; ++i) {
    double acc = T[i];
    for (int j = 0; j < 3; ++j) acc += (-0.5 * K[3 * i + j] + D * K2[3 * i + j]) * T[j];
    out[i] = acc;
  }
  out[3] = phi[0]; out[4] = phi[1]; out[5] = phi[2];
}

// Per-point deskew: T = se3_exp(alpha xi); p0 = R^T (p - t)  (deskew_constant_twist.py:51-58)
GCS_HD void deskew_point(double alpha, const double* xi, const double* p, double* p0) {
  double rho[3] = {alpha * xi[0], alpha * xi[1], alpha * xi[2]};
  double phi[3] = {alpha * xi[3], alpha * xi[4], alpha * xi[5]};
  double theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  double B, C, a, b;
  se3_BC(theta_sq, &B, &C, &a, &b);
  double K[9], K2[9];
  skew3(phi, K);
  mat3_mul(K, K, K2);
  double t[3];
  for (int i = 0; i < 3; ++i) {
    t[i] = rho[i] + (B * K[3 * i] + C * K2[3 * i]) * rho[0] + (B * K[3 * i + 1] + C * K2[3 * i + 1]) * rho[1] +
           (B * K[3 * i + 2] + C * K2[3 * i + 2]) * rho[2];
  }
  double q[3] = {p[0] - t[0], p[1] - t[1], p[2] - t[2]};
  for (int i = 0; i < 3; ++i) {
    // column i of R: R[j][i] = delta_ji + a K[j][i] + b K2[j][i]
    double acc = q[i];
    for (int j = 0; j < 3; ++j) acc += (a * K[3 * j + i] + b * K2[3 * j + i]) * q[j];
    p0[i] = acc;
  }
}

// Cyclic Jacobi eigensolver for a symmetric 3x3 (row-major a[9]); returns eigenvalues w[3]
// (unsorted) and eigenvectors as columns of V[9].  Deterministic sweep order (0,1),(0,2),(1,2).
GCS_HD void eigh3_jacobi(const double* A, double* w, double* V) {
  double a[9];
  for (int i = 0; i < 9; ++i) { a[i] = A[i]; V[i] = (i % 4 == 0) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 12; ++sweep) {
    double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    double diag = a[0] * a[0] + a[4] * a[4] + a[8] * a[8];
    if (off <= 1e-40 * diag || off == 0.0) break;
    for (int pq = 0; pq < 3; ++pq) {
      int p = pq == 2 ? 1 : 0;
      int q = pq == 0 ? 1 : 2;
      double apq = a[3 * p + q];
      if (apq == 0.0) continue;
      double app = a[4 * p], aqq = a[4 * q];
      double theta = (aqq - app) / (2.0 * apq);
      double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      double c = 1.0 / sqrt(t * t + 1.0);
      double s = t * c;
      // A' = J^T A J with J = rotation in (p,q)
      for (int k = 0; k < 3; ++k) {
        double akp = a[3 * k + p], akq = a[3 * k + q];
        a[3 * k + p] = c * akp - s * akq;
        a[3 * k + q] = s * akp + c * akq;
      }
      for (int k = 0; k < 3; ++k) {
        double apk = a[3 * p + k], aqk = a[3 * q + k];
        a[3 * p + k] = c * apk - s * aqk;
        a[3 * q + k] = s * apk + c * aqk;
      }
      a[3 * p + q] = 0.0;
      a[3 * q + p] = 0.0;
      for (int k = 0; k < 3; ++k) {
        double vkp = V[3 * k + p], vkq = V[3 * k + q];
        V[3 * k + p] = c * vkp - s * vkq;
        V[3 * k + q] = s * vkp + c * vkq;
      }
    }
  }
  w[0] = a[0]; w[1] = a[4]; w[2] = a[8];
}

GCS_HD void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// Clamped-eigenpair form of the 3x3 PSD projection, for a symmetric s that failed the fast
// paths (rank-deficient scatter: bins with one to three points).  With w_i, v_i the eigenpairs,
// V diag(max(w, eps)) V^T = s + sum_{w_i < eps} (eps - w_i) v_i v_i^T and the projection delta is
// sqrt(sum_{w_i < eps} (eps - w_i)^2), so only the clamped pairs are needed:
//   * the top eigenvalue by Newton's method on the characteristic cubic from the Gershgorin
//     bound (monotone from above; no transcendental calls) and its vector as the longest cross
//     product of two rows of s - w_1 I;
//   * the two small eigenpairs from the 2x2 projection of s onto the complement of that vector
//     (closed form, absolute accuracy ~ 1e-16 |s|, far below eps = 1e-12).
// A (near) double top eigenvalue is handled in closed form below (the bottom eigenpair is then
// separated); returns false only on non-finite input.
#ifndef GCS_DEFLATE_FROB
#define GCS_DEFLATE_FROB 1  // Newton's start (above); 0: the Gershgorin bound alone
#endif
GCS_HD __attribute__((always_inline)) bool psd3_deflate(const double* s, double* out, double* delta) {
  const double c2 = s[0] + s[4] + s[8];
  const double c1 = (s[0] * s[4] - s[1] * s[1]) + (s[0] * s[8] - s[2] * s[2]) + (s[4] * s[8] - s[5] * s[5]);
  const double c0 = s[0] * (s[4] * s[8] - s[5] * s[5]) - s[1] * (s[1] * s[8] - s[5] * s[2]) +
                    s[2] * (s[1] * s[5] - s[4] * s[2]);
  // start: the smaller of the Gershgorin bound and the Frobenius norm (|lambda| <= ||s||_F for a
  // symmetric s; exact for rank 1, within sqrt 2 for rank 2 -- the scatters of one to three points
  // that come here), so Newton starts at or above the top root and converges in a few steps
#if GCS_DEFLATE_FROB
  const double fro = sqrt((s[0] * s[0] + s[4] * s[4] + s[8] * s[8]) + 2.0 * ((s[1] * s[1] + s[2] * s[2]) + s[5] * s[5]));
#else
  const double fro = 1e308;
#endif
  double lam = fmin(fmax(fmax(s[0] + fabs(s[1]) + fabs(s[2]), s[4] + fabs(s[1]) + fabs(s[5])),
                         s[8] + fabs(s[2]) + fabs(s[5])), fro);
  if (!(lam > -1e300 && lam < 1e300)) return false;  // NaN / inf
  for (int it = 0; it < 100; ++it) {
    const double f = ((lam - c2) * lam + c1) * lam - c0;
    const double fp = (3.0 * lam - 2.0 * c2) * lam + c1;
    if (!(fp > 0.0) || !(f > 0.0)) break;
    const double step = f / fp;
    lam -= step;
    if (step <= 1e-15 * fabs(lam)) break;
  }
  const double m0 = s[0] - lam, m4 = s[4] - lam, m8 = s[8] - lam;
  // cross products of the rows (m0 s1 s2), (s1 m4 s5), (s2 s5 m8)
  const double x0 = s[1] * s[5] - s[2] * m4, x1 = s[2] * s[1] - m0 * s[5], x2 = m0 * m4 - s[1] * s[1];
  const double y0 = s[1] * m8 - s[2] * s[5], y1 = s[2] * s[2] - m0 * m8, y2 = m0 * s[5] - s[1] * s[2];
  const double z0 = m4 * m8 - s[5] * s[5], z1 = s[5] * s[2] - s[1] * m8, z2 = s[1] * s[5] - m4 * s[2];
  const double nx = x0 * x0 + x1 * x1 + x2 * x2, ny = y0 * y0 + y1 * y1 + y2 * y2, nz = z0 * z0 + z1 * z1 + z2 * z2;
  double u0 = x0, u1 = x1, u2 = x2, nmax = nx;
  if (ny > nmax) { u0 = y0; u1 = y1; u2 = y2; nmax = ny; }
  if (nz > nmax) { u0 = z0; u1 = z1; u2 = z2; nmax = nz; }
  const double mf2 = m0 * m0 + m4 * m4 + m8 * m8 + 2.0 * (s[1] * s[1] + s[2] * s[2] + s[5] * s[5]);
  if (!(nmax > 1e-12 * mf2 * mf2)) {
    // (near) double top eigenvalue (the rows of s - lam I are parallel: cross products below 1e-6 of
    // their scale, so the top gap is below 1e-6 of the distance to the bottom root): s - lam I =
    // (w3 - lam) v3 v3^T + O(gap), and v3 is the longest row, sharpened by one power step with
    // s - lam I (its other component shrinks by gap / (lam - w3) <= 1e-6 again), w3 = v3^T s v3.
    // The top pair is clamped iff lam < eps (within the gap, where a clamp is below 1e-18), so:
    // lam < eps -> every eigenvalue clamped, eps I and ||eps I - s||_F^2 (the trace / Frobenius
    // identity for sum (eps - w_i)^2); otherwise only w3 can be: s + (eps - w3) v3 v3^T.
    if (!(lam > -1e300 && lam < 1e300) || !(mf2 < 1e300)) return false;
    if (lam < kEpsPsd) {
      for (int k = 0; k < 9; ++k) out[k] = (k % 4 == 0) ? kEpsPsd : 0.0;
      const double g0 = kEpsPsd - s[0], g4 = kEpsPsd - s[4], g8 = kEpsPsd - s[8];
      *delta = sqrt((g0 * g0 + g4 * g4 + g8 * g8) + 2.0 * ((s[1] * s[1] + s[2] * s[2]) + s[5] * s[5]));
      return true;
    }
    const double r0 = m0 * m0 + s[1] * s[1] + s[2] * s[2], r1 = s[1] * s[1] + m4 * m4 + s[5] * s[5],
                 r2 = s[2] * s[2] + s[5] * s[5] + m8 * m8;
    double v0 = m0, v1 = s[1], v2 = s[2], rm = r0;
    if (r1 > rm) { v0 = s[1]; v1 = m4; v2 = s[5]; rm = r1; }
    if (r2 > rm) { v0 = s[2]; v1 = s[5]; v2 = m8; rm = r2; }
    for (int k = 0; k < 9; ++k) out[k] = s[k];
    if (!(rm > 0.0)) {  // s = lam I exactly: nothing clamped
      *delta = 0.0;
      return true;
    }
    const double p0 = m0 * v0 + s[1] * v1 + s[2] * v2, p1 = s[1] * v0 + m4 * v1 + s[5] * v2,
                 p2 = s[2] * v0 + s[5] * v1 + m8 * v2;
    const double pn = p0 * p0 + p1 * p1 + p2 * p2;
    if (pn > 0.0) { v0 = p0; v1 = p1; v2 = p2; rm = pn; }
    const double iv = 1.0 / sqrt(rm);
    v0 *= iv; v1 *= iv; v2 *= iv;
    const double w3 = v0 * (s[0] * v0 + s[1] * v1 + s[2] * v2) + v1 * (s[1] * v0 + s[4] * v1 + s[5] * v2) +
                      v2 * (s[2] * v0 + s[5] * v1 + s[8] * v2);
    double d2 = 0.0;
    if (w3 < kEpsPsd) {
      const double g = kEpsPsd - w3;
      d2 = g * g;
      out[0] += g * v0 * v0; out[1] += g * v0 * v1; out[2] += g * v0 * v2;
      out[3] += g * v1 * v0; out[4] += g * v1 * v1; out[5] += g * v1 * v2;
      out[6] += g * v2 * v0; out[7] += g * v2 * v1; out[8] += g * v2 * v2;
    }
    *delta = sqrt(d2);
    return true;
  }
  const double in = 1.0 / sqrt(nmax);
  u0 *= in; u1 *= in; u2 *= in;
  // orthonormal complement e, f of u: e = u x (axis of the smallest |u_k|), f = u x e
  const double a0 = fabs(u0), a1 = fabs(u1), a2 = fabs(u2);
  double e0, e1, e2;
  if (a0 <= a1 && a0 <= a2) { e0 = 0.0; e1 = u2; e2 = -u1; }        // u x (1,0,0)
  else if (a1 <= a2) { e0 = -u2; e1 = 0.0; e2 = u0; }               // u x (0,1,0)
  else { e0 = u1; e1 = -u0; e2 = 0.0; }                             // u x (0,0,1)
  const double ie = 1.0 / sqrt(e0 * e0 + e1 * e1 + e2 * e2);
  e0 *= ie; e1 *= ie; e2 *= ie;
  const double f0 = u1 * e2 - u2 * e1, f1 = u2 * e0 - u0 * e2, f2 = u0 * e1 - u1 * e0;
  // 2x2 projection [[a b] [b c]] of s onto span(e, f)
  const double se0 = s[0] * e0 + s[1] * e1 + s[2] * e2, se1 = s[1] * e0 + s[4] * e1 + s[5] * e2,
               se2 = s[2] * e0 + s[5] * e1 + s[8] * e2;
  const double sf0 = s[0] * f0 + s[1] * f1 + s[2] * f2, sf1 = s[1] * f0 + s[4] * f1 + s[5] * f2,
               sf2 = s[2] * f0 + s[5] * f1 + s[8] * f2;
  const double a = e0 * se0 + e1 * se1 + e2 * se2;
  const double c = f0 * sf0 + f1 * sf1 + f2 * sf2;
  const double b = 0.5 * ((e0 * sf0 + e1 * sf1 + e2 * sf2) + (f0 * se0 + f1 * se1 + f2 * se2));
  const double mean = 0.5 * (a + c), h = 0.5 * (a - c);
  const double d = sqrt(h * h + b * b);
  const double mu_hi = mean + d, mu_lo = mean - d;
  // eigenvector (p, q) of mu_hi in the (e, f) plane: the longer of (b, mu - a) and (mu - c, b)
  double p = b, q = mu_hi - a;
  const double p2 = mu_hi - c, q2 = b;
  if (p2 * p2 + q2 * q2 > p * p + q * q) { p = p2; q = q2; }
  const double pn = p * p + q * q;
  if (pn > 0.0) {
    const double ipn = 1.0 / sqrt(pn);
    p *= ipn; q *= ipn;
  } else {
    p = 1.0; q = 0.0;  // a multiple of the identity in the plane: any basis
  }
  // v_hi = p e + q f, v_lo = -q e + p f
  const double vh0 = p * e0 + q * f0, vh1 = p * e1 + q * f1, vh2 = p * e2 + q * f2;
  const double vl0 = p * f0 - q * e0, vl1 = p * f1 - q * e1, vl2 = p * f2 - q * e2;
  for (int k = 0; k < 9; ++k) out[k] = s[k];
  double d2 = 0.0;
  if (lam < kEpsPsd) {  // every eigenvalue clamped: V eps I V^T
    for (int k = 0; k < 9; ++k) out[k] = (k % 4 == 0) ? kEpsPsd : 0.0;
    d2 = (kEpsPsd - lam) * (kEpsPsd - lam) + (kEpsPsd - mu_hi) * (kEpsPsd - mu_hi) +
         (kEpsPsd - mu_lo) * (kEpsPsd - mu_lo);
  } else {
    if (mu_hi < kEpsPsd) {
      const double g = kEpsPsd - mu_hi;
      d2 += g * g;
      out[0] += g * vh0 * vh0; out[1] += g * vh0 * vh1; out[2] += g * vh0 * vh2;
      out[3] += g * vh1 * vh0; out[4] += g * vh1 * vh1; out[5] += g * vh1 * vh2;
      out[6] += g * vh2 * vh0; out[7] += g * vh2 * vh1; out[8] += g * vh2 * vh2;
    }
    if (mu_lo < kEpsPsd) {
      const double g = kEpsPsd - mu_lo;
      d2 += g * g;
      out[0] += g * vl0 * vl0; out[1] += g * vl0 * vl1; out[2] += g * vl0 * vl2;
      out[3] += g * vl1 * vl0; out[4] += g * vl1 * vl1; out[5] += g * vl1 * vl2;
      out[6] += g * vl2 * vl0; out[7] += g * vl2 * vl1; out[8] += g * vl2 * vl2;
    }
  }
  *delta = sqrt(d2);
  return true;
}

// DomainProjectionPSD for a 3x3 (primitives.py:80-123).  M_psd = V diag(max(w,eps)) V^T
// and the projection delta ||M_psd - M_sym||_F.  Exact fast path for the all-zero matrix
// (LAPACK returns V = I there, so the reference gives eps*I and delta = sqrt(3) eps exactly).
GCS_HD double psd_project3(const double* M, double* out) {
  double s[9];
  s[0] = M[0]; s[4] = M[4]; s[8] = M[8];
  s[1] = s[3] = 0.5 * (M[1] + M[3]);
  s[2] = s[6] = 0.5 * (M[2] + M[6]);
  s[5] = s[7] = 0.5 * (M[5] + M[7]);
  bool zero = true;
  for (int i = 0; i < 9; ++i) zero = zero && (s[i] == 0.0);
  if (zero) {
    for (int i = 0; i < 9; ++i) out[i] = (i % 4 == 0) ? kEpsPsd : 0.0;
    return 1.7320508075688772e-12;
  }
  GCS_PSD_COUNT(0);
  // Fast path: if M_sym - eps I is positive definite no eigenvalue is clamped, so the exact
  // projection is M_sym itself with delta 0 (the eigh rebuild differs only by rounding).
  {
    double a00 = s[0] - kEpsPsd;
    if (a00 > 0.0) {
      // (a positivity test: the reciprocals' last-ulp rounding only moves matrices within rounding of
      // a clamp between this exact path and the deflation, which agree there)
      double l00 = sqrt(a00), i00 = rcp_fast(l00), l10 = s[3] * i00, l20 = s[6] * i00;
      double a11 = s[4] - kEpsPsd - l10 * l10;
      if (a11 > 0.0) {
        double l11 = sqrt(a11), l21 = (s[7] - l20 * l10) * rcp_fast(l11);
        double a22 = s[8] - kEpsPsd - l20 * l20 - l21 * l21;
        if (a22 > 0.0) {
          for (int i = 0; i < 9; ++i) out[i] = s[i];
          return 0.0;
        }
      }
    }
  }
  // deflation inline, no call (so no private segment): at C3 about 6% of the non-empty bins (one to
  // three points) come here, so nearly every wave has such a lane
  GCS_PSD_COUNT(1);
  double dl;
  if (psd3_deflate(s, out, &dl)) return dl;
  GCS_PSD_COUNT(2);  // non-finite input: it propagates
  for (int i = 0; i < 9; ++i) out[i] = s[i] * NAN;
  return NAN;
}

// Inverse of a general 3x3 via adjugate / determinant (jnp.linalg.inv restated).
GCS_HD void inv3(const double* m, double* o) {
  double c00 = m[4] * m[8] - m[5] * m[7];
  double c01 = m[5] * m[6] - m[3] * m[8];
  double c02 = m[3] * m[7] - m[4] * m[6];
  double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  double id = 1.0 / det;
  o[0] = c00 * id;
  o[1] = (m[2] * m[7] - m[1] * m[8]) * id;
  o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  o[3] = c01 * id;
  o[4] = (m[0] * m[8] - m[2] * m[6]) * id;
  o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  o[6] = c02 * id;
  o[7] = (m[1] * m[6] - m[0] * m[7]) * id;
  o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// 3x3 SVD H = U diag(s) V^T by one-sided (Hestenes) Jacobi, s sorted descending.
// Columns of U for (numerically) zero singular values are completed orthonormally; the
// Matrix-Fisher consumer fixes det(U V^T) afterwards, so the completion sign is immaterial.
GCS_HD void svd3(const double* H, double* U, double* s, double* V) {
  double A[9];
  for (int i = 0; i < 9; ++i) { A[i] = H[i]; V[i] = (i % 4 == 0) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
    for (int pq = 0; pq < 3; ++pq) {
      int p = pq == 2 ? 1 : 0;
      int q = pq == 0 ? 1 : 2;
      double al = 0.0, be = 0.0, ga = 0.0;
      for (int k = 0; k < 3; ++k) {
        al += A[3 * k + p] * A[3 * k + p];
        be += A[3 * k + q] * A[3 * k + q];
        ga += A[3 * k + p] * A[3 * k + q];
      }
      if (ga == 0.0 || fabs(ga) <= 1e-17 * sqrt(al * be)) continue;
      rotated = true;
      double zeta = (be - al) / (2.0 * ga);
      double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      double c = 1.0 / sqrt(1.0 + t * t);
      double sn = c * t;
      for (int k = 0; k < 3; ++k) {
        double ap = A[3 * k + p], aq = A[3 * k + q];
        A[3 * k + p] = c * ap - sn * aq;
        A[3 * k + q] = sn * ap + c * aq;
        double vp = V[3 * k + p], vq = V[3 * k + q];
        V[3 * k + p] = c * vp - sn * vq;
        V[3 * k + q] = sn * vp + c * vq;
      }
    }
    if (!rotated) break;
  }
  double sv[3];
  int ord[3] = {0, 1, 2};
  for (int j = 0; j < 3; ++j) sv[j] = sqrt(A[j] * A[j] + A[3 + j] * A[3 + j] + A[6 + j] * A[6 + j]);
  // sort descending (stable on ties)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 2 - i; ++j)
      if (sv[ord[j]] < sv[ord[j + 1]]) { int tmp = ord[j]; ord[j] = ord[j + 1]; ord[j + 1] = tmp; }
  double Vs[9], As[9];
  for (int j = 0; j < 3; ++j) {
    s[j] = sv[ord[j]];
    for (int k = 0; k < 3; ++k) { Vs[3 * k + j] = V[3 * k + ord[j]]; As[3 * k + j] = A[3 * k + ord[j]]; }
  }
  for (int i = 0; i < 9; ++i) V[i] = Vs[i];
  double tiny = s[0] * 1e-13;
  int rank = 0;
  for (int j = 0; j < 3; ++j) {
    if (s[j] > tiny && s[j] > 0.0) {
      for (int k = 0; k < 3; ++k) U[3 * k + j] = As[3 * k + j] / s[j];
      rank = j + 1;
    }
  }
  if (rank == 0) {
    for (int i = 0; i < 9; ++i) U[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  double u0[3] = {U[0], U[3], U[6]};
  double u1[3];
  if (rank >= 2) {
    u1[0] = U[1]; u1[1] = U[4]; u1[2] = U[7];
  } else {
    // any unit vector orthogonal to u0: cross with the axis least aligned with it
    double ax[3] = {0.0, 0.0, 0.0};
    double a0 = fabs(u0[0]), a1 = fabs(u0[1]), a2 = fabs(u0[2]);
    ax[(a0 <= a1 && a0 <= a2) ? 0 : (a1 <= a2 ? 1 : 2)] = 1.0;
    cross3(u0, ax, u1);
    double n = sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
    for (int k = 0; k < 3; ++k) u1[k] /= n;
    U[1] = u1[0]; U[4] = u1[1]; U[7] = u1[2];
  }
  if (rank <= 2) {
    double u2[3];
    cross3(u0, u1, u2);
    U[2] = u2[0]; U[5] = u2[1]; U[8] = u2[2];
  }
}

GCS_HD double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// R_mf = U' V^T with U' = U with its last column multiplied by sign(det(U V^T)), H = U S V^T
// (matrix_fisher_evidence.py:215-222), through the Jacobi SVD.
GCS_HD void mf_rotation_svd(const double* H, double* R) {
  double U[9], s[3], V[9], UVt[9];
  svd3(H, U, s, V);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) UVt[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
  double dt = det3(UVt);
  double sg = dt > 0.0 ? 1.0 : (dt < 0.0 ? -1.0 : 0.0);
  U[2] *= sg; U[5] *= sg; U[8] *= sg;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
}

// Same R_mf.  When det(H) > 0 and H is not nearly singular, det(U V^T) = +1 and R_mf is the
// orthogonal polar factor of H: the scaled Newton iteration X <- (g X + X^{-T} / g) / 2,
// g = (|X^{-1}|_F / |X|_F)^{1/2}, reaches it in a handful of 3x3 adjugate steps (quadratic
// convergence) -- a short dependent chain on one GPU thread.  Reflections and rank-deficient H
// take the SVD.
GCS_HD void mf_rotation(const double* H, double* R) {
  double fro2 = 0.0;
  for (int k = 0; k < 9; ++k) fro2 += H[k] * H[k];
  const double fro = sqrt(fro2);
  const double d0 = det3(H);
  if (!(fro > 0.0) || !(d0 > 1e-6 * fro2 * fro)) {
    mf_rotation_svd(H, R);
    return;
  }
  double X[9];
  for (int k = 0; k < 9; ++k) X[k] = H[k];
  bool polish = false;
  for (int it = 0; it < 60; ++it) {
    double C[9] = {X[4] * X[8] - X[5] * X[7], X[5] * X[6] - X[3] * X[8], X[3] * X[7] - X[4] * X[6],
                   X[2] * X[7] - X[1] * X[8], X[0] * X[8] - X[2] * X[6], X[1] * X[6] - X[0] * X[7],
                   X[1] * X[5] - X[2] * X[4], X[2] * X[3] - X[0] * X[5], X[0] * X[4] - X[1] * X[3]};
    const double dx = X[0] * C[0] + X[1] * C[1] + X[2] * C[2];  // C / dx = X^{-T}
    double g = 1.0;
    if (!polish) {
      double nx = 0.0, nc = 0.0;
      for (int k = 0; k < 9; ++k) { nx += X[k] * X[k]; nc += C[k] * C[k]; }
      g = sqrt(sqrt(nc / nx) / fabs(dx));
    }
    const double a = 0.5 * g, b = 0.5 / (g * dx);
    double diff = 0.0;
    for (int k = 0; k < 9; ++k) {
      const double xn = a * X[k] + b * C[k];
      diff += (xn - X[k]) * (xn - X[k]);
      X[k] = xn;
    }
    if (polish) break;             // one unscaled step after convergence
    if (diff <= 1e-24) polish = true;
  }
  for (int k = 0; k < 9; ++k) R[k] = X[k];
}

// ---------------------------------------------------------------------------- short log / exp
// f64 log and exp for finite arguments in the Sinkhorn scalings' range (the classic
// reduction + minimax polynomials of the 4.4BSD / fdlibm e_log.c and e_exp.c, < 1 ulp): about a
// third of the library's instruction count (its log carries double-double steps), which is what a
// one-workgroup Sinkhorn iteration spends its time on.  No contraction: host and device round alike.
GCS_HD double log_short(double x) {  // x > 0, finite, normal
#pragma clang fp contract(off)
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int e;
  double m = frexp(x, &e);  // [0.5, 1)
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  const double f = m - 1.0;
  const double hfsq = 0.5 * f * f;
  const double s = f / (2.0 + f);
  const double dk = (double)e;
  const double z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

GCS_HD double exp_short(double x) {  // |x| < 700
#pragma clang fp contract(off)
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
  const int k = (int)(invln2 * x + (x < 0.0 ? -0.5 : 0.5));
  const double t = (double)k;
  const double hi = x - t * ln2_hi, lo = t * ln2_lo;
  const double r = hi - lo;
  const double rr = r * r;
  const double c = r - rr * (P1 + rr * (P2 + rr * (P3 + rr * (P4 + rr * P5))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return ldexp(y, k);
}

// Table-driven f64 log / exp for the Sinkhorn loop (about half of log_short / exp_short's operations,
// no divide): the argument reduced by a 129- / 64-entry table (gcs_sh_tables.h, passed in -- the
// kernel reads its LDS copy) to |f| < 2^-8 / |r| < ln2 / 128, where a degree-7 log1p / degree-5 expm1
// Taylor polynomial is below an ulp (truncation ~2e-18 / 4e-17 relative).  Within ~1 ulp of the
// library; host and device round alike (explicit fma, no contraction).
// (each split in two: the reduction with its table index, then the polynomial on the table values --
// a caller with several arguments issues every table read before the first polynomial)
GCS_HD void log_tab_reduce(double x, double& m, int& e, int& j) {  // x > 0, finite, normal
  uint64_t b;
  memcpy(&b, &x, 8);
  e = (int)(b >> 52) - 1023;
  const uint64_t mb = b & 0x000fffffffffffffull;
  j = (int)((mb + (1ull << 44)) >> 45);  // nearest 1/128 of the mantissa: 0..128
  const uint64_t mbits = mb | 0x3ff0000000000000ull;
  memcpy(&m, &mbits, 8);  // [1, 2)
}
GCS_HD double log_tab_poly(double m, int e, double inv_c, double l_hi, double l_lo) {
#pragma clang fp contract(off)
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double f = fma(m, inv_c, -1.0);  // m inv_c_j - 1 (exact product, one rounding)
  const double p = f * f *
                   fma(f, fma(f, fma(f, fma(f, fma(f, 1.0 / 7.0, -1.0 / 6.0), 0.2), -0.25), 1.0 / 3.0), -0.5);
  const double dk = (double)e;
  return fma(dk, ln2_hi, l_hi) + (f + (p + fma(dk, ln2_lo, l_lo)));
}
GCS_HD double log_tab(double x, const double* lt) {  // x > 0, finite, normal
  double m;
  int e, j;
  log_tab_reduce(x, m, e, j);
  return log_tab_poly(m, e, lt[3 * j], lt[3 * j + 1], lt[3 * j + 2]);
}
GCS_HD void exp_tab_reduce(double x, double& r, int& j, int& m) {  // |x| < 700
#pragma clang fp contract(off)
  const double kd = rint(x * kSh64ByLn2);
  const int k = (int)kd;
  r = fma(-kd, kShLn2By64Lo, fma(-kd, kShLn2By64Hi, x));
  j = k & 63;
  m = k >> 6;  // k = 64 m + j (arithmetic shift: floor)
}
GCS_HD double exp_tab_poly(double r, int m, double t_hi, double t_lo) {
#pragma clang fp contract(off)
  const double p = fma(r * r, fma(r, fma(r, fma(r, 1.0 / 120.0, 1.0 / 24.0), 1.0 / 6.0), 0.5), r);  // expm1(r)
  return ldexp(t_hi + fma(t_hi, p, t_lo), m);
}
GCS_HD double exp_tab(double x, const double* et) {  // |x| < 700
  double r;
  int j, m;
  exp_tab_reduce(x, r, j, m);
  return exp_tab_poly(r, m, et[2 * j], et[2 * j + 1]);
}

// x^y for the Sinkhorn scalings: 0 at x = 0, exp_short(y log_short(x)) for positive finite normal
// x and |y log x| < 700, the library pow otherwise (a few ulps from pow: |y log x| < ~40 here)
// The library pow out of line: inlined at each of the Sinkhorn loop's five call sites it made the
// loop body too large for the instruction cache.
__host__ __device__ __attribute__((noinline)) inline double pow_lib(double x, double y) { return pow(x, y); }
GCS_HD double pow_sinkhorn(double x, double y) {
  if (x == 0.0) return 0.0;
  if (!(x >= 2.2250738585072014e-308) || !(x <= 1.7976931348623157e308)) return pow_lib(x, y);
  const double a = y * log_short(x);
  if (!(fabs(a) < 700.0)) return pow_lib(x, y);
  return exp_short(a);
}

}  // namespace gcs
