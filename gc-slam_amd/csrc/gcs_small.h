// Small dense symmetric algebra (n <= 6) shared by host and device code: the host numerics'
// algorithms (gcs_host.cpp jacobi_eigh, psd_project with its fast paths, the right-looking Cholesky
// and the lifted inverse) restated on fixed-size arrays as __host__ __device__ routines, so the
// IMU / odometry evidence factors (gcs_imu_odom_core.h) run the same code on the host and in the
// device kernel (gcs_imu_odom.hip).  References: FS/common/primitives.py:80-123 (psd projection),
// :141-192 (lifted Cholesky solve / inverse).
#pragma once
#include "gcs_math.h"

namespace gcs {
namespace small {

constexpr int kN = 6;

// Each routine takes its size as a template argument NC when it is known at the call (the loops then unroll
// and the device keeps the arrays in registers), or NC = 0 and the run-time n (the zero-row split below).

// cyclic Jacobi, row-major n x n; w unsorted, V columns (gcs_host.cpp jacobi_eigh)
template <int NC>
GCS_HD void jacobi_eigh(int n_rt, const double* A, double* w, double* V) {
  const int n = NC ? NC : n_rt;
  double a[kN * kN];
  for (int i = 0; i < n * n; ++i) a[i] = A[i];
  for (int i = 0; i < n * n; ++i) V[i] = 0.0;
  for (int i = 0; i < n; ++i) V[i * n + i] = 1.0;
  double fro = 0.0;
  for (int i = 0; i < n * n; ++i) fro += a[i] * a[i];
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
    if (off == 0.0 || off <= 1e-36 * fro) break;
    for (int p = 0; p < n - 1; ++p) {
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (apq == 0.0) continue;
        const double app = a[p * n + p], aqq = a[q * n + q];
        if (fabs(apq) < 1e-18 * sqrt(fabs(app * aqq)) && sweep > 3) {
          a[p * n + q] = a[q * n + p] = 0.0;
          continue;
        }
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        a[p * n + q] = a[q * n + p] = 0.0;
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
    }
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

// right-looking Cholesky of A (row-major lower factor Lc, reciprocal diagonals rd): the operation order
// of gcs_host.cpp cholesky_n<N>; false when a pivot is not positive
template <int NC>
GCS_HD bool cholesky(int n_rt, const double* A, double* Lc, double* rd) {
  const int n = NC ? NC : n_rt;
  double W[kN * kN], col[kN];
  for (int i = 0; i < n * n; ++i) W[i] = A[i];
  for (int j = 0; j < n; ++j) {
    const double s = W[j * n + j];
    if (!(s > 0.0)) return false;
    const double d = sqrt(s), r = 1.0 / d;
    rd[j] = r;
    col[j] = d;
    for (int i = j + 1; i < n; ++i) col[i] = W[i * n + j] * r;
    for (int i = j + 1; i < n; ++i) {
      const double li = col[i];
      for (int k = j + 1; k <= i; ++k) W[i * n + k] -= li * col[k];
    }
    for (int i = 0; i < j; ++i) Lc[i * n + j] = 0.0;
    for (int i = j; i < n; ++i) Lc[i * n + j] = col[i];
  }
  return true;
}

// (L + eps_lift I)^{-1} through its Cholesky factor (gcs_host.cpp spd_factor_lifted + factor_inverse_n);
// a matrix not positive definite even lifted gives NaN, which the callers' finiteness checks report
template <int NC>
GCS_HD void spd_inverse_lifted(const double* L, double eps_lift, double* Linv) {
  constexpr int n = NC;
  double A[kN * kN], Lc[kN * kN], rd[kN];
  for (int i = 0; i < n * n; ++i) A[i] = L[i];
  for (int i = 0; i < n; ++i) A[i * n + i] += eps_lift;
  if (!cholesky<NC>(n, A, Lc, rd))
    for (int i = 0; i < n; ++i) rd[i] = NAN;
  double X[kN * kN], R[kN * kN];
  for (int i = 0; i < n; ++i) {
    double xi[kN];
    for (int c = 0; c < n; ++c) xi[c] = 0.0;
    for (int k = 0; k < i; ++k) {
      const double l = Lc[i * n + k];
      for (int c = 0; c <= k; ++c) xi[c] -= l * X[k * n + c];
    }
    xi[i] = 1.0;
    for (int c = 0; c <= i; ++c) xi[c] *= rd[i];
    for (int c = 0; c < n; ++c) X[i * n + c] = xi[c];
  }
  for (int i = 0; i < n * n; ++i) R[i] = 0.0;
  for (int k = 0; k < n; ++k)
    for (int i = 0; i <= k; ++i) {
      const double xi = X[k * n + i];
      for (int j = 0; j <= i; ++j) R[i * n + j] += xi * X[k * n + j];
    }
  for (int i = 0; i < n * n; ++i) Linv[i] = R[i];
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) Linv[i * n + j] = Linv[j * n + i];
}

// domain_projection_psd_core (primitives.py:80-123) with the host's declared fast paths (DESIGN.md
// section 3 item 5): exactly-zero rows split off, and sym(M) returned when sym(M) - eps I has a
// Cholesky factor; cert6 (the certificate form) always takes the eigen-decomposition.
template <int NC>
GCS_HD double psd_project(const double* M, double eps_psd, double* out, double* cert6 = nullptr) {
  constexpr int n = NC;
  double s[kN * kN];
  double sym2 = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      s[i * n + j] = 0.5 * (M[i * n + j] + M[j * n + i]);
      const double d = s[i * n + j] - M[i * n + j];
      sym2 += d * d;
    }
  double w[kN], V[kN * kN];
  if (!cert6) {
    // the exactly-zero rows split off (the host's compacted active block), here in place: the active
    // block keeps its indices, an inactive row / column is the identity in the Cholesky test (its pivot
    // 1, its column 0: the active entries take the compact factorisation's operations) and zero in the
    // Jacobi (its pairs are skipped, so the active pairs rotate in the compact order).  Every index is
    // static, so the device keeps the arrays in registers.
    bool act[kN];
    int na = 0;
    for (int i = 0; i < n; ++i) {
      bool z = true;
      for (int j = 0; j < n; ++j) z = z && s[i * n + j] == 0.0;
      act[i] = !z;
      na += z ? 0 : 1;
    }
    if (na < n) {
      for (int i = 0; i < n * n; ++i) out[i] = 0.0;
      for (int i = 0; i < n; ++i) out[i * n + i] = eps_psd;
      double d2 = (double)(n - na) * eps_psd * eps_psd;
      if (na > 0) {
        double sub[kN * kN], A[kN * kN], Lc[kN * kN], rd[kN];
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < n; ++j) {
            const bool aa = act[i] && act[j];
            sub[i * n + j] = aa ? 0.5 * (s[i * n + j] + s[j * n + i]) : 0.0;
            A[i * n + j] = aa ? sub[i * n + j] - (i == j ? eps_psd : 0.0) : (i == j ? 1.0 : 0.0);
          }
        double da = 0.0;
        if (cholesky<NC>(n, A, Lc, rd)) {
          for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j)
              if (act[i] && act[j]) out[i * n + j] = sub[i * n + j];
        } else {
          jacobi_eigh<NC>(n, sub, w, V);
          for (int k = 0; k < n; ++k) w[k] = w[k] > eps_psd ? w[k] : eps_psd;
          double dd2 = 0.0;
          for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
              if (!(act[i] && act[j])) continue;
              double v = 0.0;
              for (int k = 0; k < n; ++k)
                if (act[k]) v += V[i * n + k] * w[k] * V[j * n + k];
              out[i * n + j] = v;
              const double dd = v - sub[i * n + j];
              dd2 += dd * dd;
            }
          da = sqrt(dd2);
        }
        d2 += da * da;
      }
      return sqrt(d2);
    }
    double A[kN * kN], Lc[kN * kN], rd[kN];
    for (int i = 0; i < n * n; ++i) A[i] = s[i];
    for (int i = 0; i < n; ++i) A[i * n + i] -= eps_psd;
    if (cholesky<NC>(n, A, Lc, rd)) {
      for (int i = 0; i < n * n; ++i) out[i] = s[i];
      return 0.0;
    }
  }
  bool zero = true;
  for (int i = 0; i < n * n; ++i) zero = zero && s[i] == 0.0;
  if (zero) {
    for (int i = 0; i < n * n; ++i) V[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
    for (int i = 0; i < n; ++i) w[i] = 0.0;
  } else {
    jacobi_eigh<NC>(n, s, w, V);
  }
  double emin = INFINITY, emax = -INFINITY, nn = 0.0;
  for (int k = 0; k < n; ++k) {
    w[k] = w[k] > eps_psd ? w[k] : eps_psd;
    emin = w[k] < emin ? w[k] : emin;
    emax = w[k] > emax ? w[k] : emax;
    nn += (w[k] < 10.0 * eps_psd) ? 1.0 : 0.0;
  }
  double d2 = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double v = 0.0;
      for (int k = 0; k < n; ++k) v += V[i * n + k] * w[k] * V[j * n + k];
      out[i * n + j] = v;
      const double dd = v - s[i * n + j];
      d2 += dd * dd;
    }
  const double delta = sqrt(d2);
  if (cert6) {
    cert6[0] = delta; cert6[1] = sqrt(sym2); cert6[2] = emin; cert6[3] = emax; cert6[4] = emax / emin; cert6[5] = nn;
  }
  return delta;
}

// se3_compose / se3_inverse (se3_jax.py:405-438), as gcs_host.cpp
GCS_HD void se3_compose(const double* a, const double* b, double* out) {
  double Ra[9], Rb[9], R[9];
  so3_exp(a + 3, Ra);
  so3_exp(b + 3, Rb);
  mat3_mul(Ra, Rb, R);
  for (int i = 0; i < 3; ++i) out[i] = a[i] + Ra[3 * i] * b[0] + Ra[3 * i + 1] * b[1] + Ra[3 * i + 2] * b[2];
  so3_log(R, out + 3);
}
GCS_HD void se3_inverse(const double* a, double* out) {
  double R[9], Rt[9];
  so3_exp(a + 3, R);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
  for (int i = 0; i < 3; ++i) out[i] = -(Rt[3 * i] * a[0] + Rt[3 * i + 1] * a[1] + Rt[3 * i + 2] * a[2]);
  so3_log(Rt, out + 3);
}

}  // namespace small
}  // namespace gcs
