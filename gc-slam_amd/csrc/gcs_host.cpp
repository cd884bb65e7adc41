// Host 22-D numerics (see gcs_host.h).  Each function cites the reference it restates.
#include "gcs_host.h"

#include <math.h>
#include <string.h>

#include <algorithm>

#include "gcs_math.h"

namespace gcs {
namespace host {

void jacobi_eigh(int n, const double* A, double* w, double* V) {
  double a[kMaxN * kMaxN];
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
        double apq = a[p * n + q];
        if (apq == 0.0) continue;
        double app = a[p * n + p], aqq = a[q * n + q];
        if (fabs(apq) < 1e-18 * sqrt(fabs(app * aqq)) && sweep > 3) {
          a[p * n + q] = a[q * n + p] = 0.0;
          continue;
        }
        double theta = (aqq - app) / (2.0 * apq);
        double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        a[p * n + q] = a[q * n + p] = 0.0;
        for (int k = 0; k < n; ++k) {
          double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
    }
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

template <int N>
static bool cholesky_n(const double* A, double* Lc, double* rd);

// psd_project's fast path (b) at the belief's order: sym(M), then the Cholesky test of sym(M) - eps I
// (no zero-row split: a row of the 22-D information / covariance is never exactly zero when the
// test passes, and a failing test falls back to the general path, which splits them)
static bool psd_fast_22(const double* M, double eps_psd, double* out) {
  constexpr int N = DZ;
  double A[N * N], Lc[N * N], rd[N];
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) out[i * N + j] = 0.5 * (M[i * N + j] + M[j * N + i]);
  for (int i = 0; i < N * N; ++i) A[i] = out[i];
  for (int i = 0; i < N; ++i) A[i * N + i] -= eps_psd;
  return cholesky_n<N>(A, Lc, rd);
}

// domain_projection_psd_core, FS/common/primitives.py:80-123
double psd_project(int n, const double* M, double eps_psd, double* out, double* cert6) {
  if (!cert6 && n == DZ) {
    // a zero row of sym(M) makes sym(M) - eps I indefinite, so a passing test already excludes
    // case (a) below: the result is the general fast path's
    if (psd_fast_22(M, eps_psd, out)) return 0.0;
  }
  double s[kMaxN * kMaxN];
  double sym2 = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      s[i * n + j] = 0.5 * (M[i * n + j] + M[j * n + i]);
      double d = s[i * n + j] - M[i * n + j];
      sym2 += d * d;
    }
  if (!cert6) {
    // Fast paths (declared, DESIGN.md "PSD fast path"); the certificate form always runs eigh.
    // (a) exactly-zero rows/columns split off: eigh of [A 0; 0 0] is eigh(A) plus exact zero
    //     eigenvalues, each clamped to eps_psd on the diagonal (IW padded blocks, masked evidence).
    int act[kMaxN], na = 0;
    for (int i = 0; i < n; ++i) {
      bool z = true;
      for (int j = 0; j < n && z; ++j) z = s[i * n + j] == 0.0;
      if (!z) act[na++] = i;
    }
    if (na < n) {
      for (int i = 0; i < n * n; ++i) out[i] = 0.0;
      for (int i = 0; i < n; ++i) out[i * n + i] = eps_psd;
      double d2 = (double)(n - na) * eps_psd * eps_psd;
      if (na > 0) {
        double sub[kMaxN * kMaxN], so[kMaxN * kMaxN];
        for (int i = 0; i < na; ++i)
          for (int j = 0; j < na; ++j) sub[i * na + j] = s[act[i] * n + act[j]];
        double da = psd_project(na, sub, eps_psd, so, nullptr);
        for (int i = 0; i < na; ++i)
          for (int j = 0; j < na; ++j) out[act[i] * n + act[j]] = so[i * na + j];
        d2 += da * da;
      }
      return sqrt(d2);
    }
    // (b) M_sym - eps I positive definite -> no eigenvalue is clamped: return M_sym, delta 0
    double A[kMaxN * kMaxN], Lc[kMaxN * kMaxN];
    for (int i = 0; i < n * n; ++i) A[i] = s[i];
    for (int i = 0; i < n; ++i) A[i * n + i] -= eps_psd;
    if (cholesky(n, A, Lc)) {
      for (int i = 0; i < n * n; ++i) out[i] = s[i];
      return 0.0;
    }
  }
  double w[kMaxN], V[kMaxN * kMaxN];
  bool zero = true;
  for (int i = 0; i < n * n; ++i) zero = zero && s[i] == 0.0;
  if (zero) {
    for (int i = 0; i < n * n; ++i) V[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
    for (int i = 0; i < n; ++i) w[i] = 0.0;
  } else {
    jacobi_eigh(n, s, w, V);
  }
  double emin = INFINITY, emax = -INFINITY, nn = 0.0;
  for (int k = 0; k < n; ++k) {
    w[k] = w[k] > eps_psd ? w[k] : eps_psd;
    emin = std::min(emin, w[k]);
    emax = std::max(emax, w[k]);
    nn += (w[k] < 10.0 * eps_psd) ? 1.0 : 0.0;
  }
  double d2 = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double v = 0.0;
      for (int k = 0; k < n; ++k) v += V[i * n + k] * w[k] * V[j * n + k];
      out[i * n + j] = v;
      double dd = v - s[i * n + j];
      d2 += dd * dd;
    }
  double delta = sqrt(d2);
  if (cert6) {
    cert6[0] = delta; cert6[1] = sqrt(sym2); cert6[2] = emin; cert6[3] = emax; cert6[4] = emax / emin; cert6[5] = nn;
  }
  return delta;
}

// Cholesky / triangular solves / inverse, specialised on the size (22 for the belief, 6 and 3 for
// the blocks) so the inner products unroll over contiguous rows; reciprocal diagonals replace the
// divisions.  Row-major lower factor; Ct holds Lc^{-1} transposed (row c = column c of Lc^{-1}).
// Right-looking: after column j every trailing element has subtracted L[i][j] L[k][j].  Each element
// sees the same operation sequence as the left-looking dot products (A - L0 L0 - L1 L1 ...), so the
// factor is bitwise the same, but the subtractions of one column step are independent of each other
// (a vectorisable sweep instead of a chain of dependent subtractions per element: 1.6 -> 0.4 us).
template <int N>
static bool cholesky_n(const double* A, double* Lc, double* rd) {
  double W[N * N], col[N];
  for (int i = 0; i < N * N; ++i) W[i] = A[i];
  for (int j = 0; j < N; ++j) {
    const double s = W[j * N + j];
    if (!(s > 0.0)) return false;
    const double d = sqrt(s), r = 1.0 / d;
    rd[j] = r;
    col[j] = d;
    for (int i = j + 1; i < N; ++i) col[i] = W[i * N + j] * r;
    for (int i = j + 1; i < N; ++i) {
      const double li = col[i];
      double* __restrict__ Wi = W + i * N;
      for (int k = j + 1; k <= i; ++k) Wi[k] -= li * col[k];
    }
    for (int i = 0; i < j; ++i) Lc[i * N + j] = 0.0;
    for (int i = j; i < N; ++i) Lc[i * N + j] = col[i];
  }
  return true;
}

static bool cholesky_dyn(int n, const double* A, double* Lc, double* rd) {
  for (int i = 0; i < n * n; ++i) Lc[i] = 0.0;
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= Lc[j * n + k] * Lc[j * n + k];
    if (!(s > 0.0)) return false;
    const double d = sqrt(s), r = 1.0 / d;
    Lc[j * n + j] = d;
    rd[j] = r;
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= Lc[i * n + k] * Lc[j * n + k];
      Lc[i * n + j] = t * r;
    }
  }
  return true;
}

static bool cholesky_rd(int n, const double* A, double* Lc, double* rd) {
  switch (n) {
    case DZ: return cholesky_n<DZ>(A, Lc, rd);
    case 6: return cholesky_n<6>(A, Lc, rd);
    case 3: return cholesky_n<3>(A, Lc, rd);
    default: return cholesky_dyn(n, A, Lc, rd);
  }
}

bool cholesky(int n, const double* A, double* Lc) {
  double rd[kMaxN];
  return cholesky_rd(n, A, Lc, rd);
}

// spd_cholesky_solve_lifted_core / spd_cholesky_inverse_lifted_core, primitives.py:141-192
void spd_factor_lifted(int n, const double* L, double eps_lift, SpdFactor& f) {
  double A[kMaxN * kMaxN];
  for (int i = 0; i < n * n; ++i) A[i] = L[i];
  for (int i = 0; i < n; ++i) A[i * n + i] += eps_lift;
  f.n = n;
  if (!cholesky_rd(n, A, f.Lc, f.rd))  // not PD even lifted: NaN propagates to the callers' checks
    for (int i = 0; i < n; ++i) f.rd[i] = NAN;
}

template <int N>
static void factor_solve_n(const double* Lc, const double* rd, const double* b, double* x) {
  // forward substitution by columns: y_i = (b_i - L_i0 y_0 - L_i1 y_1 ...) / L_ii, the row form's
  // operation order per element, with the updates of one step independent
  double y[N];
  for (int i = 0; i < N; ++i) y[i] = b[i];
  for (int j = 0; j < N; ++j) {
    const double yj = y[j] * rd[j];
    y[j] = yj;
    for (int i = j + 1; i < N; ++i) y[i] -= Lc[i * N + j] * yj;
  }
  // back substitution by columns of Lc (row-major rows of Lc^T): x_i = (y_i - sum_k>i Lc[k][i] x_k) / Lc[i][i]
  for (int i = N - 1; i >= 0; --i) {
    const double xi = y[i] * rd[i];
    x[i] = xi;
    const double* Li = Lc + i * N;
    for (int k = 0; k < i; ++k) y[k] -= Li[k] * xi;
  }
}

void spd_factor_solve(const SpdFactor& f, const double* b, double* x) {
  const int n = f.n;
  if (n == DZ) return factor_solve_n<DZ>(f.Lc, f.rd, b, x);
  if (n == 6) return factor_solve_n<6>(f.Lc, f.rd, b, x);
  const double* Lc = f.Lc;
  double y[kMaxN];
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= Lc[i * n + k] * y[k];
    y[i] = s * f.rd[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    const double xi = y[i] * f.rd[i];
    x[i] = xi;
    for (int k = 0; k < i; ++k) y[k] -= Lc[i * n + k] * xi;
  }
}

template <int N>
static void factor_inverse_n(const double* Lc, const double* rd, double* Linv) {
  // X = Lc^{-1} row by row (X_i = (e_i - sum_k<i Lc[i][k] X_k) / Lc[i][i]: row AXPYs), then
  // Linv = X^T X as rank-1 updates over the rows of X; both inner loops are contiguous and independent
  // (the row under construction lives in its own buffer, so its AXPYs provably do not alias the
  // finished rows they read and vectorise)
  double X[N * N], R[N * N];
  for (int i = 0; i < N; ++i) {
    double xi[N];
    for (int c = 0; c < N; ++c) xi[c] = 0.0;
    const double* Li = Lc + i * N;
    for (int k = 0; k < i; ++k) {
      const double l = Li[k];
      const double* Xk = X + k * N;
      for (int c = 0; c <= k; ++c) xi[c] -= l * Xk[c];
    }
    xi[i] = 1.0;
    for (int c = 0; c <= i; ++c) xi[c] *= rd[i];
    for (int c = 0; c < N; ++c) X[i * N + c] = xi[c];
  }
  for (int i = 0; i < N * N; ++i) R[i] = 0.0;
  for (int k = 0; k < N; ++k) {
    const double* Xk = X + k * N;
    for (int i = 0; i <= k; ++i) {
      const double xi = Xk[i];
      double* __restrict__ Ri = R + i * N;
      for (int j = 0; j <= i; ++j) Ri[j] += xi * Xk[j];
    }
  }
  for (int i = 0; i < N * N; ++i) Linv[i] = R[i];
  for (int i = 0; i < N; ++i)
    for (int j = i + 1; j < N; ++j) Linv[i * N + j] = Linv[j * N + i];
}

void spd_factor_inverse(const SpdFactor& f, double* Linv) {
  const int n = f.n;
  if (n == DZ) return factor_inverse_n<DZ>(f.Lc, f.rd, Linv);
  if (n == 6) return factor_inverse_n<6>(f.Lc, f.rd, Linv);
  if (n == 3) return factor_inverse_n<3>(f.Lc, f.rd, Linv);
  const double* Lc = f.Lc;
  double Ct[kMaxN * kMaxN];
  for (int c = 0; c < n; ++c) {
    double* C = Ct + c * n;
    for (int i = 0; i < c; ++i) C[i] = 0.0;
    C[c] = f.rd[c];
    for (int i = c + 1; i < n; ++i) {
      double s = 0.0;
      for (int k = c; k < i; ++k) s -= Lc[i * n + k] * C[k];
      C[i] = s * f.rd[i];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = i; j < n; ++j) {
      double s = 0.0;
      for (int k = j; k < n; ++k) s += Ct[i * n + k] * Ct[j * n + k];
      Linv[i * n + j] = s;
      Linv[j * n + i] = s;
    }
}

void spd_solve_lifted(int n, const double* L, const double* b, double eps_lift, double* x) {
  SpdFactor f;
  spd_factor_lifted(n, L, eps_lift, f);
  spd_factor_solve(f, b, x);
}

void spd_inverse_lifted(int n, const double* L, double eps_lift, double* Linv) {
  SpdFactor f;
  spd_factor_lifted(n, L, eps_lift, f);
  spd_factor_inverse(f, Linv);
}

void solve3(const double* A, const double* b, double* x) {
  double M[3][4];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) M[i][j] = A[3 * i + j];
    M[i][3] = b[i];
  }
  for (int c = 0; c < 3; ++c) {
    int piv = c;
    for (int r = c + 1; r < 3; ++r)
      if (fabs(M[r][c]) > fabs(M[piv][c])) piv = r;
    if (piv != c)
      for (int j = 0; j < 4; ++j) std::swap(M[c][j], M[piv][j]);
    for (int r = c + 1; r < 3; ++r) {
      double f = M[r][c] / M[c][c];
      for (int j = c; j < 4; ++j) M[r][j] -= f * M[c][j];
    }
  }
  for (int i = 2; i >= 0; --i) {
    double s = M[i][3];
    for (int j = i + 1; j < 3; ++j) s -= M[i][j] * x[j];
    x[i] = s / M[i][i];
  }
}

// se3_compose, se3_jax.py:405-424
void se3_compose(const double* a, const double* b, double* out) {
  double Ra[9], Rb[9], R[9];
  so3_exp(a + 3, Ra);
  so3_exp(b + 3, Rb);
  mat3_mul(Ra, Rb, R);
  for (int i = 0; i < 3; ++i) out[i] = a[i] + Ra[3 * i] * b[0] + Ra[3 * i + 1] * b[1] + Ra[3 * i + 2] * b[2];
  so3_log(R, out + 3);
}

// se3_inverse, se3_jax.py:427-438
void se3_inverse(const double* a, double* out) {
  double R[9], Rt[9];
  so3_exp(a + 3, R);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
  for (int i = 0; i < 3; ++i) out[i] = -(Rt[3 * i] * a[0] + Rt[3 * i + 1] * a[1] + Rt[3 * i + 2] * a[2]);
  so3_log(Rt, out + 3);
}

// se3_log, se3_jax.py:210-245: the shared host/device routine (gcs_math.h se3_log_hd)
void se3_log(const double* T, double* out) { se3_log_hd(T, out); }

// BeliefGaussianInfo.mean_increment / mean_world_pose, belief.py:373-434
void mean_increment(const Belief& b, double* dz) { spd_solve_lifted(DZ, b.L, b.h, kEpsLift, dz); }

void world_pose_from_increment(const Belief& b, const double* dz, double* pose6) {
  double e[6];
  se3_exp(dz, e);
  se3_compose(b.X_anchor, e, pose6);
}

void mean_world_pose(const Belief& b, double* pose6) {
  double dz[DZ];
  mean_increment(b, dz);
  world_pose_from_increment(b, dz, pose6);
}

// _predict_diffusion_core, predict.py:43-103
void predict_diffusion(const Belief& prev, const double* Q, double dt, Belief& pred, double* infl3,
                       double* mean_prev_out, const SpdFactor* prev_fac, const double* prev_cov) {
  const int n = DZ;
  double mean_prev[DZ], cov_buf[DZ * DZ], cov_raw[DZ * DZ], cov_psd[DZ * DZ], Lp[DZ * DZ], Lpsd[DZ * DZ];
  const double* cov_prev = prev_cov;
  if (prev_fac && prev_cov) {
    spd_factor_solve(*prev_fac, prev.h, mean_prev);
  } else {
    SpdFactor f;
    spd_factor_lifted(n, prev.L, kEpsLift, f);
    spd_factor_solve(f, prev.h, mean_prev);
    spd_factor_inverse(f, cov_buf);
    cov_prev = cov_buf;
  }
  const double lam = 0.1;  // GC_OU_DAMPING_LAMBDA, constants.py:248
  double ef = exp(-2.0 * lam * dt);
  double dc = (1.0 - ef) / (2.0 * lam + kF64Eps);
  for (int i = 0; i < n * n; ++i) cov_raw[i] = ef * cov_prev[i] + dc * Q[i];
  double d1 = psd_project(n, cov_raw, kEpsPsd, cov_psd);
  spd_inverse_lifted(n, cov_psd, kEpsLift, Lp);
  double d2 = psd_project(n, Lp, kEpsPsd, Lpsd);
  memcpy(pred.X_anchor, prev.X_anchor, sizeof(pred.X_anchor));
  pred.stamp = prev.stamp + dt;
  memcpy(pred.z_lin, prev.z_lin, sizeof(pred.z_lin));
  memcpy(pred.L, Lpsd, sizeof(pred.L));
  for (int i = 0; i < n; ++i) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += Lpsd[i * n + j] * mean_prev[j];
    pred.h[i] = s;
  }
  infl3[0] = 2.0 * kEpsLift * n;
  infl3[1] = d1 + d2;
  infl3[2] = dt;
  if (mean_prev_out) memcpy(mean_prev_out, mean_prev, sizeof(mean_prev));
}

// preintegrate_imu_relative_pose_jax, imu_preintegration.py:47-147
void preintegrate_imu(int m, const double* stamps, const double* gyro, const double* accel, const double* w,
                      const double* rotvec_start, const double* gb, const double* ab, const double* g, PreintOut& out) {
  double R[9], v[3] = {0, 0, 0}, p[3] = {0, 0, 0};
  so3_exp(rotvec_start, R);
  double ess = 0.0;
  for (int i = 0; i < m; ++i) ess += w[i];
  for (int i = 0; i < m; ++i) {
    double dt = (i + 1 < m) ? stamps[i + 1] - stamps[i] : 0.0;
    dt = dt > 0.0 ? dt : 0.0;
    double dte = w[i] * dt;
    // dte == 0 (padding slots, last sample) is an exact identity step: Exp(0) = I, v and p unchanged
    if (dte == 0.0) continue;
    double om[3] = {(gyro[3 * i] - gb[0]) * dte, (gyro[3 * i + 1] - gb[1]) * dte, (gyro[3 * i + 2] - gb[2]) * dte};
    double dR[9], Rn[9];
    so3_exp(om, dR);
    mat3_mul(R, dR, Rn);
    double a_body[3] = {accel[3 * i] - ab[0], accel[3 * i + 1] - ab[1], accel[3 * i + 2] - ab[2]};
    double aw[3];
    for (int k = 0; k < 3; ++k) aw[k] = R[3 * k] * a_body[0] + R[3 * k + 1] * a_body[1] + R[3 * k + 2] * a_body[2] + g[k];
    for (int k = 0; k < 3; ++k) {
      double vn = v[k] + aw[k] * dte;
      p[k] = p[k] + v[k] * dte + 0.5 * aw[k] * (dte * dte);
      v[k] = vn;
    }
    memcpy(R, Rn, sizeof(R));
  }
  double R0[9], dR[9];
  so3_exp(rotvec_start, R0);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dR[3 * i + j] = R0[i] * R[j] + R0[3 + i] * R[3 + j] + R0[6 + i] * R[6 + j];
  for (int i = 0; i < 3; ++i) out.delta_pose[i] = R0[i] * p[0] + R0[3 + i] * p[1] + R0[6 + i] * p[2];
  for (int i = 0; i < 3; ++i) out.delta_v[i] = R0[i] * v[0] + R0[3 + i] * v[1] + R0[6 + i] * v[2];
  so3_log(dR, out.delta_pose + 3);
  out.ess = ess;
}

static const int kBlkDim[7] = {3, 3, 3, 3, 3, 1, 6};
static const int kBlkStart[7] = {0, 3, 6, 9, 12, 15, 16};

// process_noise_iw_suffstats_from_info_jax, inverse_wishart_jax.py:71-123
void process_iw_suffstats(const double* L_pred, const double* h_pred, const double* L_post, const double* h_post,
                          double* dPsi, double* dnu) {
  double mu0[DZ], mu1[DZ], Sig[DZ * DZ];
  spd_solve_lifted(DZ, L_pred, h_pred, kEpsLift, mu0);
  SpdFactor f;
  spd_factor_lifted(DZ, L_post, kEpsLift, f);
  spd_factor_solve(f, h_post, mu1);
  spd_factor_inverse(f, Sig);
  process_iw_suffstats_from(mu0, mu1, Sig, dPsi, dnu);
}

void process_iw_suffstats_from(const double* mu0, const double* mu1, const double* Sig, double* dPsi, double* dnu) {
  for (int i = 0; i < 7 * 36; ++i) dPsi[i] = 0.0;
  for (int b = 0; b < 7; ++b) {
    int s0 = kBlkStart[b], d = kBlkDim[b];
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j)
        dPsi[b * 36 + i * 6 + j] = (mu1[s0 + i] - mu0[s0 + i]) * (mu1[s0 + j] - mu0[s0 + j]) + Sig[(s0 + i) * DZ + s0 + j];
    dnu[b] = 1.0;
  }
}

// create_datasheet_process_noise_state, structures/inverse_wishart_jax.py:42-80
void datasheet_iw_state(double* nu, double* Psi) {
  const double sig[7] = {1e-4, 8.7e-7, 9.5e-5, 1e-8, 1e-6, 1e-6, 1e-8};
  for (int i = 0; i < 7 * 36; ++i) Psi[i] = 0.0;
  for (int b = 0; b < 7; ++b) {
    nu[b] = kBlkDim[b] + 1.0 + 0.5;
    for (int i = 0; i < kBlkDim[b]; ++i) Psi[b * 36 + i * 6 + i] = sig[b] * 0.5;
  }
}

static double softplus(double x) { return x > 0.0 ? x + log1p(exp(-x)) : log1p(exp(x)); }

// process_noise_state_to_Q_jax, inverse_wishart_jax.py:35-68
void process_noise_Q(const double* nu, const double* Psi, double* Q) {
  double Qr[DZ * DZ];
  for (int i = 0; i < DZ * DZ; ++i) Qr[i] = 0.0;
  for (int b = 0; b < 7; ++b) {
    double denom = softplus(50.0 * (nu[b] - kBlkDim[b] - 1.0)) / 50.0 + 1e-12;
    int s0 = kBlkStart[b];
    int e = std::min(s0 + 6, DZ) - s0;
    for (int i = 0; i < e; ++i)
      for (int j = 0; j < e; ++j) {
        double mask = (i < kBlkDim[b] && j < kBlkDim[b]) ? 1.0 : 0.0;
        Qr[(s0 + i) * DZ + s0 + j] = Psi[b * 36 + i * 6 + j] / denom * mask;
      }
  }
  psd_project(DZ, Qr, kEpsPsd, Q);
}

// process_noise_iw_apply_suffstats_jax, inverse_wishart_jax.py:126-185
void process_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                      double* Psi_out, double* cert2) {
  const double rho[7] = {0.99, 0.995, 0.95, 0.999, 0.999, 0.9999, 0.9999};
  double dsum = 0.0, nsum = 0.0;
  for (int b = 0; b < 7; ++b) {
    double raw[36];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) {
        double mask = (i < kBlkDim[b] && j < kBlkDim[b]) ? 1.0 : 0.0;
        raw[i * 6 + j] = (rho[b] * Psi[b * 36 + i * 6 + j] + dPsi[b * 36 + i * 6 + j]) * mask;
      }
    dsum += psd_project(6, raw, kEpsPsd, Psi_out + b * 36);
    double nu_raw = rho[b] * nu[b] + dnu[b];
    double nu_min = kBlkDim[b] + 1.0 + 0.5;
    double nu_floor = nu_min + softplus(nu_raw - nu_min);
    double nn = 1000.0 - softplus(1000.0 - nu_floor);
    nsum += fabs(nn - nu_raw);
    nu_out[b] = nn;
  }
  cert2[0] = dsum;
  cert2[1] = nsum;
}

// sum_m w_m r_m r_m^T / (sum w + eps), symmetrised, PSD-projected, times dt
// (measurement_noise_iw_jax.py:150-162 / :202-213)
static void weighted_outer_psd(double wsum, const double* S_acc, double dt, double* out) {
  double S[9];
  const double inv = 1.0 / (wsum + kEpsMass);
  for (int k = 0; k < 9; ++k) S[k] = S_acc[k] * inv;
  double Ss[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ss[3 * i + j] = 0.5 * (S[3 * i + j] + S[3 * j + i]);
  psd_project(3, Ss, kEpsPsd, out);
  for (int k = 0; k < 9; ++k) out[k] *= dt;
}

// The pipeline's dt_imu / valid mask / omega_avg (pipeline.py:522-548) around
// imu_gyro_meas_iw_suffstats_from_avg_rate_jax (measurement_noise_iw_jax.py:130-167) and
// imu_accel_meas_iw_suffstats_from_gravity_dir_jax (:170-218); gyro + accel summed (pipeline.py:1024-1025).
void imu_meas_iw_suffstats(int m, const double* stamps, const double* gyro, const double* accel, const double* w_int,
                           const double* gb, const double* ab, const double* rotvec0, const double* g, double* dPsi,
                           double* dnu) {
  int n_valid = 0;
  double tmin = INFINITY, tmax = -INFINITY, wsum = 0.0, om[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < m; ++i) {
    if (!(stamps[i] > 0.0)) continue;
    ++n_valid;
    tmin = std::min(tmin, stamps[i]);
    tmax = std::max(tmax, stamps[i]);
    wsum += w_int[i];
  }
  double dt = n_valid >= 2 ? (tmax - tmin) / std::max(n_valid - 1, 1) : 0.0;
  dt = std::max(dt, 1e-12);
  const double inv = 1.0 / (wsum + kEpsMass);
  for (int i = 0; i < m; ++i) {
    if (!(stamps[i] > 0.0)) continue;
    const double wn = w_int[i] * inv;
    for (int k = 0; k < 3; ++k) om[k] += wn * (gyro[3 * i + k] - gb[k]);
  }
  double R0[9], f[3];
  so3_exp(rotvec0, R0);
  for (int k = 0; k < 3; ++k) f[k] = -(R0[k] * g[0] + R0[3 + k] * g[1] + R0[6 + k] * g[2]);  // -R0^T g
  double Sg[9] = {}, Sa[9] = {};
  for (int i = 0; i < m; ++i) {
    if (!(stamps[i] > 0.0)) continue;
    const double w = w_int[i];
    double rg[3], ra[3];
    for (int k = 0; k < 3; ++k) {
      rg[k] = (gyro[3 * i + k] - gb[k]) - om[k];
      ra[k] = (accel[3 * i + k] - ab[k]) - f[k];
    }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        Sg[3 * a + b] += w * rg[a] * rg[b];
        Sa[3 * a + b] += w * ra[a] * ra[b];
      }
  }
  for (int k = 0; k < 27; ++k) dPsi[k] = 0.0;
  weighted_outer_psd(wsum, Sg, dt, dPsi);
  weighted_outer_psd(wsum, Sa, dt, dPsi + 9);
  dnu[0] = 1.0;
  dnu[1] = 1.0;
  dnu[2] = 0.0;
}

// create_datasheet_measurement_noise_state, structures/measurement_noise_iw_jax.py:37-68
void datasheet_meas_iw_state(double* nu, double* Psi) {
  const double sig[3] = {8.7e-7, 9.5e-5, 0.01};  // constants.py:190,201,210
  for (int b = 0; b < 3; ++b) {
    nu[b] = 3.0 + 1.0 + 0.5;
    for (int k = 0; k < 9; ++k) Psi[9 * b + k] = (k % 4 == 0) ? sig[b] * 0.5 : 0.0;
  }
}

// measurement_noise_apply_suffstats_jax, measurement_noise_iw_jax.py:59-100
void meas_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                   double* Psi_out, double* cert2) {
  const double rho[3] = {0.995, 0.995, 0.99};  // constants.py:279-281
  double dsum = 0.0, nsum = 0.0;
  for (int b = 0; b < 3; ++b) {
    double raw[9], sym[9];
    for (int k = 0; k < 9; ++k) raw[k] = rho[b] * Psi[9 * b + k] + dPsi[9 * b + k];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) sym[3 * i + j] = 0.5 * (raw[3 * i + j] + raw[3 * j + i]);
    dsum += psd_project(3, sym, kEpsPsd, Psi_out + 9 * b);
    const double nu_raw = rho[b] * nu[b] + dnu[b];
    const double nu_min = 3.0 + 1.0 + 0.5;
    const double nu_floor = nu_min + softplus(nu_raw - nu_min);
    const double nn = 1000.0 - softplus(1000.0 - nu_floor);
    nsum += fabs(nn - nu_raw);
    nu_out[b] = nn;
  }
  cert2[0] = dsum;
  cert2[1] = nsum;
}

// _bch3_correction, recompose.py:50-91
void bch3(const double* xi1, const double* xi2, double* out) {
  double c1[3], c2[3], c3[3];
  cross3(xi1 + 3, xi2, c1);
  cross3(xi1, xi2 + 3, c2);
  cross3(xi1 + 3, xi2 + 3, c3);
  for (int i = 0; i < 3; ++i) {
    out[i] = 0.5 * (c1[i] + c2[i]);
    out[3 + i] = 0.5 * c3[i];
  }
}

}  // namespace host
}  // namespace gcs
