// Step 9 IMU / odometry evidence family (host C++): the reference's _compute_imu_odom_branch
// (FS/backend/pipeline.py:595-776) and the operators it calls, restated in C++.  Every factor
// writes a 3x3 / diagonal block of the 22-D evidence; the certificate fields that feed the
// pipeline (trigger magnitudes, ESS, NLL) are returned alongside.  FS = fl_ws/src/fl_slam_poc/fl_slam_poc.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gcs_host.h"
#include "gcs_imu_odom_core.h"
#include "gcs_math.h"

namespace gcs {
namespace host {

namespace {

double median(std::vector<double>& v) {  // numpy / jnp median: mean of the two middle values for even n
  const size_t n = v.size(), k = n / 2;
  std::nth_element(v.begin(), v.begin() + k, v.end());
  const double hi = v[k];
  if (n % 2) return hi;
  return 0.5 * (*std::max_element(v.begin(), v.begin() + k) + hi);
}

}  // namespace

// compute_imu_integration_time, FS/backend/pipeline.py:262-313
double imu_integration_time(int m, const double* stamps, double t_start, double t_end) {
  const double eps = 1e-9;
  std::vector<double> v;
  v.reserve(m);
  for (int i = 0; i < m; ++i)
    if (stamps[i] > t_start - eps && stamps[i] <= t_end + eps && stamps[i] > 0.0) v.push_back(stamps[i]);
  if (v.size() < 2) return 0.0;
  std::sort(v.begin(), v.end());
  double dt = 0.0;
  for (size_t i = 1; i < v.size(); ++i) dt += std::max(v[i] - v[i - 1], 0.0);
  return std::max(0.0, std::min(dt, t_end - t_start));
}

// dt_imu and omega_avg, FS/backend/pipeline.py:522-548
void imu_rate_stats(int m, const double* stamps, const double* gyro, const double* w_int, const double* gb,
                    double* dt_imu, double* omega_avg) {
  int n_valid = 0;
  double tmin = INFINITY, tmax = -INFINITY, wsum = 0.0;
  for (int i = 0; i < m; ++i) {
    if (!(stamps[i] > 0.0)) continue;
    ++n_valid;
    tmin = std::min(tmin, stamps[i]);
    tmax = std::max(tmax, stamps[i]);
    wsum += w_int[i];
  }
  double dt = n_valid >= 2 ? (tmax - tmin) / std::max(n_valid - 1, 1) : 0.0;
  *dt_imu = std::max(dt, 1e-12);
  const double inv = 1.0 / (wsum + kEpsMass);
  omega_avg[0] = omega_avg[1] = omega_avg[2] = 0.0;
  for (int i = 0; i < m; ++i) {
    if (!(stamps[i] > 0.0)) continue;
    const double wn = w_int[i] * inv;
    for (int k = 0; k < 3; ++k) omega_avg[k] += wn * (gyro[3 * i + k] - gb[k]);
  }
}

// measurement_noise_mean_jax (IW mode), FS/backend/operators/measurement_noise_iw_jax.py:38-56
void meas_iw_mode(const double* nu3, const double* Psi3x9, int idx, double* Sigma) {
  double S[9];
  const double den = nu3[idx] + 3.0 + 1.0;
  for (int k = 0; k < 9; ++k) S[k] = Psi3x9[9 * idx + k] / den;
  psd_project(3, S, kEpsPsd, Sigma);
}

// kappa_from_resultant_v2 / _kappa_continuous_formula, FS/backend/operators/kappa.py:84-127,172-234
double kappa_scalar(double R_bar) { return kappa_scalar_hd(R_bar); }

// The window's per-sample statistics in sample order (imu_evidence.py:276-399): transport consistency
// e_i = |d a_i / dt + w_i x a_i| (central differences), its MAD scale, the reliability weights
// exp(-(e_i / sigma)^2 / 2) and the weighted resultant of the unit accelerations
ImuVmfStats imu_vmf_stats(const ImuOdomInputs& in) {
  const int m = in.m;
  const double* ab = in.accel_bias;
  std::vector<double> a((size_t)m * 3), e(m);
  for (int i = 0; i < m; ++i)
    for (int k = 0; k < 3; ++k) a[3 * i + k] = in.accel[3 * i + k] - ab[k];
  const double dt = in.dt_imu;
  for (int i = 0; i < m; ++i) {  // _compute_transport_consistency (:276-333)
    double df[3];
    for (int k = 0; k < 3; ++k) {
      if (i == 0) df[k] = (a[3 + k] - a[k]) / (dt + kEpsMass);
      else if (i == m - 1) df[k] = (a[3 * i + k] - a[3 * (i - 1) + k]) / (dt + kEpsMass);
      else df[k] = (a[3 * (i + 1) + k] - a[3 * (i - 1) + k]) / (2 * dt + kEpsMass);
    }
    double c[3];
    cross3(in.gyro + 3 * i, &a[3 * i], c);
    double ex = df[0] + c[0], ey = df[1] + c[1], ez = df[2] + c[2];
    e[i] = sqrt(ex * ex + ey * ey + ez * ez);
  }
  std::vector<double> tmp(e);  // _compute_reliability_weights (:336-367), MAD scale
  const double med = median(tmp);
  for (int i = 0; i < m; ++i) tmp[i] = fabs(e[i] - med);
  ImuVmfStats v{};
  v.sigma = median(tmp) / 0.6745 + kEpsMass;
  for (int i = 0; i < m; ++i) {  // _accel_resultant_direction_weighted_jax (:370-399)
    const double q = e[i] / v.sigma;
    const double rel = exp(-0.5 * (q * q));
    v.rel_sum += rel;
    const double w = in.w_int[i] * rel;
    v.ess_w += w;
    v.ess_raw += in.w_int[i];
    const double* ai = &a[3 * i];
    const double n = sqrt(ai[0] * ai[0] + ai[1] * ai[1] + ai[2] * ai[2]);
    for (int k = 0; k < 3; ++k) v.S[k] += w * (ai[k] / (n + kEpsMass));
  }
  return v;
}

void imu_odom_branch(const ImuOdomInputs& in, ImuOdomOut& out) { imu_odom_assemble(in, imu_vmf_stats(in), out); }

// FusionScaleFromCertificates, FS/backend/operators/fusion.py:46-142 (excitation_total = 0: no
// reference operator fills an ExcitationCert, certificates.py:564-567)
double fusion_scale(double cond, double ess, double nll, double power_beta, double dt_asym, double z_to_xy,
                    double excitation_total, double alpha_min, double alpha_max, double c0_cond, double* quality_out) {
  const double cond_q = c0_cond / (cond + c0_cond);
  const double supp_q = ess / (ess + 1.0);
  const double mis_q = exp(-nll);
  const double dt_q = std::min(std::max(dt_asym, 0.0), 1.0);
  const double z_q = std::min(std::max(z_to_xy / (z_to_xy + 1.0), 0.0), 1.0);
  const double exc_q = std::min(std::max(excitation_total / (excitation_total + 1.0), 0.0), 1.0);
  const double base = sqrt(cond_q * supp_q);
  const double q = base * mis_q * dt_q * z_q * exc_q * std::min(std::max(power_beta, 0.0), 1.0);
  if (quality_out) *quality_out = q;
  const double a = alpha_min + (alpha_max - alpha_min) * q;
  return std::min(std::max(a, alpha_min), alpha_max);
}

// Pose-block conditioning of the tempered evidence, FS/backend/pipeline.py:1155-1177
void pose6_conditioning(const double* L_ev, double* eig_min, double* eig_max, double* cond, double* near_null) {
  double P[36], w[6], V[36];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      double v = 0.5 * (L_ev[i * DZ + j] + L_ev[j * DZ + i]);
      P[6 * i + j] = std::isfinite(v) ? v : 0.0;
    }
  jacobi_eigh(6, P, w, V);
  double lo = INFINITY, hi = -INFINITY, nn = 0.0;
  for (int k = 0; k < 6; ++k) {
    nn += w[k] <= kEpsPsd ? 1.0 : 0.0;
    const double c = std::isfinite(w[k]) ? std::max(w[k], kEpsPsd) : kEpsPsd;
    lo = std::min(lo, c);
    hi = std::max(hi, c);
  }
  *eig_min = lo;
  *eig_max = hi;
  *cond = hi / lo;
  *near_null = nn;
}

}  // namespace host
}  // namespace gcs
