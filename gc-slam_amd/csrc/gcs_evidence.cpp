// Step 9 IMU / odometry evidence family (host C++): the reference's _compute_imu_odom_branch
// (FS/backend/pipeline.py:595-776) and the operators it calls, restated in C++.  Every factor
// writes a 3x3 / diagonal block of the 22-D evidence; the certificate fields that feed the
// pipeline (trigger magnitudes, ESS, NLL) are returned alongside.  FS = fl_ws/src/fl_slam_poc/fl_slam_poc.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gcs_host.h"
#include "gcs_math.h"

namespace gcs {
namespace host {

namespace {

double cert_trigger(const EvCert& c) {  // CertBundle.total_trigger_magnitude, FS/common/certificates.py:439-455
  return c.lift + c.psd + c.mer + fabs(1.0 - c.trust_alpha);
}

void add_block3(double* L, int i0, const double* B3, double s) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) L[(i0 + i) * DZ + i0 + j] += s * B3[3 * i + j];
}

void matvec3(const double* A, const double* x, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

double quad3(const double* A, const double* x) {
  double y[3];
  matvec3(A, x, y);
  return x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
}

// PSD-project a 3x3 covariance, then its lifted Cholesky inverse (lift_strength = eps_lift * 3)
void info_from_cov3(const double* S, double* L3) {
  double Sp[9];
  psd_project(3, S, kEpsPsd, Sp);
  spd_inverse_lifted(3, Sp, kEpsLift, L3);
}

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
double kappa_scalar(double R_bar) {
  const double R = std::min(std::max(R_bar, 0.0), 1.0 - kEpsR);
  const double R2 = R * R;
  const double k_low = (R * (3.0 - R2)) / (1.0 - R2 + kEpsR);
  const double k_high = -log(std::max(1.0 - R2, kEpsR));
  const double s = 1.0 / (1.0 + exp(-(R - kKappaR0) / std::max(kKappaTau, 1e-6)));
  return (1.0 - s) * k_low + s * k_high;
}

void imu_odom_branch(const ImuOdomInputs& in, ImuOdomOut& out) {
  memset(&out, 0, sizeof(out));
  EvCert* all[11] = {&out.odom, &out.imu, &out.dep, &out.gyro, &out.preint, &out.planar, &out.vz, &out.vel, &out.wz,
                     &out.kin, &out.odom_dep};
  for (EvCert* c : all) *c = EvCert{};
  double* L = out.L;
  double* h = out.h;
  const double* pp = in.pose_pred;
  double Rpred[9], R0[9];
  so3_exp(pp + 3, Rpred);
  so3_exp(in.pose0 + 3, R0);

  // odom_quadratic_evidence, FS/backend/operators/odom_evidence.py:39-154
  double Lod[36], hod[6], xi_od[6];
  {
    double inv_pred[6], Terr[6];
    se3_inverse(pp, inv_pred);
    se3_compose(inv_pred, in.odom_pose, Terr);  // se3_relative(odom, pred) = pred^-1 o odom
    se3_log(Terr, xi_od);
    double cp[36];
    psd_project(6, in.odom_cov, kEpsPsd, cp);
    spd_inverse_lifted(6, cp, kEpsLift, Lod);
    for (int i = 0; i < 6; ++i) {
      double s = 0.0;
      for (int j = 0; j < 6; ++j) s += Lod[6 * i + j] * xi_od[j];
      hod[i] = s;
    }
    double nll = 0.0;
    for (int i = 0; i < 6; ++i) nll += xi_od[i] * hod[i];
    out.odom.nll = 0.5 * nll;
    out.odom.lift = kEpsLift * 6;
  }

  // imu_vmf_gravity_evidence_time_resolved, FS/backend/operators/imu_evidence.py:276-559
  double Himu[9], g_rot[3];
  {
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
    const double sigma = median(tmp) / 0.6745 + kEpsMass;
    double S[3] = {0, 0, 0}, ess_w = 0.0, ess_raw = 0.0, rel_sum = 0.0;
    for (int i = 0; i < m; ++i) {  // _accel_resultant_direction_weighted_jax (:370-399)
      const double q = e[i] / sigma;
      const double rel = exp(-0.5 * (q * q));
      rel_sum += rel;
      const double w = in.w_int[i] * rel;
      ess_w += w;
      ess_raw += in.w_int[i];
      const double* ai = &a[3 * i];
      const double n = sqrt(ai[0] * ai[0] + ai[1] * ai[1] + ai[2] * ai[2]);
      for (int k = 0; k < 3; ++k) S[k] += w * (ai[k] / (n + kEpsMass));
    }
    const double Sn = sqrt(S[0] * S[0] + S[1] * S[1] + S[2] * S[2]);
    double xbar[3] = {S[0] / (Sn + kEpsMass), S[1] / (Sn + kEpsMass), S[2] / (Sn + kEpsMass)};
    const double Rbar = Sn / (ess_w + kEpsMass);
    const double kappa = kappa_scalar(Rbar);
    const double* g = in.gravity;
    const double gn = sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]) + kEpsMass;
    const double mg[3] = {-g[0] / gn, -g[1] / gn, -g[2] / gn};
    double mu0[3];
    for (int k = 0; k < 3; ++k) mu0[k] = Rpred[k] * mg[0] + Rpred[3 + k] * mg[1] + Rpred[6 + k] * mg[2];  // R^T (-g_hat)
    double cr[3];
    cross3(mu0, xbar, cr);
    for (int k = 0; k < 3; ++k) g_rot[k] = -kappa * cr[k];
    const double xd = xbar[0] * mu0[0] + xbar[1] * mu0[1] + xbar[2] * mu0[2];
    double H[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        H[3 * i + j] = kappa * ((i == j ? xd : 0.0) - 0.5 * (xbar[i] * mu0[j] + mu0[i] * xbar[j]));
    double Hs[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Hs[3 * i + j] = 0.5 * (H[3 * i + j] + H[3 * j + i]);
    double c6[6];
    psd_project(3, Hs, kEpsPsd, Himu, c6);
    const double mean_rel = rel_sum / m;
    out.imu.ess = ess_w;
    out.imu.support = mean_rel;
    out.imu.nll = (-kappa * xd) / (ess_w + kEpsMass);
    out.imu.psd = c6[0];
    out.imu.mer = ess_w / (ess_raw + kEpsMass);
    out.imu.trust_alpha = mean_rel;
    out.kappa = kappa;
    out.transport_sigma = sigma;
    out.ess_weighted = ess_w;
    out.mean_reliability = mean_rel;
  }
  // imu_dependence_inflation (:562-589)
  {
    const double s = std::max(out.transport_sigma, 0.0);
    out.imu_scale = 1.0 / (1.0 + s * s + kEpsMass);
    out.dep.trust_alpha = out.imu_scale;
  }

  // imu_gyro_rotation_evidence, FS/backend/operators/imu_gyro_evidence.py:38-163
  double Lgy[9], hgy[3];
  {
    const double dt_pos = std::max(in.dt_int, 0.0), dt_eff = dt_pos + kEpsMass, ms = dt_pos / dt_eff;
    double Rd[9], Rend[9], Rdiff[9], r[3];
    so3_exp(in.drot_int, Rd);
    mat3_mul(R0, Rd, Rend);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        Rdiff[3 * i + j] = Rpred[i] * Rend[j] + Rpred[3 + i] * Rend[3 + j] + Rpred[6 + i] * Rend[6 + j];
    so3_log(Rdiff, r);
    double S[9], Lr[9];
    for (int k = 0; k < 9; ++k) S[k] = in.Sigma_g[k] * dt_eff;
    info_from_cov3(S, Lr);
    for (int k = 0; k < 9; ++k) Lgy[k] = ms * Lr[k];
    matvec3(Lgy, r, hgy);
    out.gyro.nll = 0.5 * quad3(Lr, r);
    out.gyro.lift = kEpsLift * 3;
  }

  // imu_preintegration_factor, FS/backend/operators/imu_preintegration_factor.py:46-180
  double Lv[9], Lp[9], rv[3], rp[3], msp;
  {
    double dvw[3], dpw[3];
    matvec3(R0, in.dv_int, dvw);
    matvec3(R0, in.dp_int, dpw);
    const double* ps = in.pose0;
    const double* vs = in.mu_prev + 6;
    for (int k = 0; k < 3; ++k) {
      rv[k] = (vs[k] + dvw[k]) - in.mu_inc[6 + k];
      rp[k] = (ps[k] + vs[k] * in.dt_int + dpw[k]) - pp[k];
    }
    const double dt_pos = std::max(in.dt_int, 0.0), dt_eff = dt_pos + kEpsMass;
    msp = dt_pos / dt_eff;
    double Sv[9], Sp[9];
    for (int k = 0; k < 9; ++k) {
      Sv[k] = in.Sigma_a[k] * dt_eff;
      Sp[k] = in.Sigma_a[k] * (dt_eff * dt_eff * dt_eff);
    }
    info_from_cov3(Sv, Lv);
    info_from_cov3(Sp, Lp);
    out.preint.nll = 0.5 * quad3(Lv, rv) + 0.5 * quad3(Lp, rp);
    out.preint.lift = kEpsLift * 3 + kEpsLift * 3;
  }

  // planar_z_prior / velocity_z_prior, FS/backend/operators/planar_prior.py:55-195
  const double prec_z = 1.0 / (in.planar_z_sigma * in.planar_z_sigma);
  const double r_z = in.planar_z_ref - pp[2];
  out.planar.nll = 0.5 * r_z * r_z * prec_z;
  const double prec_vz = 1.0 / (in.planar_vz_sigma * in.planar_vz_sigma);
  const double r_vz = -in.mu_inc[8];

  // odom_velocity_evidence, FS/backend/operators/odom_twist_evidence.py:58-149
  double Lvel[9], hvel[3];
  {
    double vb[3], r[3], Sv[9];
    for (int k = 0; k < 3; ++k) vb[k] = Rpred[k] * in.mu_inc[6] + Rpred[3 + k] * in.mu_inc[7] + Rpred[6 + k] * in.mu_inc[8];
    for (int k = 0; k < 3; ++k) r[k] = in.odom_twist[k] - vb[k];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Sv[3 * i + j] = in.odom_twist_cov[6 * i + j];
    info_from_cov3(Sv, Lvel);
    matvec3(Lvel, r, hvel);
    out.vel.nll = 0.5 * quad3(Lvel, r);
    out.vel.lift = kEpsLift * 3;
  }
  // odom_yawrate_evidence (:157-228)
  const double sigma_wz = sqrt(std::max(in.odom_twist_cov[6 * 5 + 5], 1e-12));
  const double prec_wz = 1.0 / (sigma_wz * sigma_wz);
  const double r_wz = in.odom_twist[5] - in.omega_avg[2];
  out.wz.nll = 0.5 * r_wz * r_wz * prec_wz;

  // pose_twist_kinematic_consistency (:251-397) and odom_dependence_inflation (:400-430)
  double Lkt[9], Lkr[9], rt[3], rr[3];
  {
    const double dt = in.dt_sec;
    double dp[3], Rrel[9], dth[3];
    matvec3(R0, in.odom_twist, dp);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rrel[3 * i + j] = R0[i] * Rpred[j] + R0[3 + i] * Rpred[3 + j] + R0[6 + i] * Rpred[6 + j];
    so3_log(Rrel, dth);
    for (int k = 0; k < 3; ++k) {
      rt[k] = dp[k] * dt - (pp[k] - in.pose0[k]);
      rr[k] = in.odom_twist[3 + k] * dt - dth[k];
    }
    const double dt2 = dt * dt + kEpsPsd;
    double St[9], Sr[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        St[3 * i + j] = dt2 * in.odom_twist_cov[6 * i + j];
        Sr[3 * i + j] = dt2 * in.odom_twist_cov[6 * (3 + i) + 3 + j];
      }
    info_from_cov3(St, Lkt);
    info_from_cov3(Sr, Lkr);
    out.kin.nll = 0.5 * quad3(Lkt, rt) + 0.5 * quad3(Lkr, rr);
    out.kin.lift = kEpsLift * 3 + kEpsLift * 3;
    const double mag = sqrt(rt[0] * rt[0] + rt[1] * rt[1] + rt[2] * rt[2]) + sqrt(rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2]);
    out.odom_scale = 1.0 / (1.0 + mag * mag + kEpsMass);
    out.odom_dep.trust_alpha = out.odom_scale;
  }

  // sum with the dependence scales (pipeline.py:733-750)
  const double so = out.odom_scale, si = out.imu_scale;
  for (int i = 0; i < 6; ++i) {
    for (int j = 0; j < 6; ++j) L[i * DZ + j] += so * Lod[6 * i + j];
    h[i] += so * hod[i];
  }
  add_block3(L, 3, Himu, si);
  for (int k = 0; k < 3; ++k) h[3 + k] += si * (-g_rot[k]);
  add_block3(L, 3, Lgy, si);
  for (int k = 0; k < 3; ++k) h[3 + k] += si * hgy[k];
  double Lps[9], Lvs[9], hp3[3], hv3[3];
  for (int k = 0; k < 9; ++k) { Lps[k] = msp * Lp[k]; Lvs[k] = msp * Lv[k]; }
  matvec3(Lps, rp, hp3);
  matvec3(Lvs, rv, hv3);
  add_block3(L, 0, Lps, 1.0);
  add_block3(L, 6, Lvs, 1.0);
  for (int k = 0; k < 3; ++k) { h[k] += hp3[k]; h[6 + k] += hv3[k]; }
  L[2 * DZ + 2] += prec_z;
  h[2] += prec_z * r_z;
  L[8 * DZ + 8] += prec_vz;
  h[8] += prec_vz * r_vz;
  add_block3(L, 6, Lvel, so);
  for (int k = 0; k < 3; ++k) h[6 + k] += so * hvel[k];
  L[5 * DZ + 5] += so * prec_wz;
  h[5] += so * (prec_wz * r_wz);
  double hkt[3], hkr[3];
  matvec3(Lkt, rt, hkt);
  matvec3(Lkr, rr, hkr);
  add_block3(L, 0, Lkt, 1.0);
  add_block3(L, 3, Lkr, 1.0);
  for (int k = 0; k < 3; ++k) { h[k] += hkt[k]; h[3 + k] += hkr[k]; }

  double T = 0.0;
  for (EvCert* c : all) T += cert_trigger(*c);
  out.trigger = T;
}

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
