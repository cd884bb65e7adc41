// Step 9's IMU / odometry evidence family (FS/backend/pipeline.py:595-776 and the eleven factor files,
// FS = fl_ws/src/fl_slam_poc/fl_slam_poc) as one __host__ __device__ assembly: the host branch
// (gcs_evidence.cpp imu_odom_branch) and the device kernel (gcs_imu_odom.hip k_imu_odom) run this same
// code on the window's per-sample statistics (ImuVmfStats), which each computes its own way -- the host
// in sample order, the device in one workgroup's fixed-order block sums.  The small dense algebra it
// calls is gcs_small.h.
#pragma once
#include <math.h>

#include "gcs_host.h"
#include "gcs_math.h"
#include "gcs_small.h"

namespace gcs {
namespace host {

// the per-sample part of imu_vmf_gravity_evidence_time_resolved (imu_evidence.py:276-399): the
// reliability-weighted resultant and weights, and the transport-consistency MAD scale
struct ImuVmfStats {
  double S[3];     // sum_i w_int_i rel_i a_i / (|a_i| + eps)
  double ess_w;    // sum_i w_int_i rel_i
  double ess_raw;  // sum_i w_int_i
  double rel_sum;  // sum_i rel_i
  double sigma;    // median |e_i - median e| / 0.6745 + eps
};

GCS_HD double ev_max(double a, double b) { return (a < b) ? b : a; }  // std::max, NaN included

GCS_HD double ev_cert_trigger(const EvCert& c) {  // CertBundle.total_trigger_magnitude, certificates.py:439-455
  return c.lift + c.psd + c.mer + fabs(1.0 - c.trust_alpha);
}

GCS_HD void ev_add_block3(double* L, int i0, const double* B3, double s) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) L[(i0 + i) * DZ + i0 + j] += s * B3[3 * i + j];
}

GCS_HD void ev_matvec3(const double* A, const double* x, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

GCS_HD double ev_quad3(const double* A, const double* x) {
  double y[3];
  ev_matvec3(A, x, y);
  return x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
}

// PSD-project a 3x3 covariance, then its lifted Cholesky inverse (lift_strength = eps_lift * 3)
GCS_HD void ev_info_from_cov3(const double* S, double* L3) {
  double Sp[9];
  small::psd_project<3>(S, kEpsPsd, Sp);
  small::spd_inverse_lifted<3>(Sp, kEpsLift, L3);
}

// kappa_from_resultant_v2 / _kappa_continuous_formula, FS/backend/operators/kappa.py:84-127,172-234
GCS_HD double kappa_scalar_hd(double R_bar) {
  const double Rc = (R_bar < 0.0) ? 0.0 : R_bar;              // std::min(std::max(R_bar, 0), 1 - eps_r)
  const double R = (1.0 - kEpsR < Rc) ? 1.0 - kEpsR : Rc;
  const double R2 = R * R;
  const double k_low = (R * (3.0 - R2)) / (1.0 - R2 + kEpsR);
  const double k_high = -log(ev_max(1.0 - R2, kEpsR));
  const double s = 1.0 / (1.0 + exp(-(R - kKappaR0) / ev_max(kKappaTau, 1e-6)));
  return (1.0 - s) * k_low + s * k_high;
}

// The factors' results ahead of their sum: each io_part_* fills its own fields here and its own
// certificate fields of ImuOdomOut, reading only the inputs, so the parts are independent -- the host
// runs them in order, the device kernel one per wave (gcs_imu_odom.hip k_imu_odom_assemble) -- and
// io_sum adds them in the pipeline's order (pipeline.py:733-750).
struct ImuOdomParts {
  double Lod[36], hod[6];                                // odom_quadratic_evidence
  double Himu[9], g_rot[3];                              // imu_vmf_gravity_evidence_time_resolved
  double Lgy[9], hgy[3];                                 // imu_gyro_rotation_evidence
  double Lv[9], Lp[9], rv[3], rp[3], msp;                // imu_preintegration_factor
  double Lvel[9], hvel[3];                               // odom_velocity_evidence
  double Lkt[9], Lkr[9], rt[3], rr[3];                   // pose_twist_kinematic_consistency
};
constexpr int kIoParts = 6;

GCS_HD void io_init(ImuOdomOut& out) {
  for (int i = 0; i < DZ * DZ; ++i) out.L[i] = 0.0;
  for (int i = 0; i < DZ; ++i) out.h[i] = 0.0;
  out.trigger = out.kappa = out.transport_sigma = out.ess_weighted = out.mean_reliability = 0.0;
  out.imu_scale = out.odom_scale = 0.0;
  out.odom = out.imu = out.dep = out.gyro = out.preint = out.planar = EvCert{};
  out.vz = out.vel = out.wz = out.kin = out.odom_dep = EvCert{};
}

// odom_quadratic_evidence, FS/backend/operators/odom_evidence.py:39-154
GCS_HD void io_part_odom(const ImuOdomInputs& in, ImuOdomParts& p, ImuOdomOut& out) {
  double xi_od[6];
  double inv_pred[6], Terr[6];
  small::se3_inverse(in.pose_pred, inv_pred);
  small::se3_compose(inv_pred, in.odom_pose, Terr);  // se3_relative(odom, pred) = pred^-1 o odom
  se3_log_hd(Terr, xi_od);
  double cp[36];
  small::psd_project<6>(in.odom_cov, kEpsPsd, cp);
  small::spd_inverse_lifted<6>(cp, kEpsLift, p.Lod);
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
    for (int j = 0; j < 6; ++j) s += p.Lod[6 * i + j] * xi_od[j];
    p.hod[i] = s;
  }
  double nll = 0.0;
  for (int i = 0; i < 6; ++i) nll += xi_od[i] * p.hod[i];
  out.odom.nll = 0.5 * nll;
  out.odom.lift = kEpsLift * 6;
}

// imu_vmf_gravity_evidence_time_resolved, FS/backend/operators/imu_evidence.py:276-559 (the per-sample
// transport consistency, MAD scale and reliability-weighted sums arrive in v: ImuVmfStats), and
// imu_dependence_inflation (:562-589)
GCS_HD void io_part_imu(const ImuOdomInputs& in, const ImuVmfStats& v, ImuOdomParts& p, ImuOdomOut& out) {
  double Rpred[9];
  so3_exp(in.pose_pred + 3, Rpred);
  const int m = in.m;
  const double Sn = sqrt(v.S[0] * v.S[0] + v.S[1] * v.S[1] + v.S[2] * v.S[2]);
  double xbar[3] = {v.S[0] / (Sn + kEpsMass), v.S[1] / (Sn + kEpsMass), v.S[2] / (Sn + kEpsMass)};
  const double ess_w = v.ess_w, ess_raw = v.ess_raw, rel_sum = v.rel_sum, sigma = v.sigma;
  const double Rbar = Sn / (ess_w + kEpsMass);
  const double kappa = kappa_scalar_hd(Rbar);
  const double* g = in.gravity;
  const double gn = sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]) + kEpsMass;
  const double mg[3] = {-g[0] / gn, -g[1] / gn, -g[2] / gn};
  double mu0[3];
  for (int k = 0; k < 3; ++k) mu0[k] = Rpred[k] * mg[0] + Rpred[3 + k] * mg[1] + Rpred[6 + k] * mg[2];  // R^T (-g_hat)
  double cr[3];
  cross3(mu0, xbar, cr);
  for (int k = 0; k < 3; ++k) p.g_rot[k] = -kappa * cr[k];
  const double xd = xbar[0] * mu0[0] + xbar[1] * mu0[1] + xbar[2] * mu0[2];
  double H[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      H[3 * i + j] = kappa * ((i == j ? xd : 0.0) - 0.5 * (xbar[i] * mu0[j] + mu0[i] * xbar[j]));
  double Hs[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Hs[3 * i + j] = 0.5 * (H[3 * i + j] + H[3 * j + i]);
  double c6[6];
  small::psd_project<3>(Hs, kEpsPsd, p.Himu, c6);
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
  const double sg = ev_max(sigma, 0.0);
  out.imu_scale = 1.0 / (1.0 + sg * sg + kEpsMass);
  out.dep.trust_alpha = out.imu_scale;
}

// imu_gyro_rotation_evidence, FS/backend/operators/imu_gyro_evidence.py:38-163
GCS_HD void io_part_gyro(const ImuOdomInputs& in, ImuOdomParts& p, ImuOdomOut& out) {
  double Rpred[9], R0[9];
  so3_exp(in.pose_pred + 3, Rpred);
  so3_exp(in.pose0 + 3, R0);
  const double dt_pos = ev_max(in.dt_int, 0.0), dt_eff = dt_pos + kEpsMass, ms = dt_pos / dt_eff;
  double Rd[9], Rend[9], Rdiff[9], r[3];
  so3_exp(in.drot_int, Rd);
  mat3_mul(R0, Rd, Rend);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Rdiff[3 * i + j] = Rpred[i] * Rend[j] + Rpred[3 + i] * Rend[3 + j] + Rpred[6 + i] * Rend[6 + j];
  so3_log(Rdiff, r);
  double S[9], Lr[9];
  for (int k = 0; k < 9; ++k) S[k] = in.Sigma_g[k] * dt_eff;
  ev_info_from_cov3(S, Lr);
  for (int k = 0; k < 9; ++k) p.Lgy[k] = ms * Lr[k];
  ev_matvec3(p.Lgy, r, p.hgy);
  out.gyro.nll = 0.5 * ev_quad3(Lr, r);
  out.gyro.lift = kEpsLift * 3;
}

// imu_preintegration_factor, FS/backend/operators/imu_preintegration_factor.py:46-180
GCS_HD void io_part_preint(const ImuOdomInputs& in, ImuOdomParts& p, ImuOdomOut& out) {
  double R0[9];
  so3_exp(in.pose0 + 3, R0);
  const double* pp = in.pose_pred;
  double dvw[3], dpw[3];
  ev_matvec3(R0, in.dv_int, dvw);
  ev_matvec3(R0, in.dp_int, dpw);
  const double* ps = in.pose0;
  const double* vs = in.mu_prev + 6;
  for (int k = 0; k < 3; ++k) {
    p.rv[k] = (vs[k] + dvw[k]) - in.mu_inc[6 + k];
    p.rp[k] = (ps[k] + vs[k] * in.dt_int + dpw[k]) - pp[k];
  }
  const double dt_pos = ev_max(in.dt_int, 0.0), dt_eff = dt_pos + kEpsMass;
  p.msp = dt_pos / dt_eff;
  double Sv[9], Sp[9];
  for (int k = 0; k < 9; ++k) {
    Sv[k] = in.Sigma_a[k] * dt_eff;
    Sp[k] = in.Sigma_a[k] * (dt_eff * dt_eff * dt_eff);
  }
  ev_info_from_cov3(Sv, p.Lv);
  ev_info_from_cov3(Sp, p.Lp);
  out.preint.nll = 0.5 * ev_quad3(p.Lv, p.rv) + 0.5 * ev_quad3(p.Lp, p.rp);
  out.preint.lift = kEpsLift * 3 + kEpsLift * 3;
}

// odom_velocity_evidence, FS/backend/operators/odom_twist_evidence.py:58-149
GCS_HD void io_part_vel(const ImuOdomInputs& in, ImuOdomParts& p, ImuOdomOut& out) {
  double Rpred[9];
  so3_exp(in.pose_pred + 3, Rpred);
  double vb[3], r[3], Sv[9];
  for (int k = 0; k < 3; ++k) vb[k] = Rpred[k] * in.mu_inc[6] + Rpred[3 + k] * in.mu_inc[7] + Rpred[6 + k] * in.mu_inc[8];
  for (int k = 0; k < 3; ++k) r[k] = in.odom_twist[k] - vb[k];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Sv[3 * i + j] = in.odom_twist_cov[6 * i + j];
  ev_info_from_cov3(Sv, p.Lvel);
  ev_matvec3(p.Lvel, r, p.hvel);
  out.vel.nll = 0.5 * ev_quad3(p.Lvel, r);
  out.vel.lift = kEpsLift * 3;
}

// pose_twist_kinematic_consistency (odom_twist_evidence.py:251-397) and odom_dependence_inflation (:400-430)
GCS_HD void io_part_kin(const ImuOdomInputs& in, ImuOdomParts& p, ImuOdomOut& out) {
  double Rpred[9], R0[9];
  so3_exp(in.pose_pred + 3, Rpred);
  so3_exp(in.pose0 + 3, R0);
  const double* pp = in.pose_pred;
  const double dt = in.dt_sec;
  double dp[3], Rrel[9], dth[3];
  ev_matvec3(R0, in.odom_twist, dp);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rrel[3 * i + j] = R0[i] * Rpred[j] + R0[3 + i] * Rpred[3 + j] + R0[6 + i] * Rpred[6 + j];
  so3_log(Rrel, dth);
  for (int k = 0; k < 3; ++k) {
    p.rt[k] = dp[k] * dt - (pp[k] - in.pose0[k]);
    p.rr[k] = in.odom_twist[3 + k] * dt - dth[k];
  }
  const double dt2 = dt * dt + kEpsPsd;
  double St[9], Sr[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      St[3 * i + j] = dt2 * in.odom_twist_cov[6 * i + j];
      Sr[3 * i + j] = dt2 * in.odom_twist_cov[6 * (3 + i) + 3 + j];
    }
  ev_info_from_cov3(St, p.Lkt);
  ev_info_from_cov3(Sr, p.Lkr);
  out.kin.nll = 0.5 * ev_quad3(p.Lkt, p.rt) + 0.5 * ev_quad3(p.Lkr, p.rr);
  out.kin.lift = kEpsLift * 3 + kEpsLift * 3;
  const double mag = sqrt(p.rt[0] * p.rt[0] + p.rt[1] * p.rt[1] + p.rt[2] * p.rt[2]) +
                     sqrt(p.rr[0] * p.rr[0] + p.rr[1] * p.rr[1] + p.rr[2] * p.rr[2]);
  out.odom_scale = 1.0 / (1.0 + mag * mag + kEpsMass);
  out.odom_dep.trust_alpha = out.odom_scale;
}

// part k of the six (the device kernel's wave k)
GCS_HD void io_part(int k, const ImuOdomInputs& in, const ImuVmfStats& v, ImuOdomParts& p, ImuOdomOut& out) {
  switch (k) {
    case 0: io_part_odom(in, p, out); break;
    case 1: io_part_imu(in, v, p, out); break;
    case 2: io_part_gyro(in, p, out); break;
    case 3: io_part_preint(in, p, out); break;
    case 4: io_part_vel(in, p, out); break;
    default: io_part_kin(in, p, out); break;
  }
}

// the planar z / v_z priors and the odometry yaw rate (planar_prior.py:55-195, odom_twist_evidence.py:157-228),
// then the sum with the dependence scales (pipeline.py:733-750) and the certificates' trigger
GCS_HD void io_sum(const ImuOdomInputs& in, const ImuOdomParts& p, ImuOdomOut& out) {
  double* L = out.L;
  double* h = out.h;
  const double* pp = in.pose_pred;
  const double prec_z = 1.0 / (in.planar_z_sigma * in.planar_z_sigma);
  const double r_z = in.planar_z_ref - pp[2];
  out.planar.nll = 0.5 * r_z * r_z * prec_z;
  const double prec_vz = 1.0 / (in.planar_vz_sigma * in.planar_vz_sigma);
  const double r_vz = -in.mu_inc[8];
  const double sigma_wz = sqrt(ev_max(in.odom_twist_cov[6 * 5 + 5], 1e-12));
  const double prec_wz = 1.0 / (sigma_wz * sigma_wz);
  const double r_wz = in.odom_twist[5] - in.omega_avg[2];
  out.wz.nll = 0.5 * r_wz * r_wz * prec_wz;

  const double so = out.odom_scale, si = out.imu_scale;
  for (int i = 0; i < 6; ++i) {
    for (int j = 0; j < 6; ++j) L[i * DZ + j] += so * p.Lod[6 * i + j];
    h[i] += so * p.hod[i];
  }
  ev_add_block3(L, 3, p.Himu, si);
  for (int k = 0; k < 3; ++k) h[3 + k] += si * (-p.g_rot[k]);
  ev_add_block3(L, 3, p.Lgy, si);
  for (int k = 0; k < 3; ++k) h[3 + k] += si * p.hgy[k];
  double Lps[9], Lvs[9], hp3[3], hv3[3];
  for (int k = 0; k < 9; ++k) { Lps[k] = p.msp * p.Lp[k]; Lvs[k] = p.msp * p.Lv[k]; }
  ev_matvec3(Lps, p.rp, hp3);
  ev_matvec3(Lvs, p.rv, hv3);
  ev_add_block3(L, 0, Lps, 1.0);
  ev_add_block3(L, 6, Lvs, 1.0);
  for (int k = 0; k < 3; ++k) { h[k] += hp3[k]; h[6 + k] += hv3[k]; }
  L[2 * DZ + 2] += prec_z;
  h[2] += prec_z * r_z;
  L[8 * DZ + 8] += prec_vz;
  h[8] += prec_vz * r_vz;
  ev_add_block3(L, 6, p.Lvel, so);
  for (int k = 0; k < 3; ++k) h[6 + k] += so * p.hvel[k];
  L[5 * DZ + 5] += so * prec_wz;
  h[5] += so * (prec_wz * r_wz);
  double hkt[3], hkr[3];
  ev_matvec3(p.Lkt, p.rt, hkt);
  ev_matvec3(p.Lkr, p.rr, hkr);
  ev_add_block3(L, 0, p.Lkt, 1.0);
  ev_add_block3(L, 3, p.Lkr, 1.0);
  for (int k = 0; k < 3; ++k) { h[k] += hkt[k]; h[3 + k] += hkr[k]; }

  const EvCert* all[11] = {&out.odom, &out.imu, &out.dep, &out.gyro, &out.preint, &out.planar, &out.vz, &out.vel,
                           &out.wz, &out.kin, &out.odom_dep};
  double T = 0.0;
  for (const EvCert* c : all) T += ev_cert_trigger(*c);
  out.trigger = T;
}

GCS_HD void imu_odom_assemble(const ImuOdomInputs& in, const ImuVmfStats& v, ImuOdomOut& out) {
  io_init(out);
  ImuOdomParts p;
  for (int k = 0; k < kIoParts; ++k) io_part(k, in, v, p, out);
  io_sum(in, p, out);
}

}  // namespace host
}  // namespace gcs

namespace gcs {
// the device branch's output record (gcs_imu_odom.hip): host::ImuOdomOut, then dt_int, dt_imu, omega_avg
constexpr int kIoOutWords = (int)(sizeof(host::ImuOdomOut) / sizeof(double)) + 5;
static_assert(sizeof(host::ImuOdomOut) % sizeof(double) == 0, "a record of doubles");
}  // namespace gcs
