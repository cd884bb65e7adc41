// Host-side 22-D numerics: the tail of the per-scan pipeline (predict, tempering, fusion,
// recompose, IW, hypothesis combine).  Restates FS/common/primitives.py, FS/common/belief.py
// and the small operators in FS/backend/operators/ in C++ (the 22x22 algebra is latency bound;
// SURVEY.md section 7 step 5 places it on host C++ or one workgroup).
#pragma once
#include <stdint.h>

namespace gcs {
namespace host {

constexpr int DZ = 22;

// Symmetric eigen-decomposition by cyclic Jacobi (row-major n x n); w unsorted, V columns.
void jacobi_eigh(int n, const double* A, double* w, double* V);
// domain_projection_psd_core; cert6 = [delta, sym_delta, eig_min, eig_max, cond, near_null]
double psd_project(int n, const double* M, double eps_psd, double* out, double* cert6 = nullptr);
bool cholesky(int n, const double* A, double* Lc);
void spd_solve_lifted(int n, const double* L, const double* b, double eps_lift, double* x);
void spd_inverse_lifted(int n, const double* L, double eps_lift, double* Linv);

// One Cholesky factor of L + eps_lift I (spd_cholesky_*_lifted_core, primitives.py:141-192),
// reused by every solve / inverse of the same matrix in a scan.
// Largest matrix order of the host numerics (the 22-D state; public entry points reject larger n);
// it sizes the stack working arrays.
constexpr int kMaxN = 24;
struct SpdFactor {
  int n = 0;
  double Lc[kMaxN * kMaxN];
  double rd[kMaxN];  // 1 / diag(Lc)
};
void spd_factor_lifted(int n, const double* L, double eps_lift, SpdFactor& f);
void spd_factor_solve(const SpdFactor& f, const double* b, double* x);
void spd_factor_inverse(const SpdFactor& f, double* Linv);
void solve3(const double* A, const double* b, double* x);  // LU with partial pivoting

struct Belief {
  double X_anchor[6];
  double stamp;
  double z_lin[DZ];
  double L[DZ * DZ];
  double h[DZ];
};

void se3_compose(const double* a, const double* b, double* out);
void se3_inverse(const double* a, double* out);
void se3_log(const double* T, double* out);
void mean_increment(const Belief& b, double* dz);
void mean_world_pose(const Belief& b, double* pose6);
// world pose from an already solved mean increment (belief.py:400-434)
void world_pose_from_increment(const Belief& b, const double* dz, double* pose6);

// predict_diffusion (predict.py:43-103); infl = [lift_strength, psd_delta, dt_scale]
// prev_fac / prev_cov (optional): spd_factor_lifted(prev.L) and its inverse, already computed
void predict_diffusion(const Belief& prev, const double* Q, double dt, Belief& pred, double* infl3,
                       double* mean_prev_out = nullptr /*DZ, optional: prev's mean increment*/,
                       const SpdFactor* prev_fac = nullptr, const double* prev_cov = nullptr);

struct PreintOut {
  double delta_pose[6];  // [R0^T p, Log(R0^T R_end)]: delta_pose[0:3] is delta_p_body
  double delta_v[3];     // R0^T v_end
  double ess;
};
void preintegrate_imu(int m, const double* stamps, const double* gyro, const double* accel, const double* w,
                      const double* rotvec_start, const double* gb, const double* ab, const double* g, PreintOut& out);

// IW process noise (inverse_wishart_jax.py)
void process_iw_suffstats(const double* L_pred, const double* h_pred, const double* L_post, const double* h_post,
                          double* dPsi /*7x36*/, double* dnu /*7*/);
// same from the solved means and posterior covariance (shared with the rest of the scan tail)
void process_iw_suffstats_from(const double* mu_pred, const double* mu_post, const double* Sig_post, double* dPsi,
                               double* dnu);
void datasheet_iw_state(double* nu, double* Psi);
void process_noise_Q(const double* nu, const double* Psi, double* Q);
void process_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                      double* Psi_out, double* cert2);

// IW measurement noise, blocks [gyro, accel, lidar] (measurement_noise_iw_jax.py).  w_int: the
// scan-to-scan IMU window weights (padded samples, stamp <= 0, are masked here).
void imu_meas_iw_suffstats(int m, const double* stamps, const double* gyro, const double* accel, const double* w_int,
                           const double* gyro_bias, const double* accel_bias, const double* rotvec0,
                           const double* gravity_W, double* dPsi /*3x9*/, double* dnu /*3*/);
void datasheet_meas_iw_state(double* nu /*3*/, double* Psi /*3x9*/);
void meas_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                   double* Psi_out, double* cert2);

void bch3(const double* xi1, const double* xi2, double* out);

// ---------------------------------------------------------------- step 9 IMU / odometry family
// (gcs_evidence.cpp; FS/backend/pipeline.py:595-776)
// The CertBundle fields the pipeline reads back from one operator (FS/common/certificates.py:22-109):
// support, mismatch and the influence fields of total_trigger_magnitude (identity defaults).
struct EvCert {
  double ess = 0.0, support = 1.0, nll = 0.0;
  double lift = 0.0, psd = 0.0, mer = 0.0, trust_alpha = 1.0;
};
struct ImuOdomInputs {
  int m;                                  // IMU window length (>= 2)
  const double *stamps, *gyro, *accel;    // [m], [m*3], [m*3]
  const double* w_int;                    // scan-to-scan window weights [m] (unmasked)
  double dt_imu, dt_int, dt_sec;
  const double* omega_avg;                // [3] (pipeline.py:536-548)
  const double* drot_int;                 // scan-to-scan preintegration: delta rotvec [3]
  const double* dp_int;                   //   delta p (start body frame) [3]
  const double* dv_int;                   //   delta v (start body frame) [3]
  const double* pose0;                    // belief_prev.mean_world_pose [6]
  const double* pose_pred;                // belief_pred.mean_world_pose [6]
  const double* mu_prev;                  // belief_prev.mean_increment [22]
  const double* mu_inc;                   // belief_pred.mean_increment [22]
  const double* accel_bias;               // mu_inc[12:15]
  const double* gravity;                  // gravity_W * imu_gravity_scale
  const double *Sigma_g, *Sigma_a;        // 3x3
  const double *odom_pose, *odom_cov;     // [6], 6x6
  const double *odom_twist, *odom_twist_cov;  // [6], 6x6
  double planar_z_ref, planar_z_sigma, planar_vz_sigma;
};
struct ImuOdomOut {
  double L[DZ * DZ], h[DZ];  // L_imu_odom, h_imu_odom (pipeline.py:745-750)
  EvCert odom, imu, dep, gyro, preint, planar, vz, vel, wz, kin, odom_dep;  // all_certs order
  double trigger;            // sum of the eleven certs' trigger magnitudes
  double kappa, transport_sigma, ess_weighted, mean_reliability, imu_scale, odom_scale;
};
double imu_integration_time(int m, const double* stamps, double t_start, double t_end);
void imu_rate_stats(int m, const double* stamps, const double* gyro, const double* w_int, const double* gyro_bias,
                    double* dt_imu, double* omega_avg);
void meas_iw_mode(const double* nu3, const double* Psi3x9, int idx, double* Sigma3x3);
double kappa_scalar(double R_bar);
void imu_odom_branch(const ImuOdomInputs& in, ImuOdomOut& out);
double fusion_scale(double cond, double ess, double nll, double power_beta, double dt_asym, double z_to_xy,
                    double excitation_total, double alpha_min, double alpha_max, double c0_cond, double* quality);
void pose6_conditioning(const double* L_ev, double* eig_min, double* eig_max, double* cond, double* near_null);

}  // namespace host
}  // namespace gcs
