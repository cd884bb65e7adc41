"""IMU / odometry evidence family of step 9 (test oracle only): numpy restatement of the
reference's `_compute_imu_odom_branch` (FS/backend/pipeline.py:595-776) and the operators it
calls, plus FusionScaleFromCertificates with the pose-6 conditioning (pipeline.py:1150-1192,
fusion.py:46-142).

Reference paths are relative to /root/reference; FS = fl_ws/src/fl_slam_poc/fl_slam_poc.

Certificates are plain dicts holding the CertBundle fields the pipeline reads back
(FS/common/certificates.py:22-109): support (ess_total, support_frac), mismatch (nll_per_ess),
conditioning (cond) and the influence fields of `total_trigger_magnitude` (:439-455).
"""

from __future__ import annotations

import math

import numpy as np

from . import se3
from .ops import EPS_LIFT, EPS_MASS, EPS_PSD, EPS_R, KAPPA_R0, KAPPA_TAU, trigger_magnitude
from .primitives import psd_project, spd_inverse_lifted

D_Z = 22
# FS/common/constants.py
IMU_GYRO_NOISE_DENSITY = 8.7e-7   # :190
IMU_ACCEL_NOISE_DENSITY = 9.5e-5  # :201
PLANAR_Z_REF = 0.0                # :294
PLANAR_Z_SIGMA = 0.1              # :305
PLANAR_VZ_SIGMA = 0.01            # :310
ALPHA_MIN = ALPHA_MAX = 1.0       # :89-90
C0_COND = 1e6                     # :92
ODOM_COV_MISSING = 1e12           # backend_node.py:2048-2051 (no odom yet) and :939-940 (twist)


def cert(**kw):
    """CertBundle defaults (certificates.py:22-109) overridden by kw."""
    c = dict(ess_total=0.0, support_frac=1.0, nll_per_ess=0.0, cond=1.0, lift_strength=0.0,
             psd_projection_delta=0.0, nu_projection_delta=0.0, mass_epsilon_ratio=0.0, anchor_drift_rho=0.0,
             dt_scale=1.0, extrinsic_scale=1.0, trust_alpha=1.0, power_beta=1.0)
    c.update(kw)
    return c


def aggregate(certs):
    """aggregate_certificates (certificates.py:511-700) for the fields read downstream."""
    n = len(certs)
    return cert(ess_total=sum(c["ess_total"] for c in certs) / n,
                support_frac=sum(c["support_frac"] for c in certs) / n,
                nll_per_ess=sum(c["nll_per_ess"] for c in certs),
                cond=max(c["cond"] for c in certs),
                lift_strength=sum(c["lift_strength"] for c in certs),
                psd_projection_delta=sum(c["psd_projection_delta"] for c in certs),
                mass_epsilon_ratio=max(c["mass_epsilon_ratio"] for c in certs),
                trust_alpha=min(c["trust_alpha"] for c in certs),
                power_beta=min(c["power_beta"] for c in certs))


def _block(L3, i0):
    L = np.zeros((D_Z, D_Z))
    L[i0:i0 + 3, i0:i0 + 3] = L3
    return L


# ---------------------------------------------------------------- pipeline helpers
def compute_imu_integration_time(stamps, t_start, t_end):
    """compute_imu_integration_time, FS/backend/pipeline.py:262-313."""
    s = np.asarray(stamps, np.float64)
    eps = 1e-9
    v = s[(s > t_start - eps) & (s <= t_end + eps) & (s > 0.0)]
    if v.shape[0] < 2:
        return 0.0
    v = np.sort(v)
    dt = float(np.sum(np.maximum(v[1:] - v[:-1], 0.0)))
    return max(0.0, min(dt, t_end - t_start))


def dt_imu_and_omega_avg(stamps, gyro, w_int, gyro_bias):
    """Average IMU period and debiased weighted mean rate, FS/backend/pipeline.py:522-548."""
    s = np.asarray(stamps, np.float64)
    valid = s > 0.0
    n_valid = int(valid.sum())
    dt_imu = float((np.sort(s[valid])[-1] - np.sort(s[valid])[0]) / max(n_valid - 1, 1)) if n_valid >= 2 else 0.0
    dt_imu = max(dt_imu, 1e-12)
    w = np.asarray(w_int, np.float64) * valid
    wn = w / (w.sum() + EPS_MASS)
    omega_avg = np.einsum("m,mi->i", wn, np.asarray(gyro, np.float64) - np.asarray(gyro_bias)[None, :])
    if not np.all(np.isfinite(omega_avg)):
        raise ValueError(f"omega_avg contains non-finite values: {omega_avg}")
    return dt_imu, omega_avg


def measurement_noise_mean(nu, Psi, idx):
    """measurement_noise_mean_jax (IW mode), FS/backend/operators/measurement_noise_iw_jax.py:38-56."""
    return psd_project(Psi[idx] / (nu[idx] + 3.0 + 1.0), EPS_PSD)[0]


def kappa_from_resultant_v2(R_bar, eps_r=EPS_R):
    """kappa_from_resultant_v2 + _kappa_continuous_formula, FS/backend/operators/kappa.py:84-127,172-234."""
    R = min(max(float(R_bar), 0.0), 1.0 - eps_r)
    R2 = R * R
    k_low = (R * (3.0 - R2)) / (1.0 - R2 + eps_r)
    k_high = -math.log(max(1.0 - R2, eps_r))
    s = 1.0 / (1.0 + math.exp(-(R - KAPPA_R0) / max(KAPPA_TAU, 1e-6)))
    return (1.0 - s) * k_low + s * k_high


# ---------------------------------------------------------------- operators
def odom_quadratic_evidence(pose_pred, odom_pose, odom_cov):
    """FS/backend/operators/odom_evidence.py:39-154."""
    T_err = se3.se3_compose(se3.se3_inverse(pose_pred), odom_pose)        # se3_relative(odom, pred)
    xi = se3.se3_log(T_err)
    cov_psd, _ = psd_project(odom_cov, EPS_PSD)
    L6, lift = spd_inverse_lifted(cov_psd, EPS_LIFT)
    L = np.zeros((D_Z, D_Z))
    L[0:6, 0:6] = L6
    dz = np.zeros(D_Z)
    dz[0:6] = xi
    h = L @ dz
    nll = 0.5 * (xi @ L6 @ xi)
    return L, h, cert(nll_per_ess=nll, lift_strength=lift)


def _transport_consistency(a, gyro, dt):
    """_compute_transport_consistency, FS/backend/operators/imu_evidence.py:276-333."""
    df = np.zeros_like(a)
    df[1:-1] = (a[2:] - a[:-2]) / (2 * dt + EPS_MASS)
    df[0] = (a[1] - a[0]) / (dt + EPS_MASS)
    df[-1] = (a[-1] - a[-2]) / (dt + EPS_MASS)
    return np.linalg.norm(df + np.cross(gyro, a), axis=1)


def imu_vmf_gravity_evidence_time_resolved(rotvec, accel, gyro, weights, accel_bias, gravity_W, dt_imu):
    """FS/backend/operators/imu_evidence.py:402-559 (with :336-399)."""
    R0 = se3.so3_exp(rotvec)
    g = np.asarray(gravity_W, np.float64)
    g_hat = g / (np.linalg.norm(g) + EPS_MASS)
    accel = np.asarray(accel, np.float64)
    gyro = np.asarray(gyro, np.float64)
    w_base = np.asarray(weights, np.float64)
    ab = np.asarray(accel_bias, np.float64)
    a = accel - ab[None, :]
    e = _transport_consistency(a, gyro, dt_imu)
    med = np.median(e)
    sigma = np.median(np.abs(e - med)) / 0.6745 + EPS_MASS
    rel = np.exp(-0.5 * (e / sigma) ** 2)
    w = w_base * rel
    ess_w, ess_raw = w.sum(), w_base.sum()
    x = a / (np.linalg.norm(a, axis=1, keepdims=True) + EPS_MASS)
    S = np.sum(w[:, None] * x, axis=0)
    S_norm = np.linalg.norm(S)
    xbar = S / (S_norm + EPS_MASS)
    Rbar = S_norm / (ess_w + EPS_MASS)
    kappa = kappa_from_resultant_v2(Rbar)
    mu0 = R0.T @ (-g_hat)
    g_rot = -kappa * np.cross(mu0, xbar)
    H = kappa * ((xbar @ mu0) * np.eye(3) - 0.5 * (np.outer(xbar, mu0) + np.outer(mu0, xbar)))
    H = 0.5 * (H + H.T)
    H_psd, hc = psd_project(H, EPS_PSD)
    L = _block(H_psd, 3)
    h = np.zeros(D_Z)
    h[3:6] = -g_rot
    nll = float(-kappa * (mu0 @ xbar))
    mean_rel = float(np.mean(rel))
    c = cert(ess_total=float(ess_w), support_frac=mean_rel, nll_per_ess=nll / (float(ess_w) + EPS_MASS),
             cond=hc[4], psd_projection_delta=hc[0], mass_epsilon_ratio=float(ess_w) / (float(ess_raw) + EPS_MASS),
             trust_alpha=mean_rel)
    return L, h, c, dict(kappa=kappa, transport_sigma=float(sigma), ess_weighted=float(ess_w), mean_reliability=mean_rel)


def imu_dependence_inflation(transport_sigma):
    """FS/backend/operators/imu_evidence.py:562-589."""
    s = max(float(transport_sigma), 0.0)
    scale = 1.0 / (1.0 + s * s + EPS_MASS)
    return scale, cert(trust_alpha=scale)


def imu_gyro_rotation_evidence(rv_start, rv_end_pred, drv_meas, Sigma_g, dt_int):
    """FS/backend/operators/imu_gyro_evidence.py:38-163."""
    dt_pos = max(float(dt_int), 0.0)
    R_end_imu = se3.so3_exp(rv_start) @ se3.so3_exp(drv_meas)
    r = se3.so3_log(se3.so3_exp(rv_end_pred).T @ R_end_imu)
    dt_eff = dt_pos + EPS_MASS
    ms = dt_pos / dt_eff
    Sig_psd, _ = psd_project(np.asarray(Sigma_g) * dt_eff, EPS_PSD)
    Lr, lift = spd_inverse_lifted(Sig_psd, EPS_LIFT)
    Ls = ms * Lr
    h = np.zeros(D_Z)
    h[3:6] = Ls @ r
    nll = 0.5 * (r @ Lr @ r)
    return _block(Ls, 3), h, cert(nll_per_ess=nll, lift_strength=lift), r


def imu_preintegration_factor(p_start, rv_start, v_start, p_end_pred, v_end_pred, dv_body, dp_body, Sigma_a, dt_int):
    """FS/backend/operators/imu_preintegration_factor.py:46-180."""
    R = se3.so3_exp(rv_start)
    v_imu = v_start + R @ dv_body
    p_imu = p_start + v_start * dt_int + R @ dp_body
    r_v, r_p = v_imu - v_end_pred, p_imu - p_end_pred
    dt_pos = max(float(dt_int), 0.0)
    dt_eff = dt_pos + EPS_MASS
    ms = dt_pos / dt_eff
    Sa = np.asarray(Sigma_a, np.float64)
    Lv, lv = spd_inverse_lifted(psd_project(Sa * dt_eff, EPS_PSD)[0], EPS_LIFT)
    Lp, lp = spd_inverse_lifted(psd_project(Sa * dt_eff ** 3, EPS_PSD)[0], EPS_LIFT)
    L = _block(ms * Lp, 0) + _block(ms * Lv, 6)
    h = np.zeros(D_Z)
    h[0:3] = (ms * Lp) @ r_p
    h[6:9] = (ms * Lv) @ r_v
    nll = 0.5 * (r_v @ Lv @ r_v) + 0.5 * (r_p @ Lp @ r_p)
    return L, h, cert(nll_per_ess=nll, lift_strength=lv + lp)


def planar_z_prior(pose_pred, z_ref, sigma_z):
    """FS/backend/operators/planar_prior.py:55-130."""
    r = float(z_ref - pose_pred[2])
    p = 1.0 / sigma_z ** 2
    L = np.zeros((D_Z, D_Z))
    L[2, 2] = p
    h = np.zeros(D_Z)
    h[2] = p * r
    return L, h, cert(nll_per_ess=0.0)


def velocity_z_prior(vz_pred, sigma_vz):
    """FS/backend/operators/planar_prior.py:138-195."""
    p = 1.0 / sigma_vz ** 2
    L = np.zeros((D_Z, D_Z))
    L[8, 8] = p
    h = np.zeros(D_Z)
    h[8] = p * (-float(vz_pred))
    return L, h, cert()


def odom_velocity_evidence(v_pred_world, R_world_body, v_odom_body, Sigma_v):
    """FS/backend/operators/odom_twist_evidence.py:58-149."""
    r = np.asarray(v_odom_body) - R_world_body.T @ np.asarray(v_pred_world)
    L3, lift = spd_inverse_lifted(psd_project(Sigma_v, EPS_PSD)[0], EPS_LIFT)
    h = np.zeros(D_Z)
    h[6:9] = L3 @ r
    return _block(L3, 6), h, cert(lift_strength=lift)


def odom_yawrate_evidence(wz_pred, wz_odom, sigma_wz):
    """FS/backend/operators/odom_twist_evidence.py:157-228."""
    r = float(wz_odom) - float(wz_pred)
    p = 1.0 / (float(sigma_wz) ** 2)
    L = np.zeros((D_Z, D_Z))
    L[5, 5] = p
    h = np.zeros(D_Z)
    h[5] = p * r
    return L, h, cert()


def pose_twist_kinematic_consistency(pose_prev, pose_curr, v_body, omega_body, dt, Sigma_v, Sigma_omega):
    """FS/backend/operators/odom_twist_evidence.py:251-397."""
    R_prev = se3.so3_exp(pose_prev[3:6])
    R_curr = se3.so3_exp(pose_curr[3:6])
    dp_pred = R_prev @ np.asarray(v_body) * dt
    dth_pred = np.asarray(omega_body) * dt
    r_t = dp_pred - (pose_curr[:3] - pose_prev[:3])
    r_r = dth_pred - se3.so3_log(R_prev.T @ R_curr)
    dt2 = dt * dt + EPS_PSD
    Lt, lt = spd_inverse_lifted(psd_project(dt2 * np.asarray(Sigma_v), EPS_PSD)[0], EPS_LIFT)
    Lr, lr = spd_inverse_lifted(psd_project(dt2 * np.asarray(Sigma_omega), EPS_PSD)[0], EPS_LIFT)
    h = np.zeros(D_Z)
    h[0:3] = Lt @ r_t
    h[3:6] = Lr @ r_r
    return _block(Lt, 0) + _block(Lr, 3), h, cert(lift_strength=lt + lr), r_t, r_r


def odom_dependence_inflation(r_trans, r_rot):
    """FS/backend/operators/odom_twist_evidence.py:400-430."""
    mag = float(np.linalg.norm(r_trans) + np.linalg.norm(r_rot))
    scale = 1.0 / (1.0 + mag * mag + EPS_MASS)
    return scale, cert(trust_alpha=scale)


# ---------------------------------------------------------------- the branch
def imu_odom_branch(*, pose0, pose_pred, mu_prev, mu_inc, imu_stamps, imu_gyro, imu_accel, w_int, dt_imu, omega_avg,
                    dt_int, pre_int, gravity_W, Sigma_g, Sigma_a, odom_pose, odom_cov, odom_twist, odom_twist_cov,
                    dt_sec, planar_z_ref=PLANAR_Z_REF, planar_z_sigma=PLANAR_Z_SIGMA,
                    planar_vz_sigma=PLANAR_VZ_SIGMA):
    """_compute_imu_odom_branch, FS/backend/pipeline.py:595-776 (z_lin_pose, which only the live
    primitive path's visual_pose_evidence reads, is not formed).  Returns L, h, the certs in the
    reference's append order, and diagnostics."""
    odom_twist = np.asarray(odom_twist, np.float64)
    odom_twist_cov = np.asarray(odom_twist_cov, np.float64)
    L_odom, h_odom, c_odom = odom_quadratic_evidence(pose_pred, np.asarray(odom_pose, np.float64), odom_cov)
    L_imu, h_imu, c_imu, imu_info = imu_vmf_gravity_evidence_time_resolved(pose_pred[3:6], imu_accel, imu_gyro, w_int,
                                                                           mu_inc[12:15], gravity_W, dt_imu)
    s_dep, c_dep = imu_dependence_inflation(imu_info["transport_sigma"])
    L_gyro, h_gyro, c_gyro, _ = imu_gyro_rotation_evidence(pose0[3:6], pose_pred[3:6], pre_int["delta_pose"][3:6],
                                                           Sigma_g, dt_int)
    L_pre, h_pre, c_pre = imu_preintegration_factor(pose0[0:3], pose0[3:6], mu_prev[6:9], pose_pred[0:3], mu_inc[6:9],
                                                    pre_int["delta_v"], pre_int["delta_p"], Sigma_a, dt_int)
    L_pl, h_pl, c_pl = planar_z_prior(pose_pred, planar_z_ref, planar_z_sigma)
    L_vz, h_vz, c_vz = velocity_z_prior(mu_inc[8], planar_vz_sigma)
    L_vel, h_vel, c_vel = odom_velocity_evidence(mu_inc[6:9], se3.so3_exp(pose_pred[3:6]), odom_twist[0:3],
                                                 odom_twist_cov[0:3, 0:3])
    sigma_wz = math.sqrt(max(odom_twist_cov[5, 5], 1e-12))
    L_wz, h_wz, c_wz = odom_yawrate_evidence(omega_avg[2], odom_twist[5], sigma_wz)
    L_kin, h_kin, c_kin, r_t, r_r = pose_twist_kinematic_consistency(pose0, pose_pred, odom_twist[0:3],
                                                                     odom_twist[3:6], dt_sec, odom_twist_cov[0:3, 0:3],
                                                                     odom_twist_cov[3:6, 3:6])
    s_odom, c_odep = odom_dependence_inflation(r_t, r_r)
    L = (L_odom * s_odom + L_imu * s_dep + L_gyro * s_dep + L_pre + L_pl + L_vz + L_vel * s_odom + L_wz * s_odom
         + L_kin)
    h = (h_odom * s_odom + h_imu * s_dep + h_gyro * s_dep + h_pre + h_pl + h_vz + h_vel * s_odom + h_wz * s_odom
         + h_kin)
    certs = [c_odom, c_imu, c_dep, c_gyro, c_pre, c_pl, c_vz, c_vel, c_wz, c_kin, c_odep]
    info = dict(imu_scale=s_dep, odom_scale=s_odom, trigger=sum(trigger_magnitude(c) for c in certs), **imu_info)
    return L, h, certs, dict(odom=c_odom, imu=c_imu, gyro=c_gyro), info


def pose6_conditioning(L_ev, eps_cond=EPS_PSD):
    """Pose-block conditioning of the tempered evidence, FS/backend/pipeline.py:1155-1177."""
    Lp = 0.5 * (L_ev[0:6, 0:6] + L_ev[0:6, 0:6].T)
    Lp = np.nan_to_num(Lp, nan=0.0, posinf=0.0, neginf=0.0)
    ev = np.linalg.eigvalsh(Lp)
    evc = np.maximum(np.nan_to_num(ev, nan=eps_cond, posinf=eps_cond, neginf=eps_cond), eps_cond)
    return dict(eig_min=evc[0], eig_max=evc[-1], cond=evc[-1] / evc[0], near_null=int(np.sum(ev <= eps_cond)))


def fusion_scale_from_certificates(cert_ev, alpha_min=ALPHA_MIN, alpha_max=ALPHA_MAX, c0_cond=C0_COND,
                                   excitation_total=0.0, dt_asymmetry=0.0, z_to_xy_ratio=0.0):
    """FS/backend/operators/fusion.py:46-142.  No reference operator fills an ExcitationCert
    (certificates.py:564-567 only aggregates zeros), so excitation_total is 0 in the pipeline."""
    cond_q = c0_cond / (cert_ev["cond"] + c0_cond)
    ess = cert_ev["ess_total"]
    supp_q = ess / (ess + 1.0)
    mis_q = math.exp(-cert_ev["nll_per_ess"])
    dt_q = min(max(dt_asymmetry, 0.0), 1.0)
    z_q = min(max(z_to_xy_ratio / (z_to_xy_ratio + 1.0), 0.0), 1.0)
    exc_q = min(max(excitation_total / (excitation_total + 1.0), 0.0), 1.0)
    base = math.sqrt(cond_q * supp_q)
    quality = base * mis_q * dt_q * z_q * exc_q * min(max(cert_ev["power_beta"], 0.0), 1.0)
    alpha = min(max(alpha_min + (alpha_max - alpha_min) * quality, alpha_min), alpha_max)
    return alpha, quality
