"""Step 9 IMU / odometry evidence family (FS/backend/pipeline.py:595-776): the host C++ branch
(gcs_imu_odom_evidence, gcs_evidence.cpp) against the numpy oracle (oracle/imu_odom.py), on the
reference's own raw Kimera IMU/odometry data (tests/golden/kimera_imu_odom_windows.npz, made by
make_kimera_windows.py from /root/reference/docs/raw_sensor_dump) and on synthetic windows, plus
closed-form known answers.  Host numerics only: no GPU."""

import ctypes as C
import math

import numpy as np
import pytest

from golden_util import load
from gcslam import synthetic
from oracle import imu_odom, ops, se3

TOL = dict(rtol=1e-9, atol=1e-12)


def _inputs(st, gy, ac, t_last, t_scan, dt_sec, pose0, pose_pred, mu_prev, mu_inc, odom_pose, odom_cov, twist, twist_cov,
            sigma_warp=0.01, Sg=None, Sa=None):
    w_int = ops.smooth_window_weights(st, t_last, t_scan, sigma_warp)
    nu, Psi = ops.datasheet_measurement_noise_state()
    Sg = imu_odom.measurement_noise_mean(nu, Psi, 0) if Sg is None else Sg
    Sa = imu_odom.measurement_noise_mean(nu, Psi, 1) if Sa is None else Sa
    return dict(stamps=st, gyro=gy, accel=ac, w_int=w_int, t_last_scan=t_last, t_scan=t_scan, dt_sec=dt_sec,
                pose0=pose0, pose_pred=pose_pred, mu_prev=mu_prev, mu_inc=mu_inc,
                gravity_W=np.array(ops.GRAVITY_W), Sigma_g=Sg, Sigma_a=Sa, odom_pose=odom_pose, odom_cov_se3=odom_cov,
                odom_twist=twist, odom_twist_cov=twist_cov)


def _oracle(d):
    dt_int = imu_odom.compute_imu_integration_time(d["stamps"], d["t_last_scan"], d["t_scan"])
    dt_imu, om = imu_odom.dt_imu_and_omega_avg(d["stamps"], d["gyro"], d["w_int"], d["mu_inc"][9:12])
    pre = ops.preintegrate_imu(d["stamps"], d["gyro"], d["accel"], d["w_int"], d["pose0"][3:6], d["mu_inc"][9:12],
                               d["mu_inc"][12:15], d["gravity_W"])
    L, h, certs, named, info = imu_odom.imu_odom_branch(
        pose0=d["pose0"], pose_pred=d["pose_pred"], mu_prev=d["mu_prev"], mu_inc=d["mu_inc"], imu_stamps=d["stamps"],
        imu_gyro=d["gyro"], imu_accel=d["accel"], w_int=d["w_int"], dt_imu=dt_imu, omega_avg=om, dt_int=dt_int,
        pre_int=pre, gravity_W=d["gravity_W"], Sigma_g=d["Sigma_g"], Sigma_a=d["Sigma_a"], odom_pose=d["odom_pose"],
        odom_cov=d["odom_cov_se3"], odom_twist=d["odom_twist"], odom_twist_cov=d["odom_twist_cov"],
        dt_sec=d["dt_sec"])
    return L, h, named, info, dt_int, dt_imu, om


def _hip(lib, d):
    from gcslam import _lib as L
    keep = {k: np.ascontiguousarray(v, np.float64) for k, v in d.items() if isinstance(v, np.ndarray)}
    s = L.GcsImuOdomInputs()
    s.m = keep["stamps"].shape[0]
    for k, v in keep.items():
        setattr(s, k, v.ctypes.data)
    s.t_last_scan, s.t_scan, s.dt_sec = d["t_last_scan"], d["t_scan"], d["dt_sec"]
    s.planar_z_ref, s.planar_z_sigma, s.planar_vz_sigma = 0.0, 0.1, 0.01
    Lm, h, cert = np.zeros(484), np.zeros(22), np.zeros(L.IMU_ODOM_CERT_LEN)
    assert lib.gcs_imu_odom_evidence(C.byref(s), L.dptr(Lm), L.dptr(h), L.dptr(cert)) == 0
    return Lm.reshape(22, 22), h, cert


def _check(lib, d):
    L_o, h_o, named, info, dt_int, dt_imu, om = _oracle(d)
    L_h, h_h, cert = _hip(lib, d)
    sc = np.abs(L_o).max()
    np.testing.assert_allclose(L_h, L_o, rtol=1e-9, atol=1e-12 * sc)
    np.testing.assert_allclose(h_h, h_o, rtol=1e-9, atol=1e-12 * max(np.abs(h_o).max(), 1.0))
    np.testing.assert_allclose(cert[0], info["trigger"], rtol=1e-9)
    np.testing.assert_allclose(cert[1:7], [info["ess_weighted"], info["kappa"], info["transport_sigma"],
                                           info["imu_scale"], info["odom_scale"], info["mean_reliability"]], **TOL)
    np.testing.assert_allclose(cert[7:10], [named["odom"]["nll_per_ess"], named["imu"]["nll_per_ess"],
                                            named["gyro"]["nll_per_ess"]], rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(cert[10:15], [dt_int, dt_imu, *om], **TOL)
    assert np.all(np.isfinite(L_h)) and np.allclose(L_h, L_h.T, atol=1e-9 * sc)
    return L_o, h_o, info


def test_kimera_windows_match_oracle(lib):
    """The reference's raw bag IMU (extrinsic applied) and odometry, 11 scan windows."""
    g = load("kimera_imu_odom_windows")
    rng = np.random.default_rng(3)
    for k in range(1, g["t_scan"].shape[0]):
        pose0 = g["odom_pose"][k - 1]
        pose_pred = g["odom_pose"][k] + np.concatenate([rng.normal(0, 0.01, 3), rng.normal(0, 0.002, 3)])
        mu_prev = np.concatenate([rng.normal(0, 1e-3, 6), g["odom_twist"][k - 1][:3], rng.normal(0, 1e-4, 13)])
        mu_inc = np.concatenate([rng.normal(0, 1e-3, 6), g["odom_twist"][k][:3], rng.normal(0, 1e-3, 3),
                                 rng.normal(0, 1e-2, 3), rng.normal(0, 1e-4, 7)])
        d = _inputs(g["imu_stamps"][k], g["imu_gyro"][k], g["imu_accel"][k], float(g["t_last_scan"][k]),
                    float(g["t_scan"][k]), 0.1, pose0, pose_pred, mu_prev, mu_inc, g["odom_pose"][k],
                    g["odom_cov_se3"], g["odom_twist"][k], g["odom_twist_cov"])
        L_o, h_o, info = _check(lib, d)
        # a level, slowly moving robot: gravity direction well concentrated
        assert info["kappa"] > 1.0 and 0.0 < info["imu_scale"] <= 1.0 and 0.0 < info["odom_scale"] <= 1.0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_synthetic_windows_match_oracle(lib, seed):
    sc = synthetic.make_scan(16, 40 + seed)
    rng = np.random.default_rng(seed)
    pose0 = np.concatenate([rng.normal(0, 0.2, 3), rng.normal(0, 0.1, 3)])
    pose_pred = se3.se3_compose(pose0, np.array([0.1, 0.0, 0.0, 0.0, 0.0, 0.03]))
    mu_prev = rng.normal(0, 1e-2, 22)
    mu_inc = rng.normal(0, 1e-2, 22)
    d = _inputs(sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], sc["t_last_scan"], sc["t_scan"], 0.1, pose0,
                pose_pred, mu_prev, mu_inc, sc["odom_pose"], sc["odom_cov_se3"], sc["odom_twist"],
                sc["odom_twist_cov"], sigma_warp=0.02)
    _check(lib, d)


def test_no_odometry_defaults_are_negligible(lib):
    """Missing odometry (node defaults: identity pose, 1e12 I covariances) contributes ~1e-12 information."""
    sc = synthetic.make_scan(16, 7)
    big = imu_odom.ODOM_COV_MISSING * np.eye(6)
    z = np.zeros(22)
    d = _inputs(sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], sc["t_last_scan"], sc["t_scan"], 0.1, np.zeros(6),
                np.zeros(6), z, z, np.zeros(6), big, np.zeros(6), big)
    L_o, _, _, info, *_ = _oracle(d)
    _check(lib, d)
    assert info["odom_scale"] == pytest.approx(1.0, abs=1e-9)
    # the odometry pose / velocity / yaw-rate / kinematic factors carry 1e-12-level information
    blocks = [imu_odom.odom_quadratic_evidence(np.zeros(6), np.zeros(6), big)[0],
              imu_odom.odom_velocity_evidence(np.zeros(3), np.eye(3), np.zeros(3), big[:3, :3])[0],
              imu_odom.odom_yawrate_evidence(0.0, 0.0, math.sqrt(big[5, 5]))[0],
              imu_odom.pose_twist_kinematic_consistency(np.zeros(6), np.zeros(6), np.zeros(3), np.zeros(3), 0.1,
                                                        big[:3, :3], big[3:, 3:])[0]]
    assert max(np.abs(b).max() for b in blocks) < 1e-9


def test_known_answers():
    # planar prior (planar_prior.py:55-130): L[2,2] = 1/sigma^2, h[2] = (z_ref - z)/sigma^2
    L, h, c = imu_odom.planar_z_prior(np.array([0, 0, 0.3, 0, 0, 0.0]), 0.0, 0.1)
    assert L[2, 2] == pytest.approx(100.0) and h[2] == pytest.approx(-30.0) and ops.trigger_magnitude(c) == 0.0
    # odometry equal to the prediction: zero residual, h = 0, L = (cov + 0)^-1
    cov = np.diag([1e-2] * 3 + [1e-3] * 3)
    p = np.array([1.0, 2.0, 0.1, 0.01, -0.02, 0.5])
    L, h, c = imu_odom.odom_quadratic_evidence(p, p, cov)
    assert np.allclose(h, 0.0, atol=1e-9) and L[0, 0] == pytest.approx(100.0, rel=1e-6)
    # gyro factor with the IMU delta exactly consistent: residual 0
    rv0 = np.array([0.01, 0.02, 0.3])
    dr = np.array([0.0, 0.0, 0.05])
    end = se3.so3_log(se3.so3_exp(rv0) @ se3.so3_exp(dr))
    _, h, _, r = imu_odom.imu_gyro_rotation_evidence(rv0, end, dr, 1e-3 * np.eye(3), 0.1)
    assert np.allclose(r, 0.0, atol=1e-12) and np.allclose(h, 0.0, atol=1e-6)
    # scalar kappa = batch kappa (test_audit_invariants.py:412-426)
    for rb in (0.0, 0.3, 0.8, 0.95, 0.999999):
        assert imu_odom.kappa_from_resultant_v2(rb) == pytest.approx(float(ops.kappa_from_resultant_batch(np.array([rb]))[0]),
                                                                     rel=1e-12)
    # integration time: samples in (t0, t1], at most t1 - t0
    st = np.concatenate([np.arange(1, 30) * 0.005 + 10.0, np.zeros(10)])
    assert imu_odom.compute_imu_integration_time(st, 10.0, 10.1) == pytest.approx(0.095, abs=1e-12)
    # fusion scale: no excitation anywhere -> quality 0 -> alpha = alpha_min
    a, q = imu_odom.fusion_scale_from_certificates(dict(cond=10.0, ess_total=5.0, nll_per_ess=0.1, power_beta=0.25),
                                                   alpha_min=0.5, alpha_max=1.0, dt_asymmetry=0.3, z_to_xy_ratio=0.5)
    assert q == 0.0 and a == 0.5
    a, q = imu_odom.fusion_scale_from_certificates(dict(cond=10.0, ess_total=5.0, nll_per_ess=0.1, power_beta=0.25),
                                                   alpha_min=0.5, alpha_max=1.0, dt_asymmetry=0.3, z_to_xy_ratio=0.5,
                                                   excitation_total=2.0)
    assert 0.0 < q < 1.0 and a == pytest.approx(0.5 + 0.5 * q)
    assert math.isfinite(a)
