"""Where the 12-scan synthetic trajectory's drift from ground truth comes from (CPU, oracle only).

The GPU trajectory test (`test_gpu_trajectory.py`) finds the HIP path within 1e-6 m of the oracle
per scan, and both ~0.73 m (ATE) from the synthetic ground truth. Agreement alone cannot show that
the oracle's math is the reference's there. These tests show the mechanism and tie it to reference
lines the oracle restates.

* The fused body velocity collapses to ~0 within the first scan, even from a prior that holds the
  true velocity. The body therefore never translates; the estimate stays near the origin while the
  ground truth moves 1.17 m.
* The cause is the IMU preintegration factor: its vel block is
  h = L_v (v_imu - v_end_pred), a residual in information form
  (imu_preintegration_factor.py:46-180, called at pipeline.py:651-669). The fusion adds it to the
  predicted belief's h unshifted (fusion.py: h_post = h_pred + alpha h_evidence). With L_v
  (~1e6) far above the predicted belief's velocity information, the posterior mean is about the
  residual itself: ~0 whenever the prediction agrees with the IMU.
* With that one factor zeroed, velocity and position start to follow the motion, and the drift
  falls. The odometry factors (pose L ~1e4, twist L ~2.5e3) are three orders weaker, and removing
  them changes nothing.

These are properties of the reference's own equations, restated. Nothing here changes the product
path or the oracle.
"""

import numpy as np
import pytest

from gcslam import synthetic
from oracle import imu_odom, ops, pipeline as opipe

ORIGIN = (0.0, 0.0, 0.5)
B = 48
N_SCANS = 12


def _run(scans, belief):
    bins = ops.fibonacci_atlas(B)
    cfg = opipe.BinPathConfig(n_points_cap=2048, n_bins=B, mode="dense", lidar_origin=ORIGIN,
                              tau=ops.tau_for_bins(B))
    iw = ops.datasheet_process_noise_state()
    meas = ops.datasheet_measurement_noise_state()
    Q = ops.process_noise_Q(*iw)
    ms = opipe.MapState.empty(B)
    zs, vs = [], []
    b = belief
    for s, sc in enumerate(scans):
        r = opipe.process_scan_bin_path(b, sc, Q, cfg, bins, None, ms, meas_state=meas)
        zs.append(np.asarray(r["z_t"], np.float64))
        vs.append(r["belief"].mean_increment()[6:9])
        c = opipe.combine_and_update_noise([r], np.array([1.0]), iw, s, meas)
        Q, iw, meas = c["Q"], c["iw_state"], c["meas_state"]
        b, ms = r["belief"], r["map"]
    return np.stack(zs), np.stack(vs)


@pytest.fixture(scope="module")
def scans():
    sc = [synthetic.make_scan(4096, s) for s in range(N_SCANS)]
    gt = np.stack([synthetic.body_pose(x["scan_end_time"])[0] for x in sc])
    return sc, gt


def _ate(z, gt):
    return float(np.sqrt(np.mean(np.sum((z[:, :3] - gt) ** 2, axis=1))))


def _zeroed(fn):
    def g(*a, **k):
        out = list(fn(*a, **k))
        out[0], out[1] = out[0] * 0.0, out[1] * 0.0
        return tuple(out)
    return g


def test_velocity_collapses_even_from_the_true_velocity(scans):
    sc, gt = scans
    z0, v0 = _run(sc, ops.Belief.identity_prior())
    b = ops.Belief.identity_prior(prior_precision=1.0)
    b.h[6:9] = b.L[6:9, 6:9] @ synthetic.V_BODY          # prior mean velocity = the true 1 m/s
    z1, v1 = _run(sc, b)
    print(f"ATE vs ground truth: identity prior {_ate(z0, gt):.3f} m, true-velocity prior {_ate(z1, gt):.3f} m; "
          f"velocity after scan 0: {v1[0].round(3)}")
    assert _ate(z0, gt) > 0.5
    assert np.abs(v1[0]).max() < 0.1                      # 1 m/s gone after one scan
    assert _ate(z1, gt) > 0.4


def test_the_preintegration_residual_is_what_pins_velocity(scans, monkeypatch):
    sc, gt = scans
    z_all, v_all = _run(sc, ops.Belief.identity_prior())
    monkeypatch.setattr(imu_odom, "imu_preintegration_factor", _zeroed(imu_odom.imu_preintegration_factor))
    z_np, v_np = _run(sc, ops.Belief.identity_prior())
    monkeypatch.undo()
    monkeypatch.setattr(imu_odom, "odom_quadratic_evidence", _zeroed(imu_odom.odom_quadratic_evidence))
    monkeypatch.setattr(imu_odom, "odom_velocity_evidence", _zeroed(imu_odom.odom_velocity_evidence))
    z_no, _ = _run(sc, ops.Belief.identity_prior())
    print(f"final vx: all factors {v_all[-1, 0]:+.3f}, without preintegration {v_np[-1, 0]:+.3f} m/s; "
          f"ATE {_ate(z_all, gt):.3f} -> {_ate(z_np, gt):.3f} m; without odometry pose+velocity {_ate(z_no, gt):.3f} m")
    assert abs(v_all[-1, 0]) < 0.05
    assert v_np[-1, 0] > 0.3                             # velocity follows the motion once the residual is gone
    assert _ate(z_np, gt) < _ate(z_all, gt) - 0.2
    assert abs(_ate(z_no, gt) - _ate(z_all, gt)) < 0.02  # the odometry factors are too weak to matter
