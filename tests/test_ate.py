"""ATE as the reference's evaluation computes it (tools/evaluate_slam.py:220-270: evo association,
initial-pose or Umeyama alignment, APE translation / rotation angle): known answers on CPU."""
import math

import numpy as np
import pytest

from gcslam.outputs import ate, pose6_to_matrix


def _traj(n, seed):
    rng = np.random.default_rng(seed)
    t = np.cumsum(rng.normal(0, 0.1, (n, 3)), axis=0)
    r = np.cumsum(rng.normal(0, 0.05, (n, 3)), axis=0)
    return np.hstack([t, r])


def test_initial_alignment_removes_a_rigid_start_offset():
    gt = _traj(40, 1)
    off = pose6_to_matrix([1.0, -2.0, 0.3, 0.1, -0.2, 0.7])
    est = np.array([off @ pose6_to_matrix(p) for p in gt])  # the same motion started elsewhere
    st = np.arange(40) * 0.1
    r = ate(st, gt, st, est, align="initial")
    assert r["n"] == 40
    assert r["trans"]["rmse"] < 1e-12 and r["rot_deg"]["max"] < 1e-5  # acos near 1: ~1e-8 rad resolution
    raw = ate(st, gt, st, est, align="none")
    assert raw["trans"]["rmse"] > 1.0


def test_initial_alignment_keeps_drift_umeyama_fits_it():
    gt = _traj(50, 2)
    est = gt.copy()
    est[:, 0] += np.linspace(0, 0.5, 50)  # drift along x
    st = np.arange(50) * 0.1
    ri = ate(st, gt, st, est, align="initial")
    ru = ate(st, gt, st, est, align="umeyama")
    e = np.linspace(0, 0.5, 50)
    assert ri["trans"]["rmse"] == pytest.approx(math.sqrt(np.mean(e * e)), rel=1e-9)
    assert ri["trans"]["max"] == pytest.approx(0.5, rel=1e-9)
    assert ru["trans"]["rmse"] < ri["trans"]["rmse"]  # the best fit hides part of the drift


def test_umeyama_recovers_a_rigid_transform_and_association_drops_unmatched():
    gt = _traj(30, 3)
    off = pose6_to_matrix([0.5, 0.2, -0.1, 0.0, 0.0, 1.2])
    est = np.array([off @ pose6_to_matrix(p) for p in gt])
    st_gt = np.arange(30) * 0.1
    st_est = st_gt + 0.002
    r = ate(st_gt, gt, np.concatenate([st_est, [99.0]]), np.concatenate([est, est[:1]]), align="umeyama")
    assert r["n"] == 30 and r["trans"]["rmse"] < 1e-9
    with pytest.raises(ValueError):
        ate(st_gt, gt, st_gt + 100.0, est)
