"""Host-side boundary pieces of the L2 drop-in (no GPU): process_hypotheses (hypothesis.py:51-236
through gcs_hypothesis_barycenter), the node-level IW applies and the RuntimeManifest fields."""

import numpy as np
import pytest


def test_process_hypotheses_has_no_side_effects_and_checks_k():
    """process_hypotheses is the barycenter only (hypothesis.py:51-117): no context, no IW update,
    and K_HYP / weight-shape validation as the reference (hypothesis.py:172-175)."""
    from gcslam.pipeline import BeliefGaussianInfo, PipelineConfig, process_hypotheses
    from oracle import ops
    rng = np.random.default_rng(1)
    hyps = []
    for _ in range(4):
        A = rng.normal(size=(22, 22))
        hyps.append(BeliefGaussianInfo("GC-RIGHT-01", "a", np.zeros(6), 0.0, rng.normal(0, 1e-3, 22),
                                       A @ A.T + 22 * np.eye(22), rng.normal(size=22)))
    cfg = PipelineConfig(K_HYP=4)
    w = np.array([0.5, 0.3, 0.199, 0.001])
    b, cert, eff = process_hypotheses(hyps, w, cfg)
    ref = ops.hypothesis_barycenter(np.stack([h.L for h in hyps]), np.stack([h.h for h in hyps]),
                                    np.stack([h.z_lin for h in hyps]), w)
    np.testing.assert_allclose(b.L, ref["L"], rtol=1e-12, atol=1e-12 * np.abs(ref["L"]).max())
    np.testing.assert_allclose(b.h, ref["h"], rtol=1e-12, atol=1e-14)
    assert eff.predicted == pytest.approx(ref["spread"], rel=1e-9)
    assert cert.influence.mass_epsilon_ratio == pytest.approx((0.0025 - 0.001) / 4, rel=1e-12)
    with pytest.raises(ValueError):
        process_hypotheses(hyps[:3], w[:3], cfg)


def test_node_noise_updates_match_oracle():
    """process / measurement IW applies, Q and the IW mode (backend_node.py:2020-2023,2102-2119)."""
    from gcslam.pipeline import (datasheet_measurement_noise_state, datasheet_process_noise_state,
                                 measurement_noise_apply_suffstats, measurement_noise_mean,
                                 process_noise_iw_apply_suffstats, process_noise_state_to_Q)
    from oracle import imu_odom, ops
    rng = np.random.default_rng(2)
    ps, ms = datasheet_process_noise_state(), datasheet_measurement_noise_state()
    nu, Psi = ops.datasheet_process_noise_state()
    mnu, mPsi = ops.datasheet_measurement_noise_state()
    np.testing.assert_array_equal(ps.nu, nu)
    np.testing.assert_array_equal(ps.Psi_blocks, Psi)
    np.testing.assert_array_equal(ms.Psi_blocks, mPsi)
    for _ in range(3):
        dPsi = np.stack([np.outer(v, v) for v in rng.normal(0, 1e-3, (7, 6))]) * ops.PROCESS_BLOCK_MASKS
        mdP = np.stack([np.outer(v, v) for v in rng.normal(0, 1e-3, (3, 3))])
        ps, _ = process_noise_iw_apply_suffstats(ps, dPsi, np.ones(7))
        nu, Psi, _ = ops.process_noise_iw_apply(nu, Psi, dPsi, np.ones(7))
        ms, _ = measurement_noise_apply_suffstats(ms, mdP, np.array([1.0, 1.0, 0.0]))
        mnu, mPsi, _ = ops.measurement_noise_iw_apply(mnu, mPsi, mdP, np.array([1.0, 1.0, 0.0]))
        np.testing.assert_allclose(ps.nu, nu, rtol=1e-14)
        np.testing.assert_allclose(ps.Psi_blocks, Psi, rtol=1e-9, atol=1e-20)
        np.testing.assert_allclose(ms.Psi_blocks, mPsi, rtol=1e-9, atol=1e-20)
        np.testing.assert_allclose(process_noise_state_to_Q(ps), ops.process_noise_Q(nu, Psi), rtol=1e-9, atol=1e-20)
        for idx in range(3):
            np.testing.assert_allclose(measurement_noise_mean(ms, idx), imu_odom.measurement_noise_mean(mnu, mPsi, idx),
                                       rtol=1e-9, atol=1e-22)


def test_config_defaults_and_manifest(lib):
    import ctypes as C
    from gcslam import _lib as L
    from gcslam.pipeline import PipelineConfig, RuntimeManifest
    c = L.GcsConfig()
    assert lib.gcs_config_defaults(C.byref(c)) == 0
    assert (c.n_points_cap, c.n_bins, c.use_imu_odom, c.alpha_min, c.alpha_max, c.c0_cond) == (8192, 48, 1, 1.0, 1.0, 1e6)
    assert (c.planar_z_sigma, c.planar_vz_sigma, c.imu_gravity_scale, c.gravity_W[2]) == (0.1, 0.01, 1.0, -9.81)
    d = RuntimeManifest(config=PipelineConfig(B_BINS=100000, N_POINTS_CAP=65536, soft_assign_mode="scale")).to_dict()
    assert d["tau_soft_assign"] == pytest.approx(0.1 * 48 / 100000) and d["N_POINTS_CAP"] == 65536
    assert "declared" in d["candidate_rule"] and d["K_HYP"] == 4
