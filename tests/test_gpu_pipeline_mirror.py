"""The L2 drop-in (gcslam.pipeline: process_scan_single_hypothesis / process_hypotheses with the
reference calling convention, FS/backend/pipeline.py:316-340, :1594-1621) against the oracle, plus
the output formats it feeds (TUM line, MinimalScanTape)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)


def test_process_scan_single_hypothesis_matches_oracle():
    from gcslam import synthetic
    from gcslam.outputs import MinimalScanTape, tum_line
    from gcslam.pipeline import BeliefGaussianInfo, PipelineConfig, process_hypotheses, process_scan_single_hypothesis
    from oracle import ops, pipeline as opipe
    cfg = PipelineConfig(N_POINTS_CAP=2048, B_BINS=48, soft_assign_mode="dense", lidar_origin_base=ORIGIN,
                         max_raw_points=4096)
    ctx = cfg.make_context()
    dirs, knn = ctx.atlas()
    ocfg = opipe.BinPathConfig(n_points_cap=2048, n_bins=48, mode="dense", lidar_origin=ORIGIN, tau=ctx.cfg.tau)
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    b_ref, ms = ops.Belief.identity_prior(), opipe.MapState.empty(48)
    bel = BeliefGaussianInfo.create_identity_prior()
    for k in range(2):
        sc = synthetic.make_scan(4096, 50 + k)
        res = process_scan_single_hypothesis(
            bel, sc["points"].astype(np.float32), sc["timestamps"], sc["weights"], None, None, sc["imu_stamps"],
            sc["imu_gyro"], sc["imu_accel"], np.zeros(6), 1e12 * np.eye(6), sc["scan_start_time"],
            sc["scan_end_time"], sc["dt_sec"], sc["t_last_scan"], sc["t_scan"], Q, cfg, scan_seq=k, map_bins=ctx)
        ref = opipe.process_scan_bin_path(b_ref, sc, Q, ocfg, dirs, knn, ms)
        np.testing.assert_allclose(res.z_t, ref["z_t"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(res.belief_updated.X_anchor, ref["belief"].X_anchor, rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(res.iw_process_dPsi, ref["iw_process_dPsi"], rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(res.iw_meas_dPsi, ref["iw_meas_dPsi"], rtol=1e-9,
                                   atol=1e-13 * np.abs(ref["iw_meas_dPsi"]).max())
        assert res.iw_meas_dPsi.shape == (3, 3, 3) and np.array_equal(res.iw_meas_dnu, [1.0, 1.0, 0.0])
        tape = res.diagnostics_tape
        assert isinstance(tape, MinimalScanTape) and tape.scan_number == k and tape.L_pose6.shape == (6, 6)
        assert tape.total_trigger_magnitude == pytest.approx(ref["total_trigger"], rel=1e-6, abs=1e-9)
        assert len(tum_line(tape.timestamp, res.z_t).split()) == 8
        bel, b_ref, ms = res.belief_updated, ref["belief"], ref["map"]
    # two hypotheses -> barycenter (hypothesis.py:51-117)
    b2 = BeliefGaussianInfo(bel.chart_id, bel.anchor_id, bel.X_anchor, bel.stamp_sec, bel.z_lin * 0.5, bel.L * 2.0,
                            bel.h)
    comb, cert = process_hypotheses([bel, b2], np.array([0.7, 0.3]), cfg, ctx)
    ref = ops.hypothesis_barycenter(np.stack([bel.L, b2.L]), np.stack([bel.h, b2.h]), np.stack([bel.z_lin, b2.z_lin]),
                                    np.array([0.7, 0.3]))
    np.testing.assert_allclose(comb.L, ref["L"], rtol=1e-12, atol=1e-12 * np.abs(ref["L"]).max())
    np.testing.assert_allclose(comb.h, ref["h"], rtol=1e-12, atol=1e-14)
    ctx.close()
