"""The L2 drop-in (gcslam.pipeline: process_scan_single_hypothesis / process_hypotheses with the
reference calling convention, FS/backend/pipeline.py:316-340, :1594-1621) driven by the reference
node's exact per-scan call and unpacking sequence (FS/backend/backend_node.py:2018-2119: Sigma_g /
Sigma_a from the measurement IW state, Q from the process IW state, one
process_scan_single_hypothesis per hypothesis with odometry, weighted IW accumulation,
`combined_belief, combo_cert, combo_effect = process_hypotheses(...)`, process IW apply with weight
min(1, scan_count), Q rebuild, measurement IW apply), against the oracle; plus the output formats
(TUM line, MinimalScanTape) and the RuntimeManifest."""

import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)


def test_node_sequence_matches_oracle():
    from gcslam import synthetic
    from gcslam.certificates import CertBundle, ExpectedEffect
    from gcslam.outputs import MinimalScanTape, tum_line
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, RuntimeManifest, datasheet_measurement_noise_state,
                                 datasheet_process_noise_state, measurement_noise_apply_suffstats,
                                 measurement_noise_mean, process_hypotheses, process_noise_iw_apply_suffstats,
                                 process_noise_state_to_Q, process_scan_single_hypothesis)
    from oracle import ops, pipeline as opipe
    K_HYP = 2
    cfg = PipelineConfig(K_HYP=K_HYP, N_POINTS_CAP=2048, B_BINS=48, soft_assign_mode="dense",
                         lidar_origin_base=ORIGIN, max_raw_points=4096)
    maps = [cfg.make_context() for _ in range(K_HYP)]      # per-hypothesis MapBinStats (declared)
    manifest = RuntimeManifest.from_context(cfg, maps[0]).to_dict()
    assert manifest["N_POINTS_CAP"] == 2048 and manifest["context"]["B_BINS"] == 48
    assert "tau_rule" in manifest and "pushforward_form" in manifest["context"]
    json.dumps(manifest)
    dirs, knn = maps[0].atlas()
    ocfg = opipe.BinPathConfig(n_points_cap=2048, n_bins=48, mode="dense", lidar_origin=ORIGIN, tau=maps[0].cfg.tau)

    hyp_weights = np.full(K_HYP, 1.0 / K_HYP)                # backend_node.py:821-831
    hypotheses = [BeliefGaussianInfo.create_identity_prior() for _ in range(K_HYP)]
    process_state, meas_state = datasheet_process_noise_state(), datasheet_measurement_noise_state()
    # oracle side
    o_hyp = [ops.Belief.identity_prior() for _ in range(K_HYP)]
    o_maps = [opipe.MapState.empty(48) for _ in range(K_HYP)]
    o_proc = ops.datasheet_process_noise_state()
    o_meas = ops.datasheet_measurement_noise_state()
    for scan_count in range(3):
        sc = synthetic.make_scan(4096, 50 + scan_count)
        # per-scan noise proxies from the IW states (backend_node.py:2020-2031)
        cfg.Sigma_g = measurement_noise_mean(meas_state, 0)
        cfg.Sigma_a = measurement_noise_mean(meas_state, 1)
        Q_scan = process_noise_state_to_Q(process_state)
        o_Q = ops.process_noise_Q(*o_proc)
        np.testing.assert_allclose(Q_scan, o_Q, rtol=1e-9, atol=1e-12 * np.abs(o_Q).max())
        accum_dPsi, accum_dnu = np.zeros((7, 6, 6)), np.zeros(7)
        accum_meas_dPsi, accum_meas_dnu = np.zeros((3, 3, 3)), np.zeros(3)
        o_results = []
        for i, belief in enumerate(hypotheses):
            result = process_scan_single_hypothesis(
                belief_prev=belief, raw_points=sc["points"], raw_timestamps=sc["timestamps"],
                raw_weights=sc["weights"], raw_ring=np.zeros(4096, np.uint8), raw_tag=np.zeros(4096, np.uint8),
                imu_stamps=sc["imu_stamps"], imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"],
                odom_pose=sc["odom_pose"], odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"],
                scan_end_time=sc["scan_end_time"], dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"],
                t_scan=sc["t_scan"], Q=Q_scan, config=cfg, odom_twist=sc["odom_twist"],
                odom_twist_cov=sc["odom_twist_cov"], camera_batch=None, scan_seq=scan_count, map_bins=maps[i])
            hypotheses[i] = result.belief_updated
            w_h = float(hyp_weights[i])
            accum_dPsi = accum_dPsi + w_h * result.iw_process_dPsi
            accum_dnu = accum_dnu + w_h * result.iw_process_dnu
            accum_meas_dPsi = accum_meas_dPsi + w_h * result.iw_meas_dPsi
            accum_meas_dnu = accum_meas_dnu + w_h * result.iw_meas_dnu
            ref = opipe.process_scan_bin_path(o_hyp[i], sc, o_Q, ocfg, dirs, knn, o_maps[i], meas_state=o_meas)
            o_results.append(ref)
            np.testing.assert_allclose(result.z_t, ref["z_t"], rtol=1e-7, atol=1e-9)
            np.testing.assert_allclose(result.L_imu_odom, ref["imu_odom"]["L"], rtol=1e-7,
                                       atol=1e-9 * np.abs(ref["imu_odom"]["L"]).max())
            np.testing.assert_allclose(result.iw_process_dPsi, ref["iw_process_dPsi"], rtol=1e-6, atol=1e-12)
            np.testing.assert_allclose(result.iw_meas_dPsi, ref["iw_meas_dPsi"], rtol=1e-9,
                                       atol=1e-13 * np.abs(ref["iw_meas_dPsi"]).max())
            tape = result.diagnostics_tape
            assert isinstance(tape, MinimalScanTape) and tape.scan_number == scan_count
            assert tape.total_trigger_magnitude == pytest.approx(ref["total_trigger"], rel=1e-6, abs=1e-9)
            assert len(tum_line(tape.timestamp, result.z_t).split()) == 8
            o_hyp[i], o_maps[i] = ref["belief"], ref["map"]
        # the node's unpacking of process_hypotheses (backend_node.py:2093-2097)
        combined_belief, combo_cert, combo_effect = process_hypotheses(hypotheses=hypotheses, weights=hyp_weights,
                                                                       config=cfg)
        assert isinstance(combo_cert, CertBundle) and isinstance(combo_effect, ExpectedEffect)
        w_process = min(1, scan_count)
        process_state, _ = process_noise_iw_apply_suffstats(process_state, w_process * accum_dPsi,
                                                             w_process * accum_dnu)
        meas_state, _ = measurement_noise_apply_suffstats(meas_state, 1.0 * accum_meas_dPsi, 1.0 * accum_meas_dnu)
        oc = opipe.combine_and_update_noise(o_results, hyp_weights, o_proc, scan_count, o_meas)
        o_proc, o_meas = oc["iw_state"], oc["meas_state"]
        Lr = oc["combined"]["L"]
        np.testing.assert_allclose(combined_belief.L, Lr, rtol=1e-6, atol=1e-9 * np.abs(Lr).max())
        np.testing.assert_allclose(combined_belief.z_lin, oc["combined"]["z_lin"], rtol=1e-6, atol=1e-9)
        assert combo_effect.predicted == pytest.approx(oc["combined"]["spread"], rel=1e-5, abs=1e-12)
        np.testing.assert_allclose(process_state.nu, o_proc[0], rtol=1e-12)
        np.testing.assert_allclose(process_state.Psi_blocks, o_proc[1], rtol=1e-6, atol=1e-18)
        np.testing.assert_allclose(meas_state.Psi_blocks, o_meas[1], rtol=1e-8, atol=1e-20)
    for m in maps:
        m.close()

