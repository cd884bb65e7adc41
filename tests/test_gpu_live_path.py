"""The live primitive path closed through the L2 drop-in (gcslam.pipeline.process_scan_single_hypothesis
with primitive_map=AtlasMap; FS/backend/pipeline.py:316-1591): budget, predict, IMU preintegration,
deskew and the IMU/odometry branch (gcs_scan_begin), the map branch (surfels on the deskewed points,
recency inflation, the view over the stencil, OT association; :778-926), visual pose evidence at
z_lin_pose as the LiDAR evidence (:980-1010), tempering / fusion / recompose (gcs_scan_finish,
:1038-1230), step 12b at the fused z_t (:1232-1492) and the anchor drift -- three scans in a row, the
belief, IW states and map carried by the node sequence (backend_node.py:2018-2119, hypothesis 0's map
kept: :2079-2083), against oracle.pipeline.process_scan_primitive_path run independently with its own
belief and tiles.  Both sides fuse the device's MeasurementBatch: a cell of two or three collinear
points has no unique plane normal and the reference orients it by the sign of a rounding-level z
component (lidar_surfel_extraction.py:129-130), so the surfel extraction is checked on its own
(tests/test_gpu_surfels.py) and the loop from the batch on."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)


def _close(name, got, ref, rtol, atol):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    bad = ~(np.abs(got - ref) <= atol + rtol * np.abs(ref))
    assert not bad.any(), f"{name}: {bad.sum()} / {bad.size} outside tol; worst {np.abs(got - ref).max():.3e}"


@pytest.mark.parametrize("m_tile", [4096])
def test_live_primitive_path_closed_loop_three_scans(m_tile):
    from gcslam import synthetic
    from gcslam import primitive_map as gpm
    from gcslam.pipeline import (BeliefGaussianInfo, MapUpdateCert, PipelineConfig, datasheet_measurement_noise_state,
                                 datasheet_process_noise_state, measurement_noise_apply_suffstats,
                                 measurement_noise_mean, process_noise_iw_apply_suffstats, process_noise_state_to_Q,
                                 process_scan_single_hypothesis)
    from oracle import ops, pipeline as opipe, primitive_map as opm
    N = 8192
    # three z slabs of tiles (R_*_TILES_Z = 1, 21 tiles): the synthetic platform's z hovers around 0, so
    # a one-slab stencil (the reference default) flips between the z = 0 and z = -1 cells from scan to
    # scan and meets an empty map every other scan
    cfg = PipelineConfig(K_HYP=1, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense", lidar_origin_base=ORIGIN,
                         max_raw_points=N, primitive_map_max_size=m_tile, R_ACTIVE_TILES_Z=1, R_STENCIL_TILES_Z=1,
                         N_ACTIVE_TILES=21, N_STENCIL_TILES=21)
    ctx = cfg.make_context()
    am = gpm.create_empty_atlas_map(m_tile=m_tile, max_tiles=64)
    ocfg = opipe.PrimitivePathConfig(n_points_cap=N, lidar_origin=ORIGIN, m_tile=m_tile, r_active_z=1, r_stencil_z=1)
    belief = BeliefGaussianInfo.create_identity_prior()
    process_state, meas_state = datasheet_process_noise_state(), datasheet_measurement_noise_state()
    o_bel = ops.Belief.identity_prior()
    o_proc, o_meas = ops.datasheet_process_noise_state(), ops.datasheet_measurement_noise_state()
    tiles, nxt = {}, 0
    for scan_seq in range(3):
        sc = synthetic.make_scan(N, 70 + scan_seq)
        cfg.Sigma_g = measurement_noise_mean(meas_state, 0)
        cfg.Sigma_a = measurement_noise_mean(meas_state, 1)
        Q = process_noise_state_to_Q(process_state)
        o_Q = ops.process_noise_Q(*o_proc)
        res = process_scan_single_hypothesis(
            belief_prev=belief, raw_points=sc["points"], raw_timestamps=sc["timestamps"], raw_weights=sc["weights"],
            raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8), imu_stamps=sc["imu_stamps"],
            imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
            odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"], scan_end_time=sc["scan_end_time"],
            dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"], t_scan=sc["t_scan"], Q=Q, config=cfg,
            odom_twist=sc["odom_twist"], odom_twist_cov=sc["odom_twist_cov"], camera_batch=None, scan_seq=scan_seq,
            primitive_map=am, map_bins=ctx)
        mb = res.measurement_batch
        batch = {f: getattr(mb, f).detach().cpu().numpy() for f in ("Lambdas", "thetas", "etas", "weights",
                                                                    "valid_mask", "colors", "sources")}
        batch["valid_mask"] = batch["valid_mask"].astype(bool)
        batch["n_valid"] = mb.n_valid
        ref = opipe.process_scan_primitive_path(o_bel, sc, o_Q, ocfg, tiles, nxt, scan_seq, meas_state=o_meas,
                                                batch=batch)
        nxt = ref["next_global_id"]
        # the map branch's inputs and the LiDAR evidence
        _close(f"scan{scan_seq} z_lin_pose", res.z_lin_pose, ref["z_lin_pose"], 1e-9, 1e-12)
        assert res.measurement_batch.n_valid > 100
        assert res.map is am and isinstance(res.map_update_cert, MapUpdateCert)
        assert res.map_update_cert.n_active_tiles == 21
        assert res.map_update_cert.tile_ids_active == [int(t) for t in ref["active_tile_ids"]]
        Lr = ref["L_evidence"]
        _close(f"scan{scan_seq} L_evidence", res.L_evidence, Lr, 1e-7, 1e-9 * np.abs(Lr).max())
        # the fused pose the map update used (z_t 1e-7) and the map after step 12b (tiles 1e-10)
        _close(f"scan{scan_seq} z_t", res.z_t, ref["z_t"], 1e-7, 1e-9)
        mu = res.map_update_cert
        for k in ("insert_count_total", "fused_count", "evicted_count", "merged_count"):
            assert getattr(mu, k) == ref["map_update"][k], (scan_seq, k)
        assert am.next_global_id == nxt
        for tid in ref["active_tile_ids"]:
            g = am.read_tile(int(tid))
            for f in opm.FIELDS_I64 + ("valid_mask",):
                assert np.array_equal(g[f], tiles[int(tid)][f]), (scan_seq, tid, f)
            for f in opm.FIELDS_F64:
                r = tiles[int(tid)][f]
                _close(f"scan{scan_seq} tile {tid} {f}", g[f], r, 1e-10, 1e-10 * max(1.0, np.abs(r).max()))
        _close(f"scan{scan_seq} iw_process_dPsi", res.iw_process_dPsi, ref["iw_process_dPsi"], 1e-6, 1e-12)
        _close(f"scan{scan_seq} iw_meas_dPsi", res.iw_meas_dPsi, ref["iw_meas_dPsi"], 1e-9,
               1e-13 * np.abs(ref["iw_meas_dPsi"]).max())
        assert res.raw_cert[35] == pytest.approx(ref["total_trigger"], rel=1e-6, abs=1e-9)
        # the node's noise updates (single hypothesis, weight 1)
        process_state, _ = process_noise_iw_apply_suffstats(process_state, min(1, scan_seq) * res.iw_process_dPsi,
                                                             min(1, scan_seq) * res.iw_process_dnu)
        meas_state, _ = measurement_noise_apply_suffstats(meas_state, res.iw_meas_dPsi, res.iw_meas_dnu)
        oc = opipe.combine_and_update_noise([ref], np.ones(1), o_proc, scan_seq, o_meas)
        o_proc, o_meas = oc["iw_state"], oc["meas_state"]
        belief = res.belief_updated
        o_bel = ref["belief"]
        _close(f"scan{scan_seq} belief L", belief.L, o_bel.L, 1e-6, 1e-9 * np.abs(o_bel.L).max())
    assert am.total_count == sum(int(t["valid_mask"].sum()) for t in tiles.values())
    am.close()
    ctx.close()


def test_live_path_hypotheses_share_hypothesis0_map():
    """The node's one map over several hypotheses (backend_node.py:2036-2083): hypothesis 0 updates the
    node map in place; hypothesis 1 (update_map=False) reads it and works on device copies of the tiles
    it touches -- the node map is bit for bit unchanged by it, and its scan equals the same scan run on
    an independent copy of the node map; a second copy of the node map (another GPU's) that replays
    hypothesis 0's map_record with primitive_map_follow stays bitwise the node map."""
    from gcslam import synthetic
    from gcslam import primitive_map as gpm
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, datasheet_process_noise_state,
                                 primitive_map_follow, process_noise_state_to_Q, process_scan_single_hypothesis)
    N, m_tile = 8192, 4096
    cfg = PipelineConfig(K_HYP=2, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense", lidar_origin_base=ORIGIN,
                         max_raw_points=N, primitive_map_max_size=m_tile, R_ACTIVE_TILES_Z=1, R_STENCIL_TILES_Z=1,
                         N_ACTIVE_TILES=21, N_STENCIL_TILES=21)
    ctx0, ctx1, ctx1r = cfg.make_context(), cfg.make_context(), cfg.make_context()
    am, am2 = gpm.create_empty_atlas_map(m_tile=m_tile), gpm.create_empty_atlas_map(m_tile=m_tile)
    scratch_ref = gpm.create_empty_atlas_map(m_tile=m_tile)
    b0 = BeliefGaussianInfo.create_identity_prior()
    b1 = BeliefGaussianInfo.create_identity_prior()
    b1.X_anchor = np.array([0.03, -0.02, 0.0, 0.001, -0.002, 0.004])
    Q = process_noise_state_to_Q(datasheet_process_noise_state())

    def tiles_of(m):
        return {t: m.read_tile(t) for t in m.tile_ids}

    def same(a, b):
        assert set(a) == set(b)
        for t in a:
            for f in a[t]:
                assert np.array_equal(a[t][f], b[t][f]), (t, f)

    for scan_seq in range(3):
        sc = synthetic.make_scan(N, 90 + scan_seq)
        kw = dict(raw_points=sc["points"], raw_timestamps=sc["timestamps"], raw_weights=sc["weights"],
                  raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8), imu_stamps=sc["imu_stamps"],
                  imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
                  odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"],
                  scan_end_time=sc["scan_end_time"], dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"],
                  t_scan=sc["t_scan"], Q=Q, config=cfg, odom_twist=sc["odom_twist"],
                  odom_twist_cov=sc["odom_twist_cov"], camera_batch=None, scan_seq=scan_seq)
        r0 = process_scan_single_hypothesis(belief_prev=b0, primitive_map=am, map_bins=ctx0, **kw)
        assert r0.map is am
        node = tiles_of(am)
        r1 = process_scan_single_hypothesis(belief_prev=b1, primitive_map=am, map_bins=ctx1, update_map=False, **kw)
        assert r1.map is not am
        same(tiles_of(am), node)                      # hypothesis 1 left the node map alone
        full = gpm.create_empty_atlas_map(m_tile=m_tile)
        am.working_copy(am.tile_ids, into=full)       # 64 slots: room for the tiles step 12b creates
        r1r = process_scan_single_hypothesis(belief_prev=b1, primitive_map=full, map_bins=ctx1r, **kw)
        assert np.array_equal(r1.z_t, r1r.z_t) and np.array_equal(r1.belief_updated.L, r1r.belief_updated.L)
        for t in r1.map.tile_ids:                     # its working tiles = the full copy's after the same scan
            g, h = r1.map.read_tile(t), full.read_tile(t)
            for f in g:
                assert np.array_equal(g[f], h[f]), (scan_seq, t, f)
        full.close()
        primitive_map_follow(am2, r0.map_record, cfg)  # another GPU's copy of the node map
        same(tiles_of(am2), node)
        assert am2.next_global_id == am.next_global_id and am2.total_count == am.total_count
        b0, b1 = r0.belief_updated, r1.belief_updated
    for m in (am, am2, scratch_ref):
        m.close()
    for c in (ctx0, ctx1, ctx1r):
        c.close()
