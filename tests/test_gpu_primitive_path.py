"""The live primitive path chained on the GPU over three scans (pipeline.py:778-1011, 1232-1492):
surfels -> active / stencil tiles -> recency inflation -> map view -> OT association -> pose evidence
-> map update at z_t.  Each GPU stage is checked against the oracle applied to the GPU's inputs of
that stage, with the oracle's own map carried alongside the device map from scan to scan, so the test
covers how the operators compose (layouts, tile ids, view order, the map's evolution)."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import association as OA, primitive_evidence as OE, primitive_map as opm, se3
from gcslam import association as GA, primitive_map as gpm, synthetic
from gcslam.surfels import SurfelExtractionConfig, extract_lidar_surfels

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_primitive_path_three_scans():
    M, K = 4096, 8
    am = gpm.AtlasMap(m_tile=M, max_tiles=32, max_merge=0)
    tiles = {}
    nxt = 0
    cfg = SurfelExtractionConfig(n_surfel=1024, n_feat=512)
    cpu = lambda x: x.detach().cpu().numpy()  # noqa: E731
    for k in range(3):
        sc = synthetic.make_scan(8192, k)
        z = np.array([0.15 * k, 0.05 * k, 0.0, 0.0, 0.0, 0.03 * k])
        pts, ts, ws = (torch.as_tensor(sc[f], device=DEV) for f in ("points", "timestamps", "weights"))
        batch, _, _ = extract_lidar_surfels(pts, ts, ws, config=cfg)
        b = {f: cpu(getattr(batch, f)) for f in ("Lambdas", "thetas", "etas", "weights", "valid_mask", "colors",
                                                 "sources")}
        b["n_valid"] = batch.n_valid
        assert batch.n_valid > 100
        active = gpm.ma_hex_stencil_tile_ids(z[:3], 2.0, 1, 0)
        assert active == opm.ma_hex_stencil_tile_ids(z[:3], 2.0, 1, 0) and len(active) == 7
        # recency inflation of the active tiles, then the view over the stencil (pipeline.py:833-849)
        _, _, _, st = gpm.primitive_map_recency_inflate(am, active, 10 + k)
        s_ref = opm.recency_inflate(tiles, active, 10 + k)
        assert st.stale_precision_downscale_total == pytest.approx(s_ref[2], rel=1e-12, abs=1e-300)
        view = gpm.extract_atlas_map_view(am, active, 1024)
        v_ref = opm.extract_atlas_map_view(tiles, active, 1024, M)
        assert np.array_equal(cpu(view.candidate_slots), v_ref["candidate_slots"])
        assert np.array_equal(cpu(view.valid_mask), v_ref["valid_mask"])
        np.testing.assert_allclose(cpu(view.positions), v_ref["positions"], rtol=1e-10, atol=1e-10)
        # association on the device view; the oracle's on the same inputs
        acfg = GA.AssociationConfig(scan_seq=10 + k)
        res, cert, _ = GA.associate_primitives_ot(batch, view, acfg)
        ov = {f: cpu(getattr(view, f)) for f in ("positions", "directions", "kappas", "valid_mask",
                                                 "last_supported_scan_seq", "candidate_tile_ids", "candidate_slots",
                                                 "tile_ids")}
        ov.update(m_tile_view=1024)
        a_ref, _ = OA.associate_primitives_ot(dict(b), ov, OA.AssociationConfig(scan_seq=10 + k))
        assert np.array_equal(cpu(res.candidate_pool_indices), a_ref["candidate_pool_indices"])
        np.testing.assert_allclose(cpu(res.responsibilities), a_ref["responsibilities"], rtol=1e-9, atol=1e-15)
        # pose evidence at z (the IMU/odometry-informed linearisation point in the pipeline)
        vis, vcert, _ = GA.visual_pose_evidence(res, batch, view, z_lin_pose=z)
        assoc = dict(responsibilities=cpu(res.responsibilities), candidate_pool_indices=cpu(res.candidate_pool_indices),
                     row_masses=cpu(res.row_masses), candidate_tile_ids=cpu(res.candidate_tile_ids),
                     candidate_slots=cpu(res.candidate_slots))
        e_ref = OE.visual_pose_evidence(b, ov, assoc, z)
        assert vcert.exact == e_ref["exact"] == (k == 0)     # the first scan meets an empty map
        np.testing.assert_allclose(vis.L_pose, e_ref["L_pose"], rtol=1e-10, atol=1e-10 * np.abs(e_ref["L_pose"]).max())
        # map update at z_t (here z): fuse, novelty insertion, cull / forget
        stats = gpm.primitive_map_update(am, batch, res, z, active, float(sc["scan_end_time"]), 10 + k)
        nxt, s_ref = opm.map_update_step(tiles, nxt, b, assoc, se3.so3_exp(z[3:]), z[:3], active, M,
                                         float(sc["scan_end_time"]), 10 + k)
        assert am.next_global_id == nxt and stats["insert_count_total"] == s_ref["insert_count_total"] > 0
        assert stats["fused_count"] == s_ref["fused_count"] and stats["evicted_count"] == s_ref["evicted_count"]
        for tid in active:
            g = am.read_tile(tid)
            for f in opm.FIELDS_I64 + ("valid_mask",):
                assert np.array_equal(g[f], tiles[tid][f]), (k, tid, f)
            for f in opm.FIELDS_F64:
                r = tiles[tid][f]
                np.testing.assert_allclose(g[f], r, rtol=1e-10, atol=1e-10 * max(1.0, np.abs(r).max()),
                                           err_msg=f"scan {k} tile {tid} {f}")
    assert am.total_count == sum(int(t["valid_mask"].sum()) for t in tiles.values())
    am.close()
