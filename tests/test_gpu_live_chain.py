"""The one-call live primitive path (gcs_live_scan: begin -> surfels -> recency -> view -> association ->
visual pose evidence -> finish -> step 12b on one stream; pipeline.py:316-1591 with :778-1011,
1232-1492) against the per-operator path (GCSLAM_LIVE_CHAIN=0: one C-ABI call per operator, a host
wait after each), bit for bit: the same kernels on the same arguments must give the same belief, z_t,
certificates, batch, view, association, MapUpdateCert, map bookkeeping and every field of every tile,
scan after scan -- including scans that create tiles on slots a working copy had written, and a
hypothesis k > 0 (update_map=False) that reads the node's map through a working copy."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)
N = 8192


def _run(chain, monkeypatch, n_scans=5, hyp1_every=2):
    from gcslam import _lib as L
    from gcslam import primitive_map as gpm
    from gcslam import synthetic
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, datasheet_process_noise_state,
                                 process_noise_state_to_Q, process_scan_single_hypothesis)
    monkeypatch.setenv("GCSLAM_LIVE_CHAIN", "1" if chain else "0")
    cfg = PipelineConfig(K_HYP=1, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense", lidar_origin_base=ORIGIN,
                         max_raw_points=N, primitive_map_max_size=4096, R_ACTIVE_TILES_Z=1, R_STENCIL_TILES_Z=1,
                         N_ACTIVE_TILES=21, N_STENCIL_TILES=21)
    ctx, ctx1 = cfg.make_context(), cfg.make_context()
    am = gpm.create_empty_atlas_map(m_tile=4096, max_tiles=64)
    Q = process_noise_state_to_Q(datasheet_process_noise_state())
    belief = BeliefGaussianInfo.create_identity_prior()
    rows = []
    for s in range(n_scans):
        sc = synthetic.make_scan(N, 90 + s)
        kw = dict(raw_points=sc["points"], raw_timestamps=sc["timestamps"], raw_weights=sc["weights"],
                  raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8), imu_stamps=sc["imu_stamps"],
                  imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
                  odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"],
                  scan_end_time=sc["scan_end_time"], dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"],
                  t_scan=sc["t_scan"], Q=Q, config=cfg, odom_twist=sc["odom_twist"],
                  odom_twist_cov=sc["odom_twist_cov"], camera_batch=None, scan_seq=s, primitive_map=am)
        hyp1 = None
        if s % hyp1_every == 1:  # a second hypothesis reads the node's map (working copy), then hypothesis 0
            hyp1 = process_scan_single_hypothesis(belief_prev=belief, map_bins=ctx1, update_map=False, **kw)
        res = process_scan_single_hypothesis(belief_prev=belief, map_bins=ctx, **kw)
        belief = res.belief_updated
        row = dict(res=res, hyp1=hyp1, tiles={t: am.read_tile(t) for t in am.tile_ids},
                   book=(dict(am.tiles), dict(am.counts), am.next_global_id, am.total_count, list(am._free)))
        if hyp1 is not None:
            row["hyp1_tiles"] = {t: hyp1.map.read_tile(t) for t in hyp1.map.tile_ids}
        rows.append(row)
    ctx.close()
    ctx1.close()
    return rows


def _arr(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def _same(name, a, b):
    a, b = _arr(a), _arr(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (name, a.shape, b.shape, a.dtype, b.dtype)
    assert a.tobytes() == b.tobytes(), f"{name}: {np.flatnonzero(a.ravel() != b.ravel())[:8]}"


def _same_result(tag, r, q):
    _same(f"{tag} z_t", r.z_t, q.z_t)
    for f in ("L", "h", "z_lin", "X_anchor"):
        _same(f"{tag} belief.{f}", getattr(r.belief_updated, f), getattr(q.belief_updated, f))
    _same(f"{tag} raw_cert", r.raw_cert, q.raw_cert)
    _same(f"{tag} L_evidence", r.L_evidence, q.L_evidence)
    assert len(r.all_certs) == len(q.all_certs)
    for k, (c, d) in enumerate(zip(r.all_certs, q.all_certs)):
        assert c == d, f"{tag} cert {k}: {c} != {d}"
    mb, nb = r.measurement_batch, q.measurement_batch
    assert mb.n_valid == nb.n_valid
    for f in ("Lambdas", "thetas", "etas", "weights", "timestamps", "colors", "sources", "source_indices",
              "valid_mask"):
        _same(f"{tag} batch.{f}", getattr(mb, f), getattr(nb, f))
    for f in ("positions", "covariances", "directions", "kappas", "weights", "primitive_ids",
              "last_supported_scan_seq", "etas", "colors", "candidate_tile_ids", "candidate_slots", "valid_mask",
              "tile_ids"):
        _same(f"{tag} view.{f}", getattr(r.map_view, f), getattr(q.map_view, f))
    for f in ("responsibilities", "candidate_pool_indices", "candidate_tile_ids", "candidate_slots", "row_masses",
              "cost_matrix"):
        _same(f"{tag} association.{f}", getattr(r.association, f), getattr(q.association, f))
    assert r.association.candidate_stats == q.association.candidate_stats
    assert r.map_update_cert == q.map_update_cert, (r.map_update_cert, q.map_update_cert)
    _same(f"{tag} z_lin_pose", r.z_lin_pose, q.z_lin_pose)
    assert r.map_record["active"] == q.map_record["active"]


def _same_tiles(tag, ta, tb):
    assert sorted(ta) == sorted(tb), tag
    for t in ta:
        for f in ta[t]:
            _same(f"{tag} tile {t} {f}", ta[t][f], tb[t][f])


def test_live_chain_bitwise_equals_per_operator_path(monkeypatch):
    chain = _run(True, monkeypatch)
    per_op = _run(False, monkeypatch)
    for s, (a, b) in enumerate(zip(chain, per_op)):
        _same_result(f"scan {s}", a["res"], b["res"])
        assert a["book"] == b["book"], f"scan {s}: map bookkeeping"
        _same_tiles(f"scan {s}", a["tiles"], b["tiles"])
        if b["hyp1"] is not None:
            _same_result(f"scan {s} hyp1", a["hyp1"], b["hyp1"])
            _same_tiles(f"scan {s} hyp1", a["hyp1_tiles"], b["hyp1_tiles"])

