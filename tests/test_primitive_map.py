"""CPU tests of the primitive-map oracle (oracle/primitive_map.py): the reference's own tests for
these operators restated (test_primitive_map_merge_reduce.py, test_map_color_provenance.py) and
closed forms.  No GPU."""

import numpy as np
import pytest

from oracle import primitive_map as pm


def _merge_tile():
    """test_primitive_map_merge_reduce.py:11-73: three unit-precision primitives at x = 0, 0.01, 10."""
    t = pm.create_empty_tile(3)
    t["Lambdas"][:] = np.eye(3)
    mu = np.array([[0.0, 0.0, 0.0], [0.01, 0.0, 0.0], [10.0, 0.0, 0.0]])
    t["thetas"][:] = np.einsum("nij,nj->ni", t["Lambdas"], mu)
    t["weights"][:] = 1.0
    t["primitive_ids"][:] = [0, 1, 2]
    t["valid_mask"][:] = True
    t["cam_mass"][:] = [1.0, 0.0, 0.0]
    t["lidar_mass"][:] = [0.0, 1.0, 1.0]
    t["rgb_cam_accum"][0] = [1.0, 0.0, 0.0]
    t["rgb_cam_denom"][:] = [1.0, 0.0, 0.0]
    t["rgb"][0] = [1.0, 0.0, 0.0]
    return t


def test_merge_reduce_merges_close_pair():
    """test_primitive_map_merge_reduce.py:76-98."""
    t = _merge_tile()
    n, status, pairs = pm.merge_reduce(t, merge_threshold=0.5, max_pairs=1, max_tile_size=10)
    assert n == 1 and status == "merged" and pairs == [(0, 1)]
    assert t["valid_mask"][0] and not t["valid_mask"][1]
    assert np.isclose(t["weights"][0], 2.0)
    assert int(t["valid_mask"].sum()) == 2
    # closed form of the moment match: mean 0.005, covariance I/(1 + eps_lift) + 0.005^2 e_x e_x^T + eps_psd I
    Sm = np.eye(3) * (1.0 / (1.0 + 1e-9) + 1e-12)
    Sm[0, 0] += 0.005 ** 2
    assert np.allclose(np.linalg.solve(t["Lambdas"][0], t["thetas"][0]), [0.005, 0, 0], atol=1e-12)
    assert np.allclose(np.linalg.inv(t["Lambdas"][0]), Sm, rtol=1e-12, atol=1e-15)
    assert np.allclose(t["rgb"][0], [1.0, 0.0, 0.0])  # camera mass carried over


def test_merge_reduce_cap_and_noop():
    t = _merge_tile()
    assert pm.merge_reduce(t, merge_threshold=0.5, max_pairs=1, max_tile_size=2)[1] == "cap"
    t = _merge_tile()
    assert pm.merge_reduce(t, merge_threshold=1e-12, max_pairs=4, max_tile_size=10)[:2] == (0, "noop")


def _insert_single(tile, color, source):
    """test_map_color_provenance.py:18-38."""
    return pm.insert_masked(tile, 0, np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, 3, 3)), np.array([1.0]), 0.0,
                            np.array([True]), scan_seq=0, colors_new=np.array([color]), sources_new=np.array([source]))


def _fuse_single(tile, color, source):
    """test_map_color_provenance.py:41-66."""
    return pm.fuse(tile, np.array([0]), np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, 3, 3)), np.array([1.0]),
                   np.array([1.0]), 1.0, scan_seq=1, valid_mask=np.array([True]), colors_meas=np.array([color]),
                   sources_meas=np.array([source]))


def test_camera_then_lidar_keeps_camera_color():
    """test_map_color_provenance.py:69-74."""
    t = pm.create_empty_tile(1)
    _insert_single(t, [1.0, 0.0, 0.0], 0)
    _fuse_single(t, [0.2, 0.2, 0.2], 1)
    assert np.allclose(t["rgb"][0], [1.0, 0.0, 0.0], atol=1e-6)


def test_lidar_then_camera_switches_to_camera_color():
    """test_map_color_provenance.py:77-82."""
    t = pm.create_empty_tile(1)
    _insert_single(t, [0.2, 0.2, 0.2], 1)
    _fuse_single(t, [0.0, 1.0, 0.0], 0)
    assert np.allclose(t["rgb"][0], [0.0, 1.0, 0.0], atol=1e-6)


def test_insert_fills_empty_slots_first_with_contiguous_ids():
    t = pm.create_empty_tile(8)
    t["valid_mask"][[1, 4]] = True
    t["weights"][[1, 4]] = [0.3, 0.1]
    K = 4
    do = np.array([True, False, True, True])
    n, ids, dropped, nxt = pm.insert_masked(t, 10, np.tile(np.eye(3), (K, 1, 1)), np.ones((K, 3)), np.zeros((K, 3, 3)),
                                            np.arange(1.0, 5.0), 2.0, do, scan_seq=3)
    assert (n, dropped, nxt) == (3, 1, 13)
    assert ids.tolist() == [10, -1, 11, 12]
    # eviction targets: the empty slots in index order (mass -inf, stable): 0, 2, 3, 5; proposal 1 is
    # masked, so slot 2 stays empty
    assert t["valid_mask"].tolist() == [True, True, False, True, True, True, False, False]
    assert t["primitive_ids"][[0, 3, 5]].tolist() == [10, 11, 12] and t["weights"][0] == 1.0
    assert t["last_supported_scan_seq"][0] == 3 and t["timestamps"][0] == 2.0


def test_fuse_cull_forget_recency_closed_forms():
    t = pm.create_empty_tile(4)
    t["valid_mask"][:3] = True
    t["weights"][:3] = [1.0, 5e-5, 2.0]
    t["Lambdas"][:] = np.eye(3)
    t["thetas"][:] = 1.0
    t["last_supported_scan_seq"][:] = [10, 4, 0, 0]
    n = pm.fuse(t, np.array([0, 0, 2]), np.tile(2.0 * np.eye(3), (3, 1, 1)), np.ones((3, 3)), np.ones((3, 3, 3)),
                np.array([1.0, 2.0, 3.0]), np.array([0.5, 0.25, 1.0]), 7.0, scan_seq=11,
                valid_mask=np.array([True, True, False]))
    assert n == 2
    assert np.allclose(t["Lambdas"][0], np.eye(3) * (1.0 + 2.0 * 0.75))
    assert t["weights"][0] == 1.0 + 0.5 + 0.5 and t["weights"][2] == 2.0    # masked row adds nothing
    assert t["last_supported_scan_seq"].tolist() == [11, 4, 0, 0] and t["timestamps"][2] == 7.0
    nc, dropped, ratio = pm.cull(t, 1e-4)
    assert (nc, dropped) == (1, 5e-5) and ratio == pytest.approx(5e-5 / (2.0 + 5e-5 + 2.0 + 1e-12))
    pm.forget(t, 0.5)
    assert t["weights"][0] == 1.0
    L0 = t["Lambdas"].copy()
    s, infl, down, nv = pm.recency_inflate({0: t}, [0, 99], 11, 0.5, 0.05)
    # slot 0 was supported at 11 (dt 0), slot 1 is culled (1), slot 2 at 0: exp(-5.5) clipped to 0.05
    dec = np.array([1.0, 1.0, 0.05, 1.0])
    assert nv == 2 and down == pytest.approx((1 - dec[0]) + (1 - dec[2]))
    assert np.allclose(t["Lambdas"], L0 * dec[:, None, None])


def test_view_top_weights_stable():
    t = pm.create_empty_tile(6)
    t["valid_mask"][[0, 2, 3, 5]] = True
    t["weights"][[0, 2, 3, 5]] = [0.5, 2.0, 0.5, 0.0]
    t["etas"][:, 0, 2] = 3.0
    v = pm.extract_atlas_map_view({7: t}, [7, 8], 4, 6)
    assert v["candidate_slots"].tolist() == [2, 0, 3, 5, 0, 1, 2, 3]   # ties stay in slot order; tile 8 empty
    assert v["candidate_tile_ids"].tolist() == [7] * 4 + [8] * 4
    assert v["valid_mask"].tolist() == [True] * 4 + [False] * 4
    assert np.allclose(v["kappas"][:4], 3.0) and np.allclose(v["directions"][0], [0, 0, 3.0 / (3.0 + 1e-12)])


def test_visual_pose_evidence_oracle_closed_form():
    """visual_pose_evidence.py:104-240 on exact correspondences: map = R p + t with one candidate per
    row -> L_t^{-1} h_t = t, the scatter's rotation is R itself (h_rot = 0), and both costs vanish."""
    from oracle import primitive_evidence as OE, se3
    rng = np.random.default_rng(0)
    N = 40
    z = np.array([0.5, -1.0, 0.2, 0.1, -0.05, 0.3])
    R, t = se3.so3_exp(z[3:]), z[:3]
    p = rng.normal(size=(N, 3))
    u = rng.normal(size=(N, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    Lam = np.tile(np.eye(3), (N, 1, 1))
    etas = np.zeros((N, 3, 3))
    etas[:, 0] = 5.0 * u
    batch = dict(Lambdas=Lam, thetas=p, etas=etas, valid_mask=np.ones(N, bool), n_valid=N)
    view = dict(positions=p @ R.T + t, directions=u @ R.T, kappas=np.full(N, 5.0), valid_mask=np.ones(N, bool))
    assoc = dict(responsibilities=np.full((N, 1), 1.0 / N), candidate_pool_indices=np.arange(N)[:, None],
                 row_masses=np.full(N, 1.0 / N))
    # the measurement mean is (I + eps) ^-1 p: evaluate at the linearisation of the exact pose
    r = OE.visual_pose_evidence(batch, view, assoc, z, eps_lift=0.0, eps_mass=0.0)
    assert np.allclose(np.linalg.solve(r["L_trans"], r["h_trans"]), t, atol=1e-12)
    assert np.allclose(r["h_rot"], 0.0, atol=1e-12) and r["total_weighted_cost"] == pytest.approx(0.0, abs=1e-12)
    assert r["support_frac"] == 1.0 and r["n_associations"] == N
