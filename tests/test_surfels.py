"""LiDAR surfel extraction oracle (the live primitive path's first operator):
the reference's own smoke test restated (test_lidar_surfel_extraction_mahex3d.py:16-61) plus
closed-form cases for the MA-hex bucketing, the plane fit and the selection."""
import numpy as np
import pytest

from oracle import surfels as S


def _smoke_cfg():
    return S.SurfelExtractionConfig(n_surfel=8, n_feat=4, voxel_size_m=0.5, min_points_per_voxel=5,
                                    hex3d_num_cells_1=8, hex3d_num_cells_2=8, hex3d_num_cells_z=2,
                                    hex3d_max_occupants=32)


def _two_clusters():
    rng = np.random.default_rng(0)
    a = rng.normal(loc=[0.0, 0.0, 0.0], scale=0.01, size=(20, 3))
    b = rng.normal(loc=[1.0, 1.0, 0.0], scale=0.01, size=(20, 3))
    pts = np.vstack([a, b])
    return pts, np.linspace(0.0, 1.0, 40), np.ones(40)


def test_reference_smoke_two_clusters():
    """test_lidar_surfel_extraction_mahex3d.py:16-61 (same inputs and assertions, plus the count)."""
    pts, t, w = _two_clusters()
    cfg = _smoke_cfg()
    batch, cert, ext = S.extract_lidar_surfels(pts, t, w, cfg)
    assert batch["n_surfel"] == 8 and batch["n_feat"] == 4
    assert 0 <= batch["n_lidar_valid"] <= 8
    lid = slice(4, 12)
    assert int(batch["valid_mask"][lid].sum()) == batch["n_lidar_valid"]
    n = batch["n_lidar_valid"]
    assert np.all(np.isfinite(batch["Lambdas"][lid][:n])) and np.all(np.isfinite(batch["weights"][lid][:n]))
    assert cert["exact"] is False and cert["triggers"]
    # each tight cluster lands in cells with >= 5 points: at least one surfel per cluster
    assert n >= 2
    assert cert["support_frac"] == pytest.approx(n / 8)


def test_bucketing_first_occupants_by_index_and_clipped_counts():
    cfg = S.SurfelExtractionConfig(hex3d_num_cells_1=4, hex3d_num_cells_2=4, hex3d_num_cells_z=2,
                                   hex3d_max_occupants=3, voxel_size_m=1.0)
    # five points in one cell, one masked (sentinel), one in another cell
    p = np.array([[0.2, 0.1, 0.1], [0.3, 0.1, 0.2], [1e6, 0, 0], [0.4, 0.2, 0.3], [0.1, 0.1, 0.4],
                  [0.2, 0.2, 0.5], [2.5, 0.1, 0.1]])
    mask = np.all(np.abs(p) < 1e5, axis=1)
    b, cnt, lin = S.bin_points_3d(p, mask, cfg)
    c0 = lin[0]
    assert list(b[c0]) == [0, 1, 3]          # first three unmasked occupants in index order
    assert cnt[c0] == 3                      # five occupants, clipped to max_occupants
    assert b[lin[6]][0] == 6 and cnt[lin[6]] == 1
    assert cnt.sum() == 4
    # the hash wraps modulo the grid: a point one grid period away lands in the same cell
    q = np.array([[0.2, 0.1, 0.1], [0.2 + 8.0, 0.1, 0.1]])  # s1 += 8, s2 += 4: both whole periods
    _, _, lq = S.bin_points_3d(q, np.ones(2, bool), cfg)
    assert lq[0] == lq[1]


def test_plane_fit_closed_form():
    cfg = S.SurfelExtractionConfig()
    g = np.linspace(-0.02, 0.02, 5)
    X, Y = np.meshgrid(g, g)
    pts = np.stack([X.ravel() + 0.03, Y.ravel() + 0.02, np.full(25, 0.01)], axis=1)
    w = np.ones(25)
    t = np.arange(25) * 0.01
    idx = np.arange(25)
    cen, Sig, n, kap, ws, ts, valid, spq = S.fit_one_cell(pts, t, w, idx, 25, cfg)
    np.testing.assert_allclose(cen, [0.03, 0.02, 0.01], atol=1e-15)
    np.testing.assert_allclose(n, [0, 0, 1], atol=1e-12)
    assert valid and ws == 25.0
    assert ts == pytest.approx(np.sum(t) / (25 + 1e-12))
    assert kap == 100.0                       # sigma_perp ~ 0 -> kappa clipped at kappa_max
    var = np.mean(g * g) * 1.0                # in-plane variance of the grid along each axis
    # Sigma_reg = (Sigma^-1 + nu/psi I)^-1 along each principal axis (+ eig_min terms)
    lam = 1.0 / (var + 1e-6 + 2e-12) + 50.0
    assert Sig[0, 0] == pytest.approx(1.0 / (lam + 1e-12) + 1e-12, rel=1e-9)
    assert Sig[2, 2] == pytest.approx(1.0 / (1.0 / (1e-12 + 1e-6 + 2e-12) + 50.0 + 1e-12) + 1e-12, rel=1e-6)


def test_selection_valid_first_by_cell_id_and_padded_tail():
    pts, t, w = _two_clusters()
    cfg = _smoke_cfg()
    ext = S.extract_surfels_mahex3d(pts, t, w, cfg)
    n = ext["n_valid"]
    ids = ext["cell_ids"]
    assert np.all(np.diff(ids) > 0) and np.all(ext["cell_valid"][ids])
    assert np.all(ext["positions"][n:] == 0) and np.all(ext["covariances"][n:] == np.eye(3))
    assert n == min(int(ext["cell_valid"].sum()), cfg.n_surfel)
    # weights: the clusters' unit weights, split over their cells
    assert ext["weights"][:n].sum() <= 40.0 + 1e-9
