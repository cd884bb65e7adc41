"""LiDAR surfel extraction on the GPU (gcs_extract_lidar_surfels) against the numpy oracle
(oracle/surfels.py, lidar_surfel_extraction.py:84-431, ma_hex_web.py:221-303).

Bars: cell buckets, clipped counts and the selected cell ids bit-exact (the oracle hashes around the
device's centre, so the bucketing is checked apart from the order of the centre's sum; the centre
itself at 1e-12); surfel values at rtol 1e-9 (positions, weights, timestamps) and 1e-7 relative to
the matrix norm (covariances, information form); normals and kappas where the cell's smallest
eigenvalue is separated (gap > 1e-6 of the largest: elsewhere the plane normal is not determined).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import surfels as OS
from gcslam import synthetic
from gcslam.surfels import SurfelExtractionConfig, SurfelExtractor, extract_lidar_surfels

pytestmark = pytest.mark.gpu


def _cfg(o: OS.SurfelExtractionConfig) -> SurfelExtractionConfig:
    return SurfelExtractionConfig(**{k: getattr(o, k) for k in o.__dataclass_fields__})


def _compare(got, ref, cfg: OS.SurfelExtractionConfig):
    n = ref["n_valid"]
    assert got["n_valid"] == n
    assert np.array_equal(got["bucket"].cpu().numpy(), ref["bucket"])
    assert np.array_equal(got["count"].cpu().numpy(), ref["count"])
    ids = got["cell_ids"].cpu().numpy()
    assert np.array_equal(ids[:n], ref["cell_ids"]) and np.all(ids[n:] == -1)
    for k in ("positions", "weights", "timestamps"):
        np.testing.assert_allclose(got[k].cpu().numpy(), ref[k], rtol=1e-9, atol=1e-12, err_msg=k)
    cov = got["covariances"].cpu().numpy().reshape(-1, 3, 3)
    for i in range(cfg.n_surfel):
        sc = max(np.abs(ref["covariances"][i]).max(), 1e-300)
        np.testing.assert_allclose(cov[i], ref["covariances"][i], rtol=1e-7, atol=1e-7 * sc)
    # normals / kappas where the plane normal is determined
    nrm, kap = got["normals"].cpu().numpy(), got["kappas"].cpu().numpy()
    checked = 0
    for s, k in enumerate(ref["cell_ids"]):
        cnt = ref["count"][k]
        idx = ref["bucket"][k, :cnt]
        # eigen gap of the oracle's covariance (recomputed from the members)
        pc = np.asarray(_PTS[0])[idx] - ref["center"]
        w = np.asarray(_PTS[1])[idx]
        ws = w.sum() + 1e-12
        m = (pc * w[:, None]).sum(0) / ws
        d = pc - m
        cv = (d * w[:, None]).T @ d / ws + 1e-12 * np.eye(3)
        ev = np.linalg.eigvalsh(cv)
        if ev[1] - ev[0] > 1e-6 * ev[2]:
            np.testing.assert_allclose(nrm[s], ref["normals"][s], rtol=0, atol=1e-7)
            np.testing.assert_allclose(kap[s], ref["kappas"][s], rtol=1e-6)
            checked += 1
    return checked


_PTS = [None, None]


def _run(points, t, w, ocfg, device_center=True):
    _PTS[0], _PTS[1] = points, w
    ex = SurfelExtractor(_cfg(ocfg), max_points=max(len(points), 16))
    try:
        got = ex.extract(points, t, w, want_intermediates=True)
    finally:
        ex.close()
    mask, w_eff, c_np = OS.point_mask_and_center(points, w, ocfg.eig_min)
    # sums of +-metres cancel in a near-zero component: absolute bar 1e-13 of the coordinate scale
    np.testing.assert_allclose(got["center"], c_np, rtol=1e-12, atol=1e-13 * max(np.abs(points[mask]).max(), 1.0))
    ref = OS.extract_surfels_mahex3d(points, t, w, ocfg, center=got["center"] if device_center else None)
    return got, ref


def test_reference_smoke_two_clusters_on_gpu():
    """test_lidar_surfel_extraction_mahex3d.py:16-61 through the drop-in operator."""
    rng = np.random.default_rng(0)
    pts = np.vstack([rng.normal([0.0, 0.0, 0.0], 0.01, (20, 3)), rng.normal([1.0, 1.0, 0.0], 0.01, (20, 3))])
    t, w = np.linspace(0.0, 1.0, 40), np.ones(40)
    ocfg = OS.SurfelExtractionConfig(n_surfel=8, n_feat=4, voxel_size_m=0.5, min_points_per_voxel=5,
                                     hex3d_num_cells_1=8, hex3d_num_cells_2=8, hex3d_num_cells_z=2,
                                     hex3d_max_occupants=32)
    got, ref = _run(pts, t, w, ocfg)
    _compare(got, ref, ocfg)
    batch, cert, eff = extract_lidar_surfels(torch.from_numpy(pts).cuda(), torch.from_numpy(t).cuda(),
                                             torch.from_numpy(w).cuda(), config=_cfg(ocfg))
    assert batch.n_surfel == 8 and batch.n_feat == 4
    assert 0 <= batch.n_lidar_valid <= batch.n_surfel
    assert int(batch.valid_mask[batch.lidar_slice].sum()) == batch.n_lidar_valid
    n = batch.n_lidar_valid
    assert bool(torch.all(torch.isfinite(batch.Lambdas[batch.lidar_slice][:n])))
    assert cert.exact is False and cert.approximation_triggers
    rb = OS.lidar_measurement_batch(ref, ocfg)
    for k in ("Lambdas", "thetas", "etas", "colors"):
        g, r = getattr(batch, k).cpu().numpy(), rb[k]
        np.testing.assert_allclose(g, r, rtol=1e-7, atol=1e-7 * max(np.abs(r).max(), 1.0), err_msg=k)
    for k in ("weights", "timestamps"):
        np.testing.assert_allclose(getattr(batch, k).cpu().numpy(), rb[k], rtol=1e-9, atol=1e-12)
    for k in ("sources", "source_indices", "valid_mask"):
        assert np.array_equal(getattr(batch, k).cpu().numpy(), rb[k]), k
    assert eff.predicted == n and cert.support.support_frac == pytest.approx(n / 8)


@pytest.mark.parametrize("n_points,scan", [(8192, 0), (65536, 3)])
def test_synthetic_scan_matches_oracle(n_points, scan):
    """A VLP-16-like scan of the box room (planar walls, 1 cm range noise) at the reference's
    default configuration (voxel 0.1 m, 32 x 32 x 8 grid, 32 occupants, n_surfel 1024)."""
    sc = synthetic.make_scan(n_points, scan)
    pts = np.ascontiguousarray(sc["points"], np.float64)
    ocfg = OS.SurfelExtractionConfig()
    got, ref = _run(pts, sc["timestamps"], sc["weights"], ocfg)
    assert ref["n_valid"] > 100
    checked = _compare(got, ref, ocfg)
    assert checked > 0.5 * ref["n_valid"]


def test_sentinels_empty_input_and_capacity():
    rng = np.random.default_rng(3)
    pts = rng.normal(0, 0.3, (300, 3))
    pts[::7] = 1e6                              # parse sentinels are masked out of every cell
    t, w = np.linspace(0, 0.1, 300), rng.uniform(0.5, 1.0, 300)
    ocfg = OS.SurfelExtractionConfig(n_surfel=64, hex3d_num_cells_1=8, hex3d_num_cells_2=8, hex3d_num_cells_z=4,
                                     voxel_size_m=0.25)
    got, ref = _run(pts, t, w, ocfg)
    _compare(got, ref, ocfg)
    assert not np.isin(np.arange(0, 300, 7), got["bucket"].cpu().numpy()).any()
    ex = SurfelExtractor(_cfg(ocfg), max_points=300)
    try:
        e = ex.extract(np.zeros((0, 3)), np.zeros(0), np.zeros(0), want_intermediates=True)
        assert e["n_valid"] == 0 and int(e["count"].sum()) == 0
        assert torch.all(e["covariances"].reshape(-1, 9)[:, [0, 4, 8]] == 1.0)
        with pytest.raises(ValueError):
            ex.extract(np.zeros((301, 3)), np.zeros(301), np.zeros(301))
        a = {k: v.clone() for k, v in ex.extract(pts, t, w).items() if torch.is_tensor(v)}
        b = ex.extract(pts, t, w)
        for k in ("positions", "covariances", "normals", "Lambdas"):
            assert torch.equal(a[k], b[k])      # bitwise reproducible
    finally:
        ex.close()


@pytest.mark.parametrize("n_points,scan,cells", [(8192, 0, (32, 32, 8)), (8192, 5, (32, 32, 8)), (5000, 2, (16, 16, 8)),
                                                 (300, 1, (64, 64, 16)), (16384, 0, (32, 32, 8)),
                                                 (12000, 4, (64, 64, 16))])
def test_lds_key_sort_equals_radix_sort(monkeypatch, n_points, scan, cells):
    """k_sf_sort_lds (one workgroup: the stable (key, index) sort in LDS and the run bounds; clouds of up to
    8,192 points with 13-bit indices, up to 16,384 -- twice the reference's N_POINTS_CAP -- with 14-bit
    indices in 128 KB of LDS) against the rocPRIM radix-sort path (GCSLAM_SF_LDS_SORT=0): every output and
    intermediate bitwise equal, parse sentinels included."""
    cap = max(8192, n_points)
    sc = synthetic.make_scan(cap, scan)
    pts = np.ascontiguousarray(sc["points"][:n_points], np.float64).copy()
    pts[::97] = 1e6                      # masked points: the key past the last cell, sorted last
    t, w = sc["timestamps"][:n_points], sc["weights"][:n_points]
    cfg = SurfelExtractionConfig(hex3d_num_cells_1=cells[0], hex3d_num_cells_2=cells[1], hex3d_num_cells_z=cells[2])
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("GCSLAM_SF_LDS_SORT", flag)
        ex = SurfelExtractor(cfg, max_points=cap)
        try:
            r = ex.extract(pts, t, w, want_intermediates=True)
            outs.append({k: (v.cpu().numpy().copy() if torch.is_tensor(v) else np.asarray(v)) for k, v in r.items()})
        finally:
            ex.close()
    a, b = outs
    assert a["n_valid"] == b["n_valid"] and a["n_valid"] > 0
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k


@pytest.mark.parametrize("n_points,scan,cells", [(8192, 3, (32, 32, 8)), (300, 1, (64, 64, 16))])
def test_folded_bucket_fill_equals_cells_kernel(monkeypatch, n_points, scan, cells):
    """The bucket rows and counts written by k_sf_moments' waves (default) against the separate k_sf_cells
    launch (GCSLAM_SF_FOLD_CELLS=0): every output and intermediate bitwise equal."""
    sc = synthetic.make_scan(8192, scan)
    pts = np.ascontiguousarray(sc["points"][:n_points], np.float64).copy()
    pts[::89] = 1e6
    t, w = sc["timestamps"][:n_points], sc["weights"][:n_points]
    cfg = SurfelExtractionConfig(hex3d_num_cells_1=cells[0], hex3d_num_cells_2=cells[1], hex3d_num_cells_z=cells[2])
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("GCSLAM_SF_FOLD_CELLS", flag)
        ex = SurfelExtractor(cfg, max_points=8192)
        try:
            r = ex.extract(pts, t, w, want_intermediates=True)
            outs.append({k: (v.cpu().numpy().copy() if torch.is_tensor(v) else np.asarray(v)) for k, v in r.items()})
        finally:
            ex.close()
    a, b = outs
    assert a["n_valid"] == b["n_valid"] and a["n_valid"] > 0
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k
