"""The oracle against the committed golden fixtures (CPU).

The fixtures are oracle-generated (tests/golden/make_golden.py; the JAX reference cannot run here and
holds no golden vectors), so this suite freezes the restatement: any change to an
oracle function that moves a fixture output fails here first.  Integer outputs are compared exactly,
floating outputs at 1e-12 relative (same code, same inputs: only libm/BLAS rounding may differ)."""

import numpy as np
import pytest

from golden_util import ORIGIN, load, scan_dict
from oracle import ops, pipeline as opipe

RT = 1e-12


def _close(a, b, rtol=RT, atol=1e-15):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


def test_golden_point_stage():
    g = load("point_stage")
    pts = g["xyz_record"][:, :3].astype(np.float64)
    bud = ops.point_budget_resample(pts, g["timestamps"], g["weights"], n_points_cap=int(g["cap"]))
    assert np.array_equal(bud["indices"], g["budget_indices"])
    _close(bud["weights"], g["budget_weights"])
    dk = ops.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], float(g["t0"]), float(g["t1"]),
                                   g["xi"])
    _close(dk["points"], g["deskew_points"], atol=1e-13)
    _close(dk["weights"], g["deskew_weights"])


def _deskewed_dirs(g):
    pts = g["xyz_record"][:, :3].astype(np.float64)
    dk = ops.deskew_constant_twist(pts, g["timestamps"], g["weights"], float(g["t0"]), float(g["t1"]), g["xi"])
    return dk, ops.point_directions(dk["points"], ORIGIN)


def test_golden_soft_assign_scale():
    g = load("soft_assign_scale")
    B, K = int(g["n_bins"]), int(g["k"])
    bins = ops.fibonacci_atlas(B)
    _close(bins, g["bins"], atol=0)
    knn = ops.bin_knn_table(bins, K)
    assert np.array_equal(knn, g["knn"])                                  # bit-exact atlas table
    dk, d = _deskewed_dirs(g)
    assert np.array_equal(ops.nearest_bin(d, bins), g["nearest"])         # bit-exact nearest bins
    sa = ops.bin_soft_assign_scale(d, bins, knn, float(g["tau"]))
    assert np.array_equal(sa["indices"], g["cand_ids"])                   # bit-exact candidate ids
    _close(sa["responsibilities"], g["resp"])
    _close(sa["avg_entropy"], g["avg_entropy"])
    st = ops.scan_bin_moment_match_scale(dk["points"], dk["weights"], sa["indices"], sa["responsibilities"],
                                         ORIGIN, B)
    for k in ("N", "s_dir", "S_dir_scatter", "p_bar", "kappa_scan"):
        _close(st[k], g[f"st_{k}"], atol=1e-14)
    _close(st["Sigma_p"], g["st_Sigma_p"], rtol=1e-9, atol=1e-14)            # eigh rebuild rounding
    assert st["ess"] == pytest.approx(float(g["st_ess"]), rel=RT)


def test_golden_soft_assign_dense():
    g = load("soft_assign_dense")
    bins = ops.fibonacci_atlas(int(g["n_bins"]))
    dk, d = _deskewed_dirs(g)
    sa = ops.bin_soft_assign_dense(d, bins, float(g["tau"]))
    _close(sa["responsibilities"], g["resp"], atol=1e-300)
    st = ops.scan_bin_moment_match_dense(dk["points"], dk["weights"], sa["responsibilities"], ORIGIN)
    _close(st["N"], g["st_N"])
    _close(st["p_bar"], g["st_p_bar"], atol=1e-13)


@pytest.mark.parametrize("name", ["scan_dense_b48", "scan_scale_b1024"])
def test_golden_scan_steps(name):
    g = load(name)
    B, cap, mode = int(g["n_bins"]), int(g["cap"]), str(g["mode"])
    bins = ops.fibonacci_atlas(B)
    knn = ops.bin_knn_table(bins, 16) if mode == "scale" else None
    cfg = opipe.BinPathConfig(n_points_cap=cap, n_bins=B, mode=mode, lidar_origin=tuple(ORIGIN), tau=float(g["tau"]))
    b = ops.Belief.identity_prior()
    ms = opipe.MapState.empty(B)
    for s in range(g["out_z_t"].shape[0]):
        r = opipe.process_scan_bin_path(b, scan_dict(g, s), g["Q"], cfg, bins, knn, ms)
        _close(r["z_t"], g["out_z_t"][s], rtol=1e-10, atol=1e-13)
        _close(r["belief"].L, g["out_L"][s], rtol=1e-10, atol=1e-10 * np.abs(g["out_L"][s]).max())
        _close(r["scan_bins"]["N"], g["out_scan_N"][s], atol=1e-14)
        assert r["beta"] == pytest.approx(float(g["out_beta"][s]), rel=RT)
        _close(r["iw_meas_dPsi"], g["out_meas_dPsi"][s], rtol=1e-10, atol=1e-22)
        _close(r["iw_meas_dnu"], g["out_meas_dnu"][s])
        b, ms = r["belief"], r["map"]


def test_golden_combine():
    g = load("combine_h4")
    results = [dict(belief=ops.Belief(g["X_anchor"][k], 1.0, g["z_lin"][k], g["L"][k], g["h"][k]),
                    iw_process_dPsi=g["dPsi"][k], iw_process_dnu=np.ones(7), iw_meas_dPsi=g["meas_dPsi"][k],
                    iw_meas_dnu=g["meas_dnu"][k]) for k in range(4)]
    r = opipe.combine_and_update_noise(results, g["weights"], (g["nu0"], g["Psi0"]), 3,
                                       (g["meas_nu0"], g["meas_Psi0"]))
    _close(r["meas_state"][0], g["out_meas_nu"])
    _close(r["meas_state"][1], g["out_meas_Psi"], atol=1e-20)
    _close(r["combined"]["L"], g["out_L"], atol=1e-12)
    _close(r["combined"]["h"], g["out_h"])
    _close(r["iw_state"][1], g["out_Psi"], atol=1e-15)
    _close(r["Q"], g["out_Q"], atol=1e-18)
