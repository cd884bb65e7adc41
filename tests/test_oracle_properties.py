"""The reference's own property tests, restated against the oracle (pins the oracle; the reference
holds no golden vectors for this path -- SURVEY.md section 4).  Sources are cited per test."""

import math

import numpy as np
import pytest

from oracle import ops, se3
from oracle.primitives import inv_mass, psd_project, spd_solve_lifted


def test_point_budget_preserves_mass_and_budget():
    # archive/legacy_tests/test_operators.py:29-73
    rng = np.random.default_rng(42)
    pts = rng.standard_normal((10000, 3))
    out = ops.point_budget_resample(pts, np.linspace(0, 1, 10000), np.ones(10000))
    assert out["points"].shape[0] <= 8192
    assert abs(out["total_mass_out"] - out["total_mass_in"]) < 1e-6
    assert abs(out["weights"].sum() - out["total_mass_in"]) < 1e-6
    small = ops.point_budget_resample(pts[:100], np.linspace(0, 1, 100), np.ones(100))
    assert small["n_output"] == 100 and small["stride"] == 1


def test_point_budget_indices_are_strided():
    # point_budget.py:70,160: stride = ceil(N/cap), indices = arange(0, N, stride)
    for n, cap in ((100, 8192), (8193, 8192), (30000, 8192), (65536, 65536), (7, 3)):
        out = ops.point_budget_resample(np.zeros((n, 3)), np.zeros(n), np.ones(n), n_points_cap=cap)
        st = max(1, math.ceil(n / cap))
        assert np.array_equal(out["indices"], np.arange(0, n, st))


def test_kappa_monotone_and_nonnegative():
    # archive/legacy_tests/test_operators.py:76-114; test_audit_invariants.py:101-117
    # (the blend is not globally monotone: it dips near R=0.75-0.85; the reference asserts only
    #  k(0.1) < k(0.5) < k(0.8) and k >= 0 at 0, 0.5, 0.9, 0.99)
    assert np.all(ops.kappa_from_resultant_batch(np.array([0.0, 0.5, 0.9, 0.99])) >= 0)
    k = ops.kappa_from_resultant_batch(np.array([0.1, 0.5, 0.8]))
    assert k[0] < k[1] < k[2]
    assert np.all(ops.kappa_from_resultant_batch(np.linspace(0.0, 0.999, 2000)) >= 0)


def test_kappa_batch_equals_scalar():
    # test_audit_invariants.py:412-426 (batch vs scalar kappa_from_resultant_v2)
    for R in (0.0, 0.3, 0.8, 0.95, 0.999999):
        Rc = min(max(R, 0.0), 1.0 - ops.EPS_R)
        R2 = Rc * Rc
        kl = Rc * (3.0 - R2) / (1.0 - R2 + ops.EPS_R)
        kh = -math.log(max(1.0 - R2, ops.EPS_R))
        s = 1.0 / (1.0 + math.exp(-(Rc - 0.8) / 0.03))
        assert ops.kappa_from_resultant_batch(np.array([R]))[0] == pytest.approx((1 - s) * kl + s * kh, rel=1e-12)


def test_soft_assign_rows_sum_to_one():
    # archive/legacy_tests/test_operators.py:117-166 (rows sum to 1 within 1e-6); audit :137-146
    rng = np.random.default_rng(1)
    d = ops.point_directions(rng.standard_normal((500, 3)), np.zeros(3))
    bins = ops.fibonacci_atlas(48)
    sa = ops.bin_soft_assign_dense(d, bins, 0.1)
    assert np.allclose(sa["responsibilities"].sum(1), 1.0, atol=1e-6)
    assert np.all(sa["responsibilities"] >= 0)
    bins2 = ops.fibonacci_atlas(5000)
    knn = ops.bin_knn_table(bins2)
    sc = ops.bin_soft_assign_scale(d, bins2, knn, ops.tau_for_bins(5000))
    assert np.allclose(sc["responsibilities"].sum(1), 1.0, atol=1e-12)


def test_softmax_extreme_logits_finite():
    # test_audit_invariants.py:137-146
    d = np.array([[1.0, 0.0, 0.0]])
    bins = ops.fibonacci_atlas(48)
    sa = ops.bin_soft_assign_dense(d, bins, 1e-6)
    assert np.all(np.isfinite(sa["responsibilities"]))
    assert sa["responsibilities"].sum() == pytest.approx(1.0, abs=1e-6)


def test_psd_projection_extreme_inputs():
    # test_audit_invariants.py:119-135; test_primitives.py:53-94
    M = np.diag([1e6, -1e6, 1e-20])
    P, c = psd_project(M, 1e-6)
    assert np.linalg.eigvalsh(P).min() >= 1e-6 - 1e-12
    assert c[0] > 0
    Z, cz = psd_project(np.zeros((3, 3)))
    assert np.allclose(Z, 1e-12 * np.eye(3), atol=0) and cz[0] == pytest.approx(math.sqrt(3) * 1e-12)


def test_lifted_solve_near_singular():
    # test_audit_invariants.py:148-169
    L = np.diag([1.0, 1e-15, 1.0])
    x, lift = spd_solve_lifted(L, np.ones(3))
    assert np.all(np.isfinite(x)) and lift > 0


def test_inv_mass_total():
    inv, r = inv_mass(np.array([0.0, 1.0, 1e12]))
    assert np.all(np.isfinite(inv)) and r[0] == pytest.approx(1.0, rel=1e-3)


@pytest.mark.parametrize("angle", [1e-9, 1e-3, 1.0, 3.0, math.pi - 1e-8])
def test_so3_exp_log_roundtrip(angle):
    # test_audit_invariants.py:221-263 (small/medium/large/near-pi)
    axis = np.array([0.3, -0.5, 0.8])
    axis /= np.linalg.norm(axis)
    R = se3.so3_exp(axis * angle)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
    R2 = se3.so3_exp(se3.so3_log(R))
    assert np.allclose(R2, R, atol=1e-8)


def test_se3_exp_log_roundtrip():
    # test_audit_invariants.py:277-313
    xi = np.array([0.3, -0.2, 0.1, 0.05, -0.4, 0.2])
    assert np.allclose(se3.se3_log(se3.se3_exp(xi)), xi, atol=1e-10)


def test_deskew_zero_twist_is_identity():
    # deskew with xi = 0 is the identity on points
    rng = np.random.default_rng(3)
    p = rng.standard_normal((100, 3)) * 10
    t = np.linspace(0.0, 0.1, 100)
    out = ops.deskew_constant_twist(p, t, np.ones(100), 0.0, 0.1, np.zeros(6))
    assert np.array_equal(out["points"], p)


def test_matrix_fisher_recovers_exact_rotation():
    # MF on a synthetic exact rotation recovers R with delta_theta = 0
    rng = np.random.default_rng(5)
    B = 200
    u = ops.point_directions(rng.standard_normal((B, 3)), np.zeros(3))
    R = se3.so3_exp(np.array([0.1, -0.2, 0.3]))
    N = rng.uniform(1, 5, B)
    mf = ops.matrix_fisher_rotation(R, 0.9 * N[:, None] * u, np.zeros((B, 3, 3)), N, 0.9 * N[:, None] * (u @ R.T),
                                    np.zeros((B, 3, 3)), N)
    assert np.allclose(mf["R_mf"], R, atol=1e-10)
    assert np.allclose(mf["delta_rot"], 0.0, atol=1e-9)


def test_planar_translation_identical_correspondences():
    # a planar WLS with identical correspondences gives t exactly
    rng = np.random.default_rng(6)
    B = 64
    p = rng.standard_normal((B, 3)) * 5
    t = np.array([1.0, -2.0, 0.5])
    R = se3.so3_exp(np.array([0.0, 0.0, 0.4]))
    S = np.tile(0.01 * np.eye(3), (B, 1, 1))
    N = np.full(B, 3.0)
    Ssc = np.tile(np.diag([0.4, 0.4, 0.2]), (B, 1, 1))
    pt = ops.planar_translation(t, R, p, S, N, p @ R.T + t, S, N, Ssc, N)
    assert np.allclose(pt["t_wls"], t, atol=1e-9)


def test_info_fusion_trace_increases():
    # archive/legacy_tests/test_operators.py:389-447
    b = ops.Belief.identity_prior()
    Lev = np.diag(np.arange(1, 23, dtype=float))
    out, _ = ops.info_fusion_additive(b, Lev, np.ones(22), 1.0)
    assert np.trace(out.L) > np.trace(b.L)


def test_hypothesis_weight_floor_and_order_invariance():
    # archive/legacy_tests/test_operators.py:450-511; test_audit_invariants.py:33-95
    rng = np.random.default_rng(7)
    Ls = np.stack([np.diag(rng.uniform(1, 2, 22)) for _ in range(4)])
    hs = rng.standard_normal((4, 22))
    zs = rng.standard_normal((4, 22))
    w = np.array([0.0, 0.3, 0.3, 0.4])
    a = ops.hypothesis_barycenter(Ls, hs, zs, w)
    assert a["weights"].min() > 0
    perm = [2, 0, 3, 1]
    b = ops.hypothesis_barycenter(Ls[perm], hs[perm], zs[perm], w[perm])
    assert np.allclose(a["L"], b["L"], atol=1e-12) and np.allclose(a["h"], b["h"], atol=1e-12)


def test_iw_apply_order_invariance():
    # test_audit_invariants.py:336-406 (commutative sufficient statistics)
    nu, Psi = ops.datasheet_process_noise_state()
    rng = np.random.default_rng(8)
    d = [ops.process_noise_iw_suffstats(np.eye(22) * 2, rng.standard_normal(22), np.eye(22) * 3,
                                        rng.standard_normal(22))[0] for _ in range(3)]
    s1 = d[0] + d[1] + d[2]
    s2 = d[2] + d[0] + d[1]
    a = ops.process_noise_iw_apply(nu, Psi, s1, np.full(7, 3.0))
    b = ops.process_noise_iw_apply(nu, Psi, s2, np.full(7, 3.0))
    assert np.allclose(a[1], b[1], atol=1e-12) and np.allclose(a[0], b[0], atol=1e-12)


def test_knn_shortlist_matches_brute_force():
    bins = ops.fibonacci_atlas(3000)
    assert np.array_equal(ops.bin_knn_table(bins), ops.bin_knn_table(bins, brute=True))
    rng = np.random.default_rng(9)
    q = ops.point_directions(rng.standard_normal((2000, 3)), np.zeros(3))
    assert np.array_equal(ops.nearest_bin(q, bins), ops.nearest_bin(q, bins, brute=True))
