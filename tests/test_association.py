"""CPU tests of the association oracle (oracle/association.py): the reference's own budget test
(test_budget_assertions.py:91-118) restated, closed forms, the sort semantics, and the C-ABI's
argument checks that need no GPU."""

import numpy as np
import pytest

from assoc_util import budget_scene, make_scene
from oracle import association as OA


def test_budget_assertions_association():
    """test_budget_assertions.py:91-118 (compute cert budgets), plus what the scene pins in closed
    form: no stencil tile has id 0, so every pool entry costs 1e12 and the stable sort keeps pool
    order (candidates 0..K-1); the selected candidates' unmasked cost is 0 (same point, same vMF)."""
    batch, view = budget_scene()
    K = OA.GC_K_ASSOC
    res, cert = OA.associate_primitives_ot(batch, view, OA.AssociationConfig(k_assoc=K, k_sinkhorn=OA.GC_K_SINKHORN))
    n_total = batch["Lambdas"].shape[0]
    assert cert["largest_tensor_shape"][0] <= n_total
    assert cert["largest_tensor_shape"][1] <= K
    assert cert["segment_sum_k"] == K
    assert cert["alloc_bytes_est"] <= int(n_total * K * 8 * 4)
    np.testing.assert_array_equal(res["candidate_pool_indices"], np.tile(np.arange(K, dtype=np.int32), (n_total, 1)))
    # identical primitives (same point, same vMF): the cost and its row minimum are 0
    assert np.all(res["cost_matrix"] == 0.0)
    # symmetric unbalanced fixed point: u = v, u^7 = a^(ua) ... with a = b = 1/8, ua = vb = 1/6:
    # u = v = 64^(-1/7), pi = 64^(-2/7) (50 iterations contract by 1/36 each)
    np.testing.assert_allclose(res["responsibilities"], 64.0 ** (-2.0 / 7.0), rtol=1e-12)
    np.testing.assert_allclose(cert["transport_mass_total"], 64 * 64.0 ** (-2.0 / 7.0), rtol=1e-12)


def test_A_vmf_closed_forms():
    k = np.array([1e-14, 1e-3, 5e-3, 0.5, 3.0, 19.0, 25.0, 300.0])
    A = OA.A_vmf(k)
    ref = np.log(4 * np.pi) + np.log(np.sinh(np.maximum(k, 1e-12))) - np.log(np.maximum(k, 1e-12))
    big = k > 20
    np.testing.assert_allclose(A[~big], ref[~big], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(A[big], np.log(4 * np.pi) + k[big] - np.log(2.0) - np.log(k[big]), rtol=1e-14)
    # the branches meet continuously (sinh -> exp / 2 above 20; k + k^3/6 below 1e-2)
    for x in (20.0, 1e-2):
        lo, hi = OA.A_vmf(np.array([x * (1 - 1e-9)])), OA.A_vmf(np.array([x * (1 + 1e-9)]))
        assert abs(lo[0] - hi[0]) < 1e-7


def test_identical_primitive_costs_zero_and_direction_term():
    p = np.zeros((1, 3))
    d = np.array([[0.0, 0.0, 1.0]])
    k = np.array([7.0])
    c = OA.sparse_cost(p, d, k, p, d, k, np.zeros((1, 1), np.int64), beta=0.5)
    assert abs(c[0, 0]) < 1e-14
    # opposite directions: bc = exp(A(0) - A(k)) -> d_dir close to 1
    c2 = OA.sparse_cost(p, d, k, p, -d, k, np.zeros((1, 1), np.int64), beta=0.5)
    assert 0.49 < c2[0, 0] <= 0.5
    # a zero kappa on either side switches the direction term off (valid_dir, :195-196)
    c3 = OA.sparse_cost(p, d, np.zeros(1), p, -d, k, np.zeros((1, 1), np.int64), beta=0.5)
    assert c3[0, 0] == 0.0


def test_balanced_sinkhorn_marginals():
    """tau -> 0: ua = vb = 1, the classic Sinkhorn; with sum a = sum b the column marginal is exact
    after each v update and the row marginal converges."""
    rng = np.random.default_rng(3)
    C = rng.uniform(0, 1, (40, 8))
    a = np.full(40, 1 / 40)
    b = np.full(8, 1 / 8)
    pi = OA.sinkhorn_unbalanced(C, a, b, 0.1, 0.0, 0.0, 500)
    np.testing.assert_allclose(pi.sum(axis=0), b, rtol=1e-9)
    np.testing.assert_allclose(pi.sum(axis=1), a, rtol=1e-6)


def test_stable_ties_take_pool_order():
    """A duplicated tile gives every primitive an equal-cost twin later in the pool: lax.sort with
    num_keys=1 is stable, so the earlier pool position comes first."""
    batch, view, _ = make_scene(seed=5, n_feat=16, n_surfel=16, n_valid_cam=10, n_valid_lidar=10, m_tile=32,
                                m_tile_view=32, tile_span=1, fill=(4, 32), dup_tile=True, missing_tiles=0)
    cfg = OA.AssociationConfig(r_stencil_tiles_xy=1)
    res, _ = OA.associate_primitives_ot(batch, view, cfg)
    cand = res["candidate_pool_indices"]
    assert np.all(np.diff(np.where(batch["valid_mask"][:, None], res["cost_matrix"], 0), axis=1) >= -1e-12)
    assert cand.shape == (32, 8)


def test_empty_cases_exact():
    batch, view, _ = make_scene(seed=1, n_feat=8, n_surfel=8, n_valid_cam=0, n_valid_lidar=0, m_tile=16,
                                m_tile_view=16, tile_span=1)
    res, cert = OA.associate_primitives_ot(batch, view)
    assert cert["exact"] and np.all(res["responsibilities"] == 0)
    batch, view, _ = make_scene(seed=1, n_feat=8, n_surfel=8, n_valid_cam=4, n_valid_lidar=4, m_tile=16,
                                m_tile_view=16, tile_span=1, fill=(0, 0))
    res, cert = OA.associate_primitives_ot(batch, view)
    assert cert["exact"]


def test_unsupported_policy_raises_past_the_empty_case():
    batch, view, _ = make_scene(seed=2, n_feat=8, n_surfel=8, n_valid_cam=4, n_valid_lidar=4, m_tile=16,
                                m_tile_view=16, tile_span=1, fill=(4, 8))
    with pytest.raises(ValueError):
        OA.associate_primitives_ot(batch, view, OA.AssociationConfig(b_policy="primitive_mass"))


def test_assoc_ctx_argument_checks(lib):
    import ctypes as C
    h = C.c_void_p()
    assert lib.gcs_assoc_ctx_create(0, 16, 8, 0, C.byref(h)) == -1       # no rows
    assert lib.gcs_assoc_ctx_create(16, 16, 33, 0, C.byref(h)) == -1     # k_assoc > 32
    assert lib.gcs_assoc_ctx_create(4096, 16, 8, 0, C.byref(h)) == -1    # past the one-workgroup Sinkhorn


def test_short_log_exp_pow_accuracy(lib):
    """The Sinkhorn's short log / exp (fdlibm reductions + minimax polynomials, gcs_math.h): within
    1 ulp of numpy's over the scalings' range, and x^y within 12 ulps of numpy's pow there."""
    from gcslam import _lib as L
    rng = np.random.default_rng(0)
    x = np.concatenate([np.exp(rng.uniform(-40.0, 40.0, 100000)), rng.uniform(0.5, 2.0, 10000),
                        np.array([1.0, 0.5, 2.0, np.sqrt(0.5), 1e-300, 1e300])])
    lo, ex, pw = np.empty_like(x), np.empty_like(x), np.empty_like(x)
    y = 1.0 / 6.0
    assert lib.gcs_debug_short_log_exp(L.dptr(x), x.size, y, L.dptr(lo), L.dptr(ex), L.dptr(pw)) == 0
    ulp = lambda a, b: np.abs(a - b) / np.spacing(np.abs(b))  # noqa: E731
    assert ulp(lo, np.log(x)).max() <= 1.0
    xe = rng.uniform(-40.0, 40.0, 100000)
    lo2, ex2, pw2 = np.empty_like(xe), np.empty_like(xe), np.empty_like(xe)
    assert lib.gcs_debug_short_log_exp(L.dptr(xe), xe.size, y, L.dptr(lo2), L.dptr(ex2), L.dptr(pw2)) == 0
    assert ulp(ex2, np.exp(xe)).max() <= 1.0
    # the rounding of y log x (an ulp of |y log x|, up to 6.7 over exp(+-40)) carries into exp; at
    # 1e+-300 (|y log x| = 115, far outside the scalings' range) it is ~20 ulps
    assert ulp(pw[:-2], np.power(x[:-2], y)).max() <= 12.0
    np.testing.assert_allclose(pw[-2:], np.power(x[-2:], y), rtol=1e-14)
    z = np.zeros(1)
    o1, o2, o3 = np.empty(1), np.empty(1), np.empty(1)
    assert lib.gcs_debug_short_log_exp(L.dptr(z), 1, y, L.dptr(o1), L.dptr(o2), L.dptr(o3)) == 0
    assert o3[0] == 0.0


def test_table_log_exp_accuracy(lib):
    """The Sinkhorn loop's table-driven log / exp (gcs_math.h log_tab / exp_tab, tables from
    tools/gen_sh_tables.py): within 1 ulp of numpy's over the whole normal range / |x| < 700, exact at
    the table's own points (log 1 = 0, exp 0 = 1), NaN outside the domains."""
    from gcslam import _lib as L
    rng = np.random.default_rng(1)
    ulp = lambda a, b: np.abs(a - b) / np.spacing(np.abs(b))  # noqa: E731
    x = np.concatenate([np.exp(rng.uniform(-700.0, 700.0, 200000)), rng.uniform(0.5, 2.0, 100000),
                        1.0 + rng.uniform(-1e-3, 1e-3, 20000), 1.0 + np.arange(129) / 128.0,
                        np.nextafter(2.0, 0.0) * np.ones(1), np.array([2.2250738585072014e-308, 1.7976931348623157e308])])
    lo, ex = np.empty_like(x), np.empty_like(x)
    assert lib.gcs_debug_tab_log_exp(L.dptr(x), x.size, L.dptr(lo), L.dptr(ex)) == 0
    ref = np.log(x)
    # away from x = 1 within an ulp; near 1 (|log x| < 0.01: the log1p polynomial alone) within 2
    far = np.abs(ref) > 1e-2
    assert ulp(lo[far], ref[far]).max() <= 1.0
    assert ulp(lo[~far & (ref != 0)], ref[~far & (ref != 0)]).max() <= 2.0
    assert lo[np.flatnonzero(x == 1.0)[0]] == 0.0
    xe = np.concatenate([rng.uniform(-700.0, 700.0, 200000), rng.uniform(-1.0, 1.0, 100000),
                         np.arange(-64, 65) * np.log(2.0) / 64.0, np.array([0.0, -699.9, 699.9])])
    lo2, ex2 = np.empty_like(xe), np.empty_like(xe)
    assert lib.gcs_debug_tab_log_exp(L.dptr(xe), xe.size, L.dptr(lo2), L.dptr(ex2)) == 0
    assert ulp(ex2, np.exp(xe)).max() <= 1.0
    assert ex2[np.flatnonzero(xe == 0.0)[0]] == 1.0
    bad = np.array([0.0, -1.0, 5e-324, np.inf, np.nan, 700.0, -700.0])
    lo3, ex3 = np.empty_like(bad), np.empty_like(bad)
    assert lib.gcs_debug_tab_log_exp(L.dptr(bad), bad.size, L.dptr(lo3), L.dptr(ex3)) == 0
    assert np.isnan(lo3[[0, 1, 2, 3, 4]]).all() and np.isnan(ex3[[3, 4, 5, 6]]).all()
