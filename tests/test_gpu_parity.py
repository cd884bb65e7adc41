"""GPU parity tests: the HIP path (through the C-ABI) against the numpy oracle on the same seeded
inputs.  Integer outputs (stride indices, nearest bins, candidate ids) are compared bit-exactly;
floating outputs within the tolerances written next to each assertion (DESIGN.md "Parity")."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from gpu_util import (assert_close, derived_fields, device_scan, map_fields, map_from_fields, scan_fields,
                      scan_from_fields)
from oracle import ops, pipeline as opipe, se3
from gcslam.synthetic import scan_kwargs

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)
XI = np.array([0.1, 0.002, 0.0, 0.0, 0.001, 0.03])   # deskew twist over the scan


def _synthetic():
    from gcslam import synthetic
    return synthetic


def _ctx(**kw):
    from gcslam.context import HypothesisContext
    base = dict(lidar_origin=ORIGIN, max_raw_points=1 << 20)
    base.update(kw)
    return HypothesisContext(**base)


@pytest.fixture(scope="module")
def dense_ctx():
    c = _ctx(n_bins=48, n_points_cap=4096, mode="dense")
    yield c
    c.close()


@pytest.fixture(scope="module")
def scale_ctx():
    c = _ctx(n_bins=20000, n_points_cap=8192, mode="scale", k_cand=16)
    yield c
    c.close()


# ------------------------------------------------------------------ rows 1 + 3: budget + deskew
@pytest.mark.parametrize("n_raw", [0, 1000, 4096, 8192, 12345])
def test_point_stage_budget_deskew(dense_ctx, n_raw):
    syn = _synthetic()
    sc = syn.make_scan(16 * ((max(n_raw, 16) + 15) // 16), 0)
    n = n_raw
    rec, t, w = device_scan(sc)
    t0, t1 = sc["scan_start_time"], sc["scan_end_time"]
    out = dense_ctx.point_stage(rec, 16, t, w, n, t0, t1, XI)
    cap = dense_ctx.cap
    bud = ops.point_budget_resample(sc["points"][:n], sc["timestamps"][:n], sc["weights"][:n], n_points_cap=cap)
    # stride/selection is integer arithmetic: budget weights vanish exactly on padded rows
    wb = out["budget_weights"].cpu().numpy()
    assert np.array_equal(wb == 0.0, bud["weights"] == 0.0)
    assert_close("budget weights", wb, bud["weights"], rtol=1e-13, atol=0)          # f64 mass rescale
    dk = ops.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], t0, t1, XI)
    assert_close("deskewed points", out["points"].cpu().numpy(), dk["points"], rtol=1e-12, atol=1e-12)
    assert_close("deskewed weights", out["weights"].cpu().numpy(), dk["weights"], rtol=1e-12, atol=1e-300)
    c = out["cert"]
    assert c[0] == pytest.approx(bud["total_mass_in"], rel=1e-12, abs=1e-300)
    assert c[2] == pytest.approx(bud["total_mass_in"] / (sc["weights"][:n][bud["indices"]].sum() + 1e-12)
                                 if n else 0.0, rel=1e-12, abs=1e-300)


# ------------------------------------------------------------------ row 5: nearest bin + candidates (bit-exact)
def test_scale_atlas_tables_bit_exact(scale_ctx):
    dirs, knn = scale_ctx.atlas()
    assert np.allclose(dirs, ops.fibonacci_atlas(scale_ctx.n_bins), atol=2e-15, rtol=0)
    assert np.array_equal(knn, ops.bin_knn_table(dirs, 16))


def test_scale_soft_assign_ids_bit_exact(scale_ctx):
    syn = _synthetic()
    sc = syn.make_scan(8192, 1)
    rec, t, w = device_scan(sc)
    out = scale_ctx.point_stage(rec, 16, t, w, 8192, sc["scan_start_time"], sc["scan_end_time"], XI)
    p0 = out["points"].cpu().numpy()
    dirs, knn = scale_ctx.atlas()
    d = ops.point_directions(p0, np.array(ORIGIN))
    nearest = ops.nearest_bin(d, dirs)
    assert np.array_equal(out["nearest"].cpu().numpy(), nearest)          # bit-exact nearest bins
    ids, r = scale_ctx.bin_soft_assign()
    sa = ops.bin_soft_assign_scale(d, dirs, knn, scale_ctx.cfg.tau, nearest=nearest)
    assert np.array_equal(ids.cpu().numpy(), sa["indices"])              # bit-exact candidate ids
    assert_close("responsibilities", r.cpu().numpy(), sa["responsibilities"], rtol=1e-9, atol=1e-15)
    assert np.allclose(r.sum(1).cpu().numpy(), 1.0, atol=1e-12)
    c = out["cert"]
    assert c[6] / (8192 + 1e-12) == pytest.approx(sa["avg_entropy"], rel=1e-10)
    assert c[7] == pytest.approx(sa["max_resp"], rel=1e-12)


def test_dense_soft_assign(dense_ctx):
    syn = _synthetic()
    sc = syn.make_scan(6000 // 16 * 16, 2)
    rec, t, w = device_scan(sc)
    n = rec.shape[0]
    out = dense_ctx.point_stage(rec, 16, t, w, n, sc["scan_start_time"], sc["scan_end_time"], XI)
    p0 = out["points"].cpu().numpy()
    dirs, _ = dense_ctx.atlas()
    d = ops.point_directions(p0, np.array(ORIGIN))
    _, r = dense_ctx.bin_soft_assign()
    sa = ops.bin_soft_assign_dense(d, dirs, 0.1)
    assert_close("dense responsibilities", r.cpu().numpy(), sa["responsibilities"], rtol=1e-9, atol=1e-15)
    assert out["cert"][6] / (4096 + 1e-12) == pytest.approx(sa["avg_entropy"], rel=1e-10)


# ------------------------------------------------------------------ row 6: moment match + kappa
def _mm_reference(ctx, p0, wout):
    dirs, knn = ctx.atlas()
    d = ops.point_directions(p0, np.array(ORIGIN))
    if ctx.mode == "scale":
        sa = ops.bin_soft_assign_scale(d, dirs, knn, ctx.cfg.tau)
        return ops.scan_bin_moment_match_scale(p0, wout, sa["indices"], sa["responsibilities"], np.array(ORIGIN),
                                               ctx.n_bins)
    sa = ops.bin_soft_assign_dense(d, dirs, ctx.cfg.tau)
    return ops.scan_bin_moment_match_dense(p0, wout, sa["responsibilities"], np.array(ORIGIN))


def _check_scan_stats(got, st, amp=1.0):
    """amp scales the responsibility-driven bars: the soft-assign logits are (s - m) / tau, so a
    1-ulp difference in a direction cosine moves a responsibility by ~ulp / tau relative (tau =
    4.6e-6 at B = 1M, DESIGN.md declared tau rule); callers pass amp = max(1, 10 ulp / tau / 1e-11)."""
    ref = scan_fields(st)
    assert_close("N", got[0], ref[0], rtol=1e-11 * amp, atol=1e-14)
    assert_close("s_dir", got[1:4], ref[1:4], rtol=1e-10 * amp, atol=1e-13)
    assert_close("S_dir_scatter", got[4:13], ref[4:13], rtol=1e-10 * amp, atol=1e-13)
    assert_close("p_bar", got[13:16], ref[13:16], rtol=1e-9, atol=1e-10)
    assert_close("Sigma_p", got[16:25], ref[16:25], rtol=1e-7, atol=1e-10)       # m^2, PSD-projected
    assert_close("kappa", got[25], ref[25], rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("which", ["dense", "scale"])
def test_scan_bin_moment_match(dense_ctx, scale_ctx, which):
    ctx = dense_ctx if which == "dense" else scale_ctx
    syn = _synthetic()
    sc = syn.make_scan(8192, 3)
    rec, t, w = device_scan(sc)
    out = ctx.point_stage(rec, 16, t, w, 8192, sc["scan_start_time"], sc["scan_end_time"], XI)
    cert = ctx.scan_bin_moment_match()
    got = ctx.get_scan_stats()
    st = _mm_reference(ctx, out["points"].cpu().numpy(), out["weights"].cpu().numpy())
    _check_scan_stats(got, st)
    assert cert[3] == pytest.approx(st["psd_projection_delta"], rel=1e-3, abs=1e-9)
    assert cert[4] == pytest.approx(st["mass_epsilon_ratio"], rel=1e-12)
    ess = cert[0] ** 2 / (cert[1] + 1e-12)
    assert ess == pytest.approx(st["ess"], rel=1e-10)
    # mass conservation: sum_b N_b = sum_n w_n (responsibilities sum to one per point)
    assert got[0].sum() == pytest.approx(out["weights"].sum().item(), rel=1e-12)


# ------------------------------------------------------------------ rows 7, 8, 11: MF, planar, pushforward
def test_mf_planar_pushforward(scale_ctx):
    syn = _synthetic()
    ctx = scale_ctx
    B = ctx.n_bins
    # a map built by pushing an earlier scan (oracle restatement of row 11)
    sc0 = syn.make_scan(8192, 4)
    rec, t, w = device_scan(sc0)
    out0 = ctx.point_stage(rec, 16, t, w, 8192, sc0["scan_start_time"], sc0["scan_end_time"], XI)
    ctx.scan_bin_moment_match()
    st0 = scan_from_fields(ctx.get_scan_stats())
    for k in ("N",):
        st0[k] = st0[k]
    z0 = np.array([0.2, -0.1, 0.05, 0.01, -0.02, 0.3])
    Sig = np.diag([1e-3, 2e-3, 1e-4, 1e-5, 2e-5, 3e-5])
    Sig[0, 5] = Sig[5, 0] = 1e-6
    ctx.set_map(np.zeros((26, B)))
    ctx.pushforward(z0, Sig, 0.99)
    m_dev, d_dev = ctx.get_map()
    m_ref = ops.pose_cov_inflation_pushforward(ops.MapBinStats.empty(B), st0, z0, Sig, 0.99)
    assert_close("map stats after push", m_dev, map_fields(m_ref), rtol=1e-11, atol=1e-12)
    mu, kap, cen, Sc = ops.map_derived_stats(map_from_fields(m_dev))
    dref = derived_fields(mu, kap, cen, Sc)
    assert_close("map mu/kappa/centroid", d_dev[:7], dref[:7], rtol=1e-9, atol=1e-12)
    assert_close("map Sigma_c", d_dev[7:], dref[7:], rtol=1e-7, atol=1e-10)
    # next scan against that map
    sc1 = syn.make_scan(8192, 5)
    rec, t, w = device_scan(sc1)
    ctx.point_stage(rec, 16, t, w, 8192, sc1["scan_start_time"], sc1["scan_end_time"], XI)
    ctx.scan_bin_moment_match()
    st1 = scan_from_fields(ctx.get_scan_stats())
    m_dev_s = map_from_fields(m_dev)
    mf_dev = ctx.matrix_fisher_rotation()
    R_pred = se3.so3_exp(np.array([0.0, 0.0, 0.25]))
    mf = ops.matrix_fisher_rotation(R_pred, st1["s_dir"], st1["S_dir_scatter"], st1["N"], m_dev_s.S_dir,
                                    m_dev_s.S_dir_scatter, m_dev_s.N_dir)
    assert_close("MF H", mf_dev["H"], mf["H"], rtol=1e-10, atol=1e-10 * np.abs(mf["H"]).max())
    assert_close("MF R", mf_dev["R_mf"], mf["R_mf"], rtol=0, atol=1e-10)
    assert_close("MF s", mf_dev["svd_s"], mf["svd_s"], rtol=1e-10, atol=1e-12)
    assert mf_dev["N_eff"] == pytest.approx(mf["N_eff"], rel=1e-11)
    pt_dev = ctx.planar_translation(mf["R_mf"])
    pt = ops.planar_translation(np.zeros(3), mf["R_mf"], st1["p_bar"], st1["Sigma_p"], st1["N"], cen, Sc,
                                m_dev_s.N_pos, m_dev_s.S_dir_scatter, m_dev_s.N_dir)
    # ill-conditioned per-bin 3x3 inverses (eps-clamped covariances) -> looser relative tolerance
    assert_close("planar L", pt_dev["L_full"], pt["L_full"], rtol=1e-6, atol=1e-6 * np.abs(pt["L_full"]).max())
    assert_close("planar h", pt_dev["h_full"], pt["h_full"], rtol=1e-6, atol=1e-6 * np.abs(pt["h_full"]).max())
    assert pt_dev["N_eff"] == pytest.approx(pt["N_eff"], rel=1e-11)


# ------------------------------------------------------------------ the 14-step scan, several scans
@pytest.mark.parametrize("mode,B,cap,n_raw", [("dense", 48, 4096, 8192), ("scale", 20000, 8192, 8192)])
def test_full_pipeline_matches_oracle(mode, B, cap, n_raw):
    syn = _synthetic()
    ctx = _ctx(n_bins=B, n_points_cap=cap, mode=mode)
    dirs, knn = ctx.atlas()
    cfg = opipe.BinPathConfig(n_points_cap=cap, n_bins=B, mode=mode, lidar_origin=ORIGIN, tau=ctx.cfg.tau)
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(B)
    for k in range(3):
        sc = syn.make_scan(n_raw, k)
        ref = opipe.process_scan_bin_path(b, sc, Q, cfg, dirs, knn, ms)
        rec, t, w = device_scan(sc)
        out = ctx.scan(rec, 16, t, w, n_raw, **scan_kwargs(sc), Q=Q)
        X, stamp, z, Lm, h = ctx.get_belief()
        cert = np.array(out.cert[:])
        assert cert[30] == pytest.approx(ref["beta"], rel=1e-12)
        # T sums PSD-projection deltas; with no clamped eigenvalue a delta is reconstruction rounding
        # noise ~ 1e-16 ||M||_F (implementation-specific in the reference too), so the tolerance
        # scales with the norms of the projected matrices (planar L_full dominates).
        noise = 1e-13 * (np.linalg.norm(ref["planar"]["L_full"]) + np.linalg.norm(ref["belief_post"].L) + 1.0)
        assert cert[35] == pytest.approx(ref["total_trigger"], rel=1e-9, abs=noise)
        assert_close(f"scan{k} z_t", np.array(out.z_t[:]), ref["z_t"], rtol=1e-7, atol=1e-9)
        assert_close(f"scan{k} X_anchor", X, ref["belief"].X_anchor, rtol=1e-7, atol=1e-9)
        assert_close(f"scan{k} L", Lm, ref["belief"].L, rtol=1e-7, atol=1e-7 * np.abs(ref["belief"].L).max())
        # h = L z_lin is rounding noise when the anchor absorbed the increment (rho = 1); compare
        # the implied mean increment L^{-1} h (metres / radians) instead of h entrywise
        mu_dev = np.linalg.solve(Lm + 1e-9 * np.eye(22), h)
        mu_ref = np.linalg.solve(ref["belief"].L + 1e-9 * np.eye(22), ref["belief"].h)
        assert_close(f"scan{k} mean increment", mu_dev, mu_ref, rtol=1e-6, atol=1e-9)
        assert_close(f"scan{k} z_lin", z, ref["belief"].z_lin, rtol=1e-6, atol=1e-9)
        assert_close(f"scan{k} dPsi", np.array(out.iw_process_dPsi[:]).reshape(7, 6, 6), ref["iw_process_dPsi"],
                     rtol=1e-6, atol=1e-12)
        assert_close(f"scan{k} meas dPsi", np.array(out.iw_meas_dPsi[:]).reshape(3, 3, 3), ref["iw_meas_dPsi"],
                     rtol=1e-9, atol=1e-13 * np.abs(ref["iw_meas_dPsi"]).max())
        _check_scan_stats(ctx.get_scan_stats(), ref["scan_bins"])
        m_dev, _ = ctx.get_map()
        mref = map_fields(ref["map"].stats)
        assert_close(f"scan{k} map", m_dev, mref, rtol=1e-7, atol=1e-9 * max(np.abs(mref).max(), 1.0))
        b, ms = ref["belief"], ref["map"]
    ctx.close()


# ------------------------------------------------------------------ determinism, edge cases
def test_bitwise_determinism_scale():
    syn = _synthetic()
    outs = []
    for _ in range(2):
        ctx = _ctx(n_bins=20000, n_points_cap=8192, mode="scale")
        sc = syn.make_scan(8192, 7)
        rec, t, w = device_scan(sc)
        o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
        outs.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.cert[:])))
        ctx.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("tile,B", [(32, 20000), (64, 20000), (128, 20000), (256, 20000), (128, 60000),
                                    (256, 60000)])
def test_bin_tile_sizes_match_oracle(tile, B, monkeypatch):
    """k_bins_scale's tile shapes (32 bins x 8 lanes; 64 x 4 with phase D on wave 0; 128 x 2 and
    256 x 1 with phase D on every wave) forced through GCSLAM_BIN_TILE on the same scans, with the
    large record stage (B = 20,000: the scan is dense in the map) and the small one (B = 60,000):
    ScanBinStats and the scan's z_t against the oracle at the moment-match bars, and the manifest
    names the shape."""
    monkeypatch.setenv("GCSLAM_BIN_TILE", str(tile))
    syn = _synthetic()
    cap, n_raw = 8192, 8192
    ctx = _ctx(n_bins=B, n_points_cap=cap, mode="scale")
    assert f"{tile}-bin tiles" in ctx.describe()["backends"]["moment_match"]
    dirs, knn = ctx.atlas()
    cfg = opipe.BinPathConfig(n_points_cap=cap, n_bins=B, mode="scale", lidar_origin=ORIGIN, tau=ctx.cfg.tau)
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(B)
    for k in range(2):
        sc = syn.make_scan(n_raw, 20 + k)
        ref = opipe.process_scan_bin_path(b, sc, Q, cfg, dirs, knn, ms)
        rec, t, w = device_scan(sc)
        out = ctx.scan(rec, 16, t, w, n_raw, **scan_kwargs(sc), Q=Q)
        _check_scan_stats(ctx.get_scan_stats(), ref["scan_bins"])
        # B = 60,000 (0.14 points per bin): scan 0 meets an empty map, so the planar WLS is weighted by
        # eps-level per-bin terms and amplifies last-ulp differences of the bin sums (the lane split of
        # the gather changes their rounding) to ~5e-9 m: the B = 1024 golden's bar
        atol = 1e-9 if B == 20000 else 5e-8
        assert_close(f"tile {tile} scan{k} z_t", np.array(out.z_t[:]), ref["z_t"], rtol=1e-7, atol=atol)
        b, ms = ref["belief"], ref["map"]
    ctx.close()


@pytest.mark.parametrize("capacity", [32, 4])
def test_direct_buckets_match_sorted_bitwise(capacity):
    """gcs_scan's direct buckets (k_points' fixed member rows, ranked by point index while the bin
    kernel stages) against the sorted bucketing (k_scan, k_place, k_bucket_rank): the accumulation
    order is the same, so three consecutive scans agree bit for bit.  capacity 4: buckets overflow
    the rows, the first scan is redone sorted (cert[57] = 1) and later scans stay sorted."""
    from gcslam import _lib as L
    syn = _synthetic()
    outs = []
    for sorted_path in (False, True):
        # capacity 4: 2,000 bins, so the occupied buckets hold several points each and overflow
        ctx = _ctx(n_bins=20000 if capacity == 32 else 2000, n_points_cap=8192, mode="scale")
        if sorted_path:
            ctx.set_debug(L.DEBUG_SORTED_BUCKETS, 1)
        elif capacity != 32:
            ctx.set_debug(L.DEBUG_BUCKET_CAPACITY, capacity)
        res = []
        for k in range(3):
            sc = syn.make_scan(8192, 11 + k)
            rec, t, w = device_scan(sc)
            o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            res.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.cert[:])))
        outs.append(res)
        ctx.close()
    for k in range(3):
        for a, b in zip(outs[0][k][:3], outs[1][k][:3]):
            assert np.array_equal(a, b)
        ca, cb = outs[0][k][3], outs[1][k][3]
        assert ca[57] == (1.0 if (capacity == 4 and k == 0) else 0.0) and cb[57] == 0.0
        ca[57] = cb[57] = 0.0
        assert np.array_equal(ca, cb)


@pytest.mark.parametrize("B,cap,n_raw,k", [(20000, 8192, 8192, 16), (20000, 8192, 12345, 8), (60000, 65536, 65536, 16),
                                            (2000, 4096, 4096, 16), (20000, 3000, 9000, 16)])
def test_lean_point_kernel_matches_legacy_bitwise(B, cap, n_raw, k):
    """k_points_lean (one point per thread, 128 registers, XCD-ordered blocks, partial rows at the
    logical block) against the round-3 k_points (GCS_DEBUG_POINT_KERNEL): the same per-point
    arithmetic, so over three consecutive scans the ScanBinStats, the map, the posterior and the
    certificate vector agree bit for bit -- grids that are and are not multiples of 8 blocks, strided
    budgets, overflowing buckets (B = 2000) and K = 8."""
    from gcslam import _lib as L
    syn = _synthetic()
    outs = []
    for legacy in (False, True):
        ctx = _ctx(n_bins=B, n_points_cap=cap, mode="scale", k_cand=k)
        ctx.set_debug(L.DEBUG_POINT_KERNEL, int(legacy))
        res = []
        for s in range(3):
            sc = syn.make_scan(16 * ((n_raw + 15) // 16), 31 + s)
            rec, t, w = device_scan(sc)
            o = ctx.scan(rec, 16, t, w, n_raw, **scan_kwargs(sc))
            res.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.z_t[:]),
                        np.array(o.cert[:])))
        outs.append(res)
        ctx.close()
    for s in range(3):
        for a, b in zip(outs[0][s], outs[1][s]):
            assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("n", [4096, 12288])
def test_degenerate_same_direction_points(n):
    """All points on one ray (one giant bucket: ranked in-wave at 4096, compacted at 12288)
    and zero-weight points."""
    ctx = _ctx(n_bins=20000, n_points_cap=n, mode="scale")
    p = np.tile(np.array([[5.0, 1.0, 0.5]], np.float32), (n, 1))
    rec = np.zeros((n, 4), np.float32)
    rec[:, :3] = p
    t = np.linspace(100.0, 100.1, n)
    w = np.ones(n)
    w[::3] = 0.0
    sc = dict(xyz_record=rec, timestamps=t, weights=w)
    drec, dt, dw = device_scan(sc)
    out = ctx.point_stage(drec, 16, dt, dw, n, 100.0, 100.1, np.zeros(6))
    ctx.scan_bin_moment_match()
    got = ctx.get_scan_stats()
    st = _mm_reference(ctx, out["points"].cpu().numpy(), out["weights"].cpu().numpy())
    _check_scan_stats(got, st)
    ctx.close()


def test_empty_scan_and_zero_twist():
    ctx = _ctx(n_bins=48, n_points_cap=1024, mode="dense")
    syn = _synthetic()
    sc = syn.make_scan(64, 0)
    rec, t, w = device_scan(sc)
    o = ctx.scan(rec, 16, t, w, 0, **scan_kwargs(sc))
    assert np.all(np.isfinite(np.array(o.belief.L[:])))
    st = ctx.get_scan_stats()
    assert np.all(st[0] == 0.0)
    ctx.close()


# ------------------------------------------------------------------ full-size properties (C2 / C3)
@pytest.mark.parametrize("N,B", [(65536, 100000), (262144, 1048576)])
def test_full_size_properties(N, B):
    syn = _synthetic()
    ctx = _ctx(n_bins=B, n_points_cap=N, mode="scale")
    sc = syn.make_scan(N, 0)
    rec, t, w = device_scan(sc)
    out = ctx.point_stage(rec, 16, t, w, N, sc["scan_start_time"], sc["scan_end_time"], XI)
    cert = ctx.scan_bin_moment_match()
    st = ctx.get_scan_stats()
    wsum = out["weights"].sum().item()
    assert st[0].sum() == pytest.approx(wsum, rel=1e-11)               # mass conservation
    assert cert[0] == pytest.approx(wsum, rel=1e-11)
    assert np.all(st[0] >= 0.0) and np.all(np.isfinite(st))
    Sig = st[16:25].T.reshape(-1, 3, 3)
    active = st[0] > 1e-6
    ev = np.linalg.eigvalsh(0.5 * (Sig[active] + np.swapaxes(Sig[active], 1, 2)))
    assert ev.min() >= 1e-12 * (1 - 1e-6) - 1e-15                    # PSD with eps floor
    # nearest bins of a random sample are bit-exact vs the oracle's exact rule
    dirs, knn = ctx.atlas()
    idx = np.random.default_rng(0).choice(N, 4000, replace=False)
    d = ops.point_directions(out["points"].cpu().numpy()[idx], np.array(ORIGIN))
    assert np.array_equal(out["nearest"].cpu().numpy()[idx], ops.nearest_bin(d, dirs))
    # determinism at full size
    out2 = ctx.point_stage(rec, 16, t, w, N, sc["scan_start_time"], sc["scan_end_time"], XI, want_outputs=False)
    ctx.scan_bin_moment_match()
    assert np.array_equal(ctx.get_scan_stats(), st)
    ctx.close()


def test_launch_gate_matches_ungated_bitwise_and_times_out_loudly():
    """gcs_scan's pre-launched device front (k_points waits on the device for the prologue's deskew
    twist, GCS_DEBUG_LAUNCH_GATE = 1, the default) against the point stage launched after the prologue
    (0): the twist reaches the kernel through the gate bit for bit, so three consecutive scans agree
    exactly.  A gate that is never opened (-1) runs every point block into its timeout and the scan
    fails with an error instead of hanging; the context then scans normally again."""
    from gcslam import _lib as L
    syn = _synthetic()
    outs = []
    for gate in (1, 0):
        ctx = _ctx(n_bins=20000, n_points_cap=8192, mode="scale")
        ctx.set_debug(L.DEBUG_LAUNCH_GATE, gate)
        res = []
        for k in range(3):
            sc = syn.make_scan(8192, 31 + k)
            rec, t, w = device_scan(sc)
            o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            res.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.z_t[:]),
                        np.array(o.cert[:])))
        outs.append(res)
        if gate == 1:
            ctx.set_debug(L.DEBUG_LAUNCH_GATE, -1)
            sc = syn.make_scan(8192, 40)
            rec, t, w = device_scan(sc)
            with pytest.raises(RuntimeError, match="gate"):
                ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            ctx.set_debug(L.DEBUG_LAUNCH_GATE, 1)
            o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            assert np.all(np.isfinite(np.array(o.z_t[:])))
        ctx.close()
    for a, b in zip(outs[0], outs[1]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("capacity", [32, 4])
def test_pt_clear_handoff_matches_budget_clears_bitwise(capacity):
    """gcs_scan's k_pt zeroing the next scan's bucket counts and flag buffer (GCS_DEBUG_PT_CLEAR = 1,
    the default; k_budget then only sums the weights) against k_budget doing the clears (0): four
    consecutive scans agree bit for bit -- the flag buffers alternate, so every buffer is reused
    after a k_pt clear.  capacity 4: the first scan overflows the direct rows and is redone sorted
    (a second k_budget on the same buffers, after the first attempt's k_pt cleared the counts)."""
    from gcslam import _lib as L
    syn = _synthetic()
    outs = []
    for clear in (1, 0):
        ctx = _ctx(n_bins=20000 if capacity == 32 else 2000, n_points_cap=8192, mode="scale")
        ctx.set_debug(L.DEBUG_PT_CLEAR, clear)
        if capacity != 32:
            ctx.set_debug(L.DEBUG_BUCKET_CAPACITY, capacity)
        res = []
        for k in range(4):
            sc = syn.make_scan(8192, 61 + k)
            rec, t, w = device_scan(sc)
            o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            res.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.z_t[:]),
                        np.array(o.cert[:])))
        outs.append(res)
        ctx.close()
    for a, b in zip(outs[0], outs[1]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y, equal_nan=True)
