"""Value parity at the north-star sizes (BASELINE.json configs[1] and configs[2]), not only
properties: the HIP path through the C-ABI against the numpy oracle on the same seeded inputs.

* C2 (65,536 points x 100,000 bins, K=16, scale mode): the whole kNN candidate table bit-exact,
  then three consecutive 14-step scans from the identity prior and an empty map
  (FS/backend/pipeline.py:316-1591 bin path; binning.py:139-209) with odometry, each checked for
  z_t / X_anchor / L / IMU-odometry evidence / ScanBinStats / map at the small-case bars; plus
  the nearest bins and candidate ids of every point of a C2 point stage bit-exact.
* C3 (1,048,576 bins, 262,144-point capacity): the whole candidate table bit-exact, and a 1/8
  point subsample (32,768 points) through the point stage + ScanBinMomentMatch (ids bit-exact,
  ScanBinStats over all 1M bins at the moment-match bars).
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from gpu_util import MAP_GROUPS, assert_close, assert_close_groupwise, device_scan, map_fields
from oracle import ops, pipeline as opipe
from gcslam.synthetic import scan_kwargs
from test_gpu_parity import ORIGIN, XI, _check_scan_stats, _ctx, _mm_reference, _synthetic

pytestmark = pytest.mark.gpu


def test_c2_three_scans_value_parity():
    syn = _synthetic()
    N, B = 65536, 100000
    ctx = _ctx(n_bins=B, n_points_cap=N, mode="scale", k_cand=16)
    dirs, knn = ctx.atlas()
    assert np.array_equal(knn, ops.bin_knn_table(dirs, 16))                 # whole table, bit-exact
    cfg = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", lidar_origin=ORIGIN, tau=ctx.cfg.tau)
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(B)
    for k in range(3):
        sc = syn.make_scan(N, 60 + k)
        ref = opipe.process_scan_bin_path(b, sc, Q, cfg, dirs, knn, ms)
        rec, t, w = device_scan(sc)
        out = ctx.scan(rec, 16, t, w, N, **scan_kwargs(sc), Q=Q)
        X, _, z, Lm, h = ctx.get_belief()
        cert = np.array(out.cert[:])
        assert cert[30] == pytest.approx(ref["beta"], rel=1e-12)
        assert cert[33] == pytest.approx(ref["alpha"], rel=1e-12)
        assert_close(f"C2 scan{k} z_t", np.array(out.z_t[:]), ref["z_t"], rtol=1e-7, atol=1e-9)
        assert_close(f"C2 scan{k} X_anchor", X, ref["belief"].X_anchor, rtol=1e-7, atol=1e-9)
        assert_close(f"C2 scan{k} L", Lm, ref["belief"].L, rtol=1e-7, atol=1e-7 * np.abs(ref["belief"].L).max())
        Lio = ref["imu_odom"]["L"]
        assert_close(f"C2 scan{k} L_imu_odom", np.array(out.L_imu_odom[:]).reshape(22, 22), Lio, rtol=1e-7,
                     atol=1e-9 * np.abs(Lio).max())
        _check_scan_stats(ctx.get_scan_stats(), ref["scan_bins"])
        m_dev, _ = ctx.get_map()
        mref = map_fields(ref["map"].stats)
        assert_close(f"C2 scan{k} map", m_dev, mref, rtol=1e-7, atol=1e-9 * max(np.abs(mref).max(), 1.0))
        b, ms = ref["belief"], ref["map"]
    # every point's nearest bin and K candidate ids, bit-exact (binning.py:56-131 restricted to K)
    sc = syn.make_scan(N, 63)
    rec, t, w = device_scan(sc)
    out = ctx.point_stage(rec, 16, t, w, N, sc["scan_start_time"], sc["scan_end_time"], XI)
    d = ops.point_directions(out["points"].cpu().numpy(), np.array(ORIGIN))
    nearest = ops.nearest_bin(d, dirs)
    assert np.array_equal(out["nearest"].cpu().numpy(), nearest)
    ids, r = ctx.bin_soft_assign()
    sa = ops.bin_soft_assign_scale(d, dirs, knn, ctx.cfg.tau, nearest=nearest)
    assert np.array_equal(ids.cpu().numpy(), sa["indices"])
    assert_close("C2 responsibilities", r.cpu().numpy(), sa["responsibilities"], rtol=1e-9, atol=1e-15)
    ctx.close()


def test_c3_subsample_point_stage_and_moment_match():
    syn = _synthetic()
    cap, B, n = 262144, 1048576, 32768
    ctx = _ctx(n_bins=B, n_points_cap=cap, mode="scale", k_cand=16)
    dirs, knn = ctx.atlas()
    assert np.array_equal(knn, ops.bin_knn_table(dirs, 16))                 # whole 1M x 16 table
    sc = syn.make_scan(n, 70)
    rec, t, w = device_scan(sc)
    out = ctx.point_stage(rec, 16, t, w, n, sc["scan_start_time"], sc["scan_end_time"], XI)
    bud = ops.point_budget_resample(sc["points"], sc["timestamps"], sc["weights"], n_points_cap=cap)
    dk = ops.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], sc["scan_start_time"],
                                   sc["scan_end_time"], XI)
    assert_close("C3 deskewed points", out["points"].cpu().numpy(), dk["points"], rtol=1e-12, atol=1e-12)
    p0, wout = out["points"].cpu().numpy(), out["weights"].cpu().numpy()
    d = ops.point_directions(p0, np.array(ORIGIN))
    nearest = ops.nearest_bin(d, dirs)
    assert np.array_equal(out["nearest"].cpu().numpy(), nearest)
    ids, _ = ctx.bin_soft_assign()
    sa = ops.bin_soft_assign_scale(d, dirs, knn, ctx.cfg.tau, nearest=nearest)
    assert np.array_equal(ids.cpu().numpy(), sa["indices"])
    cert = ctx.scan_bin_moment_match()
    st = _mm_reference(ctx, p0, wout)
    # tau = 0.1 * 48 / 2^20 = 4.6e-6: responsibilities carry ~ulp / tau = 5e-11 relative rounding
    amp = max(1.0, 10 * 2.2e-16 / ctx.cfg.tau / 1e-11)
    _check_scan_stats(ctx.get_scan_stats(), st, amp=amp)
    assert cert[4] == pytest.approx(st["mass_epsilon_ratio"], rel=1e-12)
    ctx.close()


def test_c3_full_scans_value_parity():
    """BASELINE.json configs[2] at full size: two consecutive 262,144-point scans against a
    1,048,576-bin map from the identity prior (the second meets the map the first pushed), each against
    oracle.pipeline.process_scan_bin_path: z_t, X_anchor, L, every bin's ScanBinStats and the map."""
    syn = _synthetic()
    N, B = 262144, 1048576
    ctx = _ctx(n_bins=B, n_points_cap=N, mode="scale", k_cand=16)
    dirs, knn = ctx.atlas()
    cfg = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", lidar_origin=ORIGIN, tau=ctx.cfg.tau)
    b = ops.Belief.identity_prior()
    Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
    ms = opipe.MapState.empty(B)
    amp = max(1.0, 10 * 2.2e-16 / ctx.cfg.tau / 1e-11)   # tau = 4.6e-6 (see the subsample test)
    for k in range(2):
        sc = syn.make_scan(N, 80 + k)
        ref = opipe.process_scan_bin_path(b, sc, Q, cfg, dirs, knn, ms)
        rec, t, w = device_scan(sc)
        out = ctx.scan(rec, 16, t, w, N, **scan_kwargs(sc), Q=Q)
        X, _, z, Lm, h = ctx.get_belief()
        # scan 0 meets an empty map: the planar WLS is eps-weighted: 5e-8 m
        assert_close(f"C3 scan{k} z_t", np.array(out.z_t[:]), ref["z_t"], rtol=1e-7, atol=5e-8)
        assert_close(f"C3 scan{k} X_anchor", X, ref["belief"].X_anchor, rtol=1e-7, atol=5e-8)
        assert_close(f"C3 scan{k} L", Lm, ref["belief"].L, rtol=1e-5, atol=1e-7 * np.abs(ref["belief"].L).max())
        _check_scan_stats(ctx.get_scan_stats(), ref["scan_bins"], amp=amp)
        m_dev, _ = ctx.get_map()
        mref = map_fields(ref["map"].stats)
        # norm-wise per bin and field group (the rotated moments' off-diagonals cancel; gpu_util)
        assert_close_groupwise(f"C3 scan{k} map", m_dev, mref, MAP_GROUPS, rtol=1e-7 * amp,
                               atol=1e-9 * max(np.abs(mref).max(), 1.0))
        b, ms = ref["belief"], ref["map"]
    ctx.close()


def test_scan_lookback_failure_is_reported():
    """k_scan's bounded look-back spin: when it runs out the scan fails loudly (GCS_ERR_HIP ->
    RuntimeError) instead of returning results built on wrong bucket starts; the next scan is
    unaffected (gcs_ctx_set_debug test hook forces the failure path on one look-back tile).  gcs_scan
    runs the sorted bucketing here (its direct buckets have no look-back)."""
    from gcslam import _lib as L
    syn = _synthetic()
    ctx = _ctx(n_bins=20000, n_points_cap=8192, mode="scale")     # 5 look-back tiles
    ctx.set_debug(L.DEBUG_SORTED_BUCKETS, 1)
    sc = syn.make_scan(8192, 5)
    rec, t, w = device_scan(sc)
    ctx.set_debug(L.DEBUG_INJECT_SCAN_FAIL, 1)
    with pytest.raises(RuntimeError, match="spin bound"):
        ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
    with pytest.raises(RuntimeError, match="spin bound"):          # the per-operator entry point too
        ctx.point_stage(rec, 16, t, w, 8192, sc["scan_start_time"], sc["scan_end_time"], XI, want_outputs=False)
        ctx.scan_bin_moment_match()
    ctx.set_debug(L.DEBUG_INJECT_SCAN_FAIL, 0)
    ctx.set_debug(L.DEBUG_SCAN_SPIN_LIMIT, 1 << 22)
    out = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
    assert np.all(np.isfinite(np.array(out.belief.L[:])))
    with pytest.raises(ValueError):
        ctx.set_debug(99, 0)
    ctx.close()
