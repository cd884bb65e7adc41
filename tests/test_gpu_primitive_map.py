"""GPU parity of the primitive map (gcs_pmap_* through gcslam.primitive_map) against the numpy
oracle (oracle/primitive_map.py) on seeded random tiles: slot selections, ids, masks and integer
fields bit-exact; floating fields within the bars written at each assertion."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import primitive_map as opm

pytestmark = pytest.mark.gpu

M = 4096
NL = 3


def _rand_tile(rng, m=M, frac=0.6, seq_hi=40):
    t = opm.create_empty_tile(m)
    v = rng.random(m) < frac
    t["valid_mask"][:] = v
    w = rng.random(m) * 2.0
    w[rng.random(m) < 0.1] = 0.5          # exact ties (stable order by slot)
    w[rng.random(m) < 0.05] = 0.0
    t["weights"][:] = w
    A = rng.normal(size=(m, 3, 3)) * 0.3
    t["Lambdas"][:] = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * rng.uniform(0.5, 4.0, size=(m, 1, 1))
    t["thetas"][:] = rng.normal(size=(m, 3)) * 3.0
    t["etas"][:] = rng.normal(size=(m, NL, 3))
    t["timestamps"][:] = rng.uniform(0, 10, m)
    t["created_timestamps"][:] = rng.uniform(0, 10, m)
    t["last_supported_scan_seq"][:] = rng.integers(0, seq_hi, m)
    t["last_update_scan_seq"][:] = rng.integers(0, seq_hi, m)
    t["primitive_ids"][:] = rng.permutation(10 * m)[:m]
    t["colors"][:] = rng.random((m, 3))
    cam = np.where(rng.random(m) < 0.3, rng.random(m), 0.0)
    t["cam_mass"][:] = cam
    t["lidar_mass"][:] = rng.random(m)
    t["rgb_cam_accum"][:] = rng.random((m, 3)) * cam[:, None]
    t["rgb_cam_denom"][:] = cam
    t["rgb"][:] = np.where((cam > 0)[:, None], rng.random((m, 3)), 0.5)
    return t


def _map(tiles, m=M, max_merge=0):
    from gcslam.primitive_map import AtlasMap
    am = AtlasMap(m_tile=m, max_tiles=8, n_lobes=NL, max_merge=max_merge)
    for tid, t in tiles.items():
        am.write_tile(tid, t)
    return am


def _same_tile(got, ref, rtol=0.0, what=""):
    for f in opm.FIELDS_I64 + ("valid_mask",):
        assert np.array_equal(got[f], ref[f]), f"{what} {f}"
    for f in opm.FIELDS_F64:
        a, b = got[f], ref[f]
        if rtol == 0.0:
            assert np.array_equal(a, b), f"{what} {f}: max |diff| {np.abs(a - b).max()}"
        else:
            np.testing.assert_allclose(a, b, rtol=rtol, atol=rtol * max(1.0, np.abs(b).max()), err_msg=f"{what} {f}")


def test_view_matches_oracle():
    rng = np.random.default_rng(1)
    tiles = {11: _rand_tile(rng), 12: _rand_tile(rng, frac=0.2)}
    am = _map(tiles)
    v = opm.extract_atlas_map_view(tiles, [11, 99, 12], 1024, M)
    g = __import__("gcslam.primitive_map", fromlist=["x"]).extract_atlas_map_view(am, [11, 99, 12], 1024)
    cpu = lambda x: x.detach().cpu().numpy()  # noqa: E731
    assert np.array_equal(cpu(g.candidate_slots), v["candidate_slots"])          # stable top-k, ties by slot
    assert np.array_equal(cpu(g.candidate_tile_ids), v["candidate_tile_ids"])
    assert np.array_equal(cpu(g.valid_mask), v["valid_mask"])
    assert np.array_equal(cpu(g.primitive_ids), v["primitive_ids"])
    assert np.array_equal(cpu(g.last_supported_scan_seq), v["last_supported_scan_seq"])
    assert np.array_equal(cpu(g.weights), v["weights"])
    assert np.array_equal(cpu(g.etas), v["etas"]) and np.array_equal(cpu(g.colors), v["colors"])
    # LU solve / inverse of (Lambda + eps I): the pivot order is LAPACK's, the rounding may differ
    np.testing.assert_allclose(cpu(g.positions), v["positions"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(cpu(g.covariances), v["covariances"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(cpu(g.kappas), v["kappas"], rtol=1e-15, atol=0)   # same sum order, no FMA
    np.testing.assert_allclose(cpu(g.directions), v["directions"], rtol=1e-15, atol=1e-16)
    am.close()


def test_insert_masked_matches_oracle():
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(2)
    tiles = {1: _rand_tile(rng, frac=0.99), 2: _rand_tile(rng, frac=0.3), 3: _rand_tile(rng, frac=1.0)}
    tiles[3]["weights"][:] = 0.25                     # retention ties everywhere in tile 3
    tiles[3]["last_supported_scan_seq"][:] = 7
    am = _map(tiles)
    am.next_global_id = 1000
    K = 64
    ids_t = [2, 1, 3]
    P = dict(L=rng.normal(size=(3, K, 3, 3)), th=rng.normal(size=(3, K, 3)), e=rng.normal(size=(3, K, NL, 3)),
             w=rng.random((3, K)), v=rng.random((3, K)) < 0.7, c=rng.random((3, K, 3)) * 1.4 - 0.2,
             s=rng.integers(0, 2, (3, K)).astype(np.int32))
    res = gpm.primitive_map_insert_masked_tiles(am, ids_t, P["L"], P["th"], P["e"], P["w"], 5.5, P["v"], scan_seq=41,
                                                colors_new=P["c"], sources_new=P["s"])
    nxt = 1000
    for k, tid in enumerate(ids_t):
        n, ids, dropped, nxt = opm.insert_masked(tiles[tid], nxt, P["L"][k], P["th"][k], P["e"][k], P["w"][k], 5.5,
                                                 P["v"][k], scan_seq=41, colors_new=P["c"][k], sources_new=P["s"][k])
        r, cert, eff = res[k]
        assert r.n_inserted == n and eff.realized == n and (cert.exact == (dropped == 0))
        assert np.array_equal(r.new_ids.cpu().numpy(), ids)
        _same_tile(am.read_tile(tid), tiles[tid], what=f"tile {tid}")      # copies and products: bitwise
        assert am.counts[tid] == int(tiles[tid]["valid_mask"].sum())
    assert am.next_global_id == nxt
    am.close()


def test_fuse_matches_oracle():
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(3)
    tiles = {5: _rand_tile(rng), 6: _rand_tile(rng), 7: _rand_tile(rng)}
    am = _map(tiles)
    R = 3000
    tile_flat = rng.choice([5, 6, 7, 8], size=R)      # tile 8 is not active: its rows do nothing
    slots = rng.integers(0, 300, R)                   # many repeated targets
    Lm = rng.normal(size=(R, 3, 3))
    th, et, w = rng.normal(size=(R, 3)), rng.normal(size=(R, NL, 3)), rng.random(R)
    resp, valid = rng.random(R), rng.random(R) < 0.8
    cols, srcs = rng.random((R, 3)) * 1.5 - 0.25, rng.integers(0, 2, R).astype(np.int32)
    active = [6, 5, 7]
    res = gpm.primitive_map_fuse_tiles(am, active, tile_flat, slots, Lm, th, et, w, resp, 9.25, scan_seq=50,
                                       valid_mask=valid, colors_meas=cols, sources_meas=srcs)
    for k, tid in enumerate(active):
        n = opm.fuse(tiles[tid], slots, Lm, th, et, w, resp, 9.25, scan_seq=50, valid_mask=valid & (tile_flat == tid),
                     colors_meas=cols, sources_meas=srcs)
        assert res[k][0].n_fused == n
        _same_tile(am.read_tile(tid), tiles[tid], what=f"tile {tid}")      # same sum order: bitwise
    am.close()


def test_cull_forget_recency_match_oracle():
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(4)
    tiles = {1: _rand_tile(rng), 2: _rand_tile(rng)}
    tiles[1]["weights"][rng.random(M) < 0.2] = 5e-5
    am = _map(tiles)
    r, cert, eff = gpm.primitive_map_cull(am, 1, 1e-4)
    n, dropped, ratio = opm.cull(tiles[1], 1e-4)
    assert r.n_culled == n and n > 0
    assert r.mass_dropped == pytest.approx(dropped, rel=1e-13)               # fixed-order tree vs numpy pairwise
    assert cert.influence.mass_epsilon_ratio == pytest.approx(ratio, rel=1e-13)
    gpm.primitive_map_forget(am, 2, 0.995)
    opm.forget(tiles[2], 0.995)
    _, _, _, st = gpm.primitive_map_recency_inflate(am, [2, 1, 77], 45, 0.02, 0.05)
    s_ref = opm.recency_inflate(tiles, [2, 1, 77], 45, 0.02, 0.05)
    assert st.staleness_inflation_strength == pytest.approx(s_ref[0], rel=1e-12)
    assert st.staleness_cov_inflation_trace == pytest.approx(s_ref[1], rel=1e-12)
    assert st.stale_precision_downscale_total == pytest.approx(s_ref[2], rel=1e-12)
    for tid in (1, 2):   # exp on the device vs numpy: 1 ulp in the decay
        _same_tile(am.read_tile(tid), tiles[tid], rtol=1e-15, what=f"tile {tid}")
    am.close()


def test_merge_reduce_matches_oracle():
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(5)
    m = 512
    t = _rand_tile(rng, m=m, frac=0.9)
    # well-separated primitives plus a few close pairs (distinct distances)
    mu = rng.uniform(-50, 50, size=(m, 3))
    t["Lambdas"][:] = np.eye(3)[None] * rng.uniform(1.0, 2.0, size=(m, 1, 1))
    for a, b, d in ((3, 40, 0.01), (7, 8, 0.02), (100, 300, 0.005), (40, 41, 0.003), (200, 201, 0.015)):
        mu[b] = mu[a] + d
        t["Lambdas"][b] = t["Lambdas"][a]
        t["valid_mask"][[a, b]] = True
    t["thetas"][:] = np.einsum("nij,nj->ni", t["Lambdas"], mu)
    am = _map({0: t}, m=m, max_merge=m)
    r, cert, eff = gpm.primitive_map_merge_reduce(am, 0, merge_threshold=0.1, max_pairs=4, max_tile_size=2048)
    n, status, pairs = opm.merge_reduce(t, merge_threshold=0.1, max_pairs=4, max_tile_size=2048)
    assert r.n_merged == n >= 3 and am.last_merge_pairs == pairs and cert.frobenius_applied
    _same_tile(am.read_tile(0), t, rtol=1e-12, what="merged tile")
    am.close()


def test_reference_merge_and_color_tests_on_gpu():
    """test_primitive_map_merge_reduce.py:76-98 and test_map_color_provenance.py:69-82 through the
    device operators."""
    from gcslam import primitive_map as gpm
    t = opm.create_empty_tile(3)
    t["Lambdas"][:] = np.eye(3)
    t["thetas"][:] = [[0.0, 0, 0], [0.01, 0, 0], [10.0, 0, 0]]
    t["weights"][:] = 1.0
    t["primitive_ids"][:] = [0, 1, 2]
    t["valid_mask"][:] = True
    t["cam_mass"][:] = [1.0, 0.0, 0.0]
    t["lidar_mass"][:] = [0.0, 1.0, 1.0]
    t["rgb_cam_accum"][0] = [1.0, 0.0, 0.0]
    t["rgb_cam_denom"][:] = [1.0, 0.0, 0.0]
    t["rgb"][0] = [1.0, 0.0, 0.0]
    am = _map({0: t}, m=3, max_merge=3)
    am.next_global_id, am.total_count = 3, 3
    r, cert, eff = gpm.primitive_map_merge_reduce(am, 0, merge_threshold=0.5, max_pairs=1, max_tile_size=10)
    g = am.read_tile(0)
    assert r.n_merged == 1 and g["valid_mask"].tolist() == [True, False, True]
    assert np.isclose(g["weights"][0], 2.0) and am.total_count == 2 and cert.frobenius_applied and eff.realized == 1.0
    am.close()
    for first, second, want in (((1.0, 0.0, 0.0), 0, (0.2, 0.2, 0.2)), ((0.2, 0.2, 0.2), 1, (0.0, 1.0, 0.0))):
        am = gpm.AtlasMap(m_tile=1, max_tiles=1, n_lobes=NL, max_merge=0)
        gpm.primitive_map_insert_masked(am, 0, np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, NL, 3)),
                                        np.array([1.0]), 0.0, np.array([True]), colors_new=np.array([first]),
                                        sources_new=np.array([second]))
        gpm.primitive_map_fuse(am, 0, np.array([0]), np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, NL, 3)),
                               np.array([1.0]), np.array([1.0]), 1.0, scan_seq=1, valid_mask=np.array([True]),
                               colors_meas=np.array([want]), sources_meas=np.array([1 - second]))
        expect = first if second == 0 else want
        assert np.allclose(am.read_tile(0)["rgb"][0], expect, atol=1e-6)
        am.close()


def test_map_update_step_matches_oracle():
    """Step 12b (pipeline.py:1244-1447) through gcs_pmap_map_update against the oracle's restatement:
    per-block fuse into the active tiles, novelty insertion, cull / forget; a second scan merges
    (m_tile <= merge_max_tile_size)."""
    from types import SimpleNamespace
    from gcslam import primitive_map as gpm
    from oracle import se3
    rng = np.random.default_rng(6)
    m, N, K = 1024, 600, 8
    tiles = {}
    am = gpm.AtlasMap(m_tile=m, max_tiles=16, n_lobes=NL, max_merge=m)
    z = np.array([1.5, -0.7, 0.3, 0.02, -0.01, 0.4])
    R, t = se3.so3_exp(z[3:]), z[:3]
    for scan in range(2):
        p_body = rng.uniform(-5, 5, size=(N, 3))
        A = rng.normal(size=(N, 3, 3)) * 0.2
        Lam = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * rng.uniform(1, 5, size=(N, 1, 1))
        batch = dict(Lambdas=Lam, thetas=np.einsum("nij,nj->ni", Lam, p_body), etas=rng.normal(size=(N, NL, 3)),
                     weights=rng.random(N), valid_mask=rng.random(N) < 0.9, colors=rng.random((N, 3)),
                     sources=rng.integers(0, 2, N).astype(np.int32))
        wtid = opm.tile_ids_from_xyz(p_body @ R.T + t[None], 2.0)
        uniq, cnts = np.unique(wtid, return_counts=True)
        active = [int(x) for x in uniq[np.argsort(-cnts, kind="stable")][:6]] + [12345]
        ctile = rng.choice(np.array(active[:6] + [777], dtype=np.int64), size=(N, K))
        assoc = dict(responsibilities=rng.random((N, K)) / K, candidate_tile_ids=ctile,
                     candidate_slots=rng.integers(0, m, size=(N, K)), row_masses=rng.random(N) * 2.0 / N)
        nxt_ref, st_ref = opm.map_update_step(tiles, am.next_global_id, batch, assoc, R, t, active, m, 3.0 + scan,
                                              10 + scan, k_insert_tile=64, h_tile=2.0)
        st = gpm.primitive_map_update(am, SimpleNamespace(**batch), SimpleNamespace(**assoc), z, active, 3.0 + scan,
                                      10 + scan)
        assert am.next_global_id == nxt_ref
        for k in ("fused_count", "insert_count_total", "evicted_count", "merged_count"):
            assert st[k] == st_ref[k], k
        for k in ("fused_mass_total", "insert_mass_total", "insert_mass_p95", "evicted_mass_total"):
            assert st[k] == pytest.approx(st_ref[k], rel=1e-12, abs=1e-300), k
        for tid in active:   # world transforms: so3_exp and LU rounding -> 1e-12 relative
            _same_tile(am.read_tile(tid), tiles[tid], rtol=1e-11, what=f"scan {scan} tile {tid}")
            assert am.counts[tid] == int(tiles[tid]["valid_mask"].sum())
    assert st_ref["insert_count_total"] > 0 and st_ref["fused_count"] > 0
    am.close()


CASES = ["all_invalid", "ragged_blocks", "no_insert", "populated", "empty_active", "hot_slots"]


@pytest.mark.parametrize("case", CASES)
def test_map_update_edge_cases(case):
    """Step 12b edge cases against the oracle: an all-invalid MeasurementBatch (zero fused and
    inserted mass, cull / forget still run), a ragged last association block (N = 301, block 128), a zero
    insert budget, tiles already holding primitives (retention evictions on insert, merges), an
    empty active-tile list (exact no-op), and every candidate on three slots per tile (runs of ~100 rows
    per (tile, slot, block): k_pm_fuse_chunks cuts them into chunk sums, at the step-12b bar)."""
    from types import SimpleNamespace
    from gcslam import primitive_map as gpm
    from oracle import se3
    rng = np.random.default_rng(20 + CASES.index(case))
    m, N, K = 1024, (301 if case == "ragged_blocks" else 400), 8
    block = 128 if case == "ragged_blocks" else 256
    kins = 0 if case == "no_insert" else 64
    cfg = gpm.PrimitiveMapUpdateConfig(k_insert_tile=kins, block_size=block)
    z = np.array([0.4, 0.2, -0.3, -0.03, 0.02, 0.9])
    R, t = se3.so3_exp(z[3:]), z[:3]
    p_body = rng.uniform(-4, 4, size=(N, 3))
    A = rng.normal(size=(N, 3, 3)) * 0.2
    Lam = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * rng.uniform(1, 5, size=(N, 1, 1))
    valid = np.zeros(N, bool) if case == "all_invalid" else rng.random(N) < 0.85
    batch = dict(Lambdas=Lam, thetas=np.einsum("nij,nj->ni", Lam, p_body), etas=rng.normal(size=(N, NL, 3)),
                 weights=rng.random(N), valid_mask=valid, colors=rng.random((N, 3)),
                 sources=rng.integers(0, 2, N).astype(np.int32))
    wtid = opm.tile_ids_from_xyz(p_body @ R.T + t[None], 2.0)
    uniq, cnts = np.unique(wtid, return_counts=True)
    active = [] if case == "empty_active" else [int(x) for x in uniq[np.argsort(-cnts, kind="stable")][:5]]
    tiles = {}
    if case in ("populated", "all_invalid", "empty_active"):
        for tid in (active or [int(uniq[0])]):
            tt = _rand_tile(rng, m=m, frac=0.97 if case == "populated" else 0.5, seq_hi=30)
            tt["weights"][rng.random(m) < 0.05] = 1e-6      # below the cull threshold
            tiles[tid] = tt
    am = gpm.AtlasMap(m_tile=m, max_tiles=16, n_lobes=NL, max_merge=m)
    for tid, tt in tiles.items():
        am.write_tile(tid, tt)
    am.next_global_id = 50_000
    before = {tid: {k: v.copy() for k, v in tt.items()} for tid, tt in tiles.items()}
    ctile = rng.choice(np.array(active + [777], dtype=np.int64), size=(N, K))
    assoc = dict(responsibilities=rng.random((N, K)) / K, candidate_tile_ids=ctile,
                 candidate_slots=rng.integers(0, 3 if case == "hot_slots" else m, size=(N, K)),
                 row_masses=rng.random(N) * 2.0 / N)
    nxt_ref, st_ref = opm.map_update_step(tiles, 50_000, batch, assoc, R, t, active, m, 7.0, 33,
                                          k_insert_tile=kins, h_tile=2.0, block_size=block)
    st = gpm.primitive_map_update(am, SimpleNamespace(**batch), SimpleNamespace(**assoc), z, active, 7.0, 33, cfg)
    assert am.next_global_id == nxt_ref
    for k in ("fused_count", "insert_count_total", "evicted_count", "merged_count"):
        assert st[k] == st_ref[k], k
    for k in ("fused_mass_total", "insert_mass_total", "insert_mass_p95", "evicted_mass_total"):
        assert st[k] == pytest.approx(st_ref[k], rel=1e-12, abs=1e-300), k
    for tid in active:
        _same_tile(am.read_tile(tid), tiles[tid], rtol=1e-11, what=f"{case} tile {tid}")
        assert am.counts[tid] == int(tiles[tid]["valid_mask"].sum())
    if case == "all_invalid":   # the mask zeroes responsibilities and novelty; counts still follow the reference
        assert st["fused_mass_total"] == 0.0 and st["insert_mass_total"] == 0.0 and st["evicted_count"] > 0
    if case == "no_insert":
        assert st["insert_count_total"] == 0 and st["fused_count"] > 0
    if case == "populated":
        assert st["insert_count_total"] > 0
    if case == "empty_active":
        assert all(v == 0 for k, v in st.items() if k not in ("tile_ids_active",))
        for tid, tt in before.items():   # untouched
            _same_tile(am.read_tile(tid), tt, what=f"untouched tile {tid}")
    am.close()


def test_view_sparse_and_empty_tiles():
    """extract_atlas_map_view when a tile holds fewer valid primitives than m_tile_view (the top-k
    falls through to invalid slots in slot order) and when a tile is empty or absent."""
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(9)
    tiles = {3: _rand_tile(rng, frac=0.002), 4: _rand_tile(rng, frac=0.0)}
    am = _map(tiles)
    order = [4, 3, 55]
    v = opm.extract_atlas_map_view(tiles, order, 1024, M)
    g = gpm.extract_atlas_map_view(am, order, 1024)
    cpu = lambda x: x.detach().cpu().numpy()  # noqa: E731
    assert int(tiles[3]["valid_mask"].sum()) < 1024
    for f in ("candidate_slots", "candidate_tile_ids", "valid_mask", "primitive_ids", "weights"):
        assert np.array_equal(cpu(getattr(g, f)), v[f]), f
    np.testing.assert_allclose(cpu(g.positions), v["positions"], rtol=1e-12, atol=1e-12)
    am.close()


@pytest.mark.parametrize("fracs", [(0.999, 0.8, 0.8, 0.8, 0.8, 0.0), (0.01, 0.02, 0.04, 0.05, 0.001, 0.0)],
                         ids=["dense", "sparse"])
def test_reference_size_view_and_map_update(fracs):
    _reference_size_update(fracs)


def test_twice_reference_rows_map_update():
    """Step 12b past the one-group LDS merge's 16,384 fuse rows: 2,048 measurement rows (the map update's
    limit, kPropLds) x K = 12 candidates = 24,576 rows, twice the reference's 1,536 x 8 -- the fuse sort's
    multi-group k_ss_merge (no rocPRIM), against the oracle."""
    _reference_size_update((0.999, 0.8, 0.8, 0.8, 0.8, 0.0), N=2048, K=12, seed=51)


def _reference_size_update(fracs, N=1536, K=8, seed=50):
    """The reference's map sizes (GC_M_TILE = 50,000 slots, GC_M_TILE_VIEW = 1,024, 7 active tiles,
    constants.py:392,436-439; N = 512 + 1,024 measurement rows, K = 8, constants.py:350-356): the view's
    per-tile top-k over 50,000 keys (ties and an empty tile whose keys are all equal included) and
    step 12b with novelty insertion into populated tiles (eviction order by the same top-k) against
    the oracle.  dense: full and 80 % tiles (the tree of sorted runs, k_pm_topk); sparse: tiles of
    50-2,500 primitives (k_pm_topk_sparse -- a few hundred to ~2,000 besides the empty slots, the
    5 % tile past its 2,048 capacity back on the tree)."""
    from types import SimpleNamespace
    from gcslam import primitive_map as gpm
    from oracle import se3
    rng = np.random.default_rng(seed)
    m, kv = 50_000, 1024
    z = np.array([0.9, -0.4, 0.2, 0.01, -0.02, 0.3])
    R, t = se3.so3_exp(z[3:]), z[:3]
    p_body = rng.uniform(-5, 5, size=(N, 3))
    A = rng.normal(size=(N, 3, 3)) * 0.2
    Lam = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * rng.uniform(1, 5, size=(N, 1, 1))
    batch = dict(Lambdas=Lam, thetas=np.einsum("nij,nj->ni", Lam, p_body), etas=rng.normal(size=(N, NL, 3)),
                 weights=rng.random(N), valid_mask=rng.random(N) < 0.9, colors=rng.random((N, 3)),
                 sources=rng.integers(0, 2, N).astype(np.int32))
    wtid = opm.tile_ids_from_xyz(p_body @ R.T + t[None], 2.0)
    uniq, cnts = np.unique(wtid, return_counts=True)
    active = [int(x) for x in uniq[np.argsort(-cnts, kind="stable")][:7]]
    assert len(active) == 7
    tiles = {}
    for i, tid in enumerate(active[:6]):   # five populated tiles (one full), one empty; the 7th is absent
        tiles[tid] = _rand_tile(rng, m=m, frac=fracs[i], seq_hi=30)
    am = gpm.AtlasMap(m_tile=m, max_tiles=16, n_lobes=NL, max_merge=0)
    for tid, tt in tiles.items():
        am.write_tile(tid, tt)
    am.next_global_id = 10 * m
    view = gpm.extract_atlas_map_view(am, active, kv)
    v = opm.extract_atlas_map_view(tiles, active, kv, m)
    cpu = lambda x: x.detach().cpu().numpy()  # noqa: E731
    for f in ("candidate_slots", "candidate_tile_ids", "valid_mask", "primitive_ids", "weights"):
        assert np.array_equal(cpu(getattr(view, f)), v[f]), f
    np.testing.assert_allclose(cpu(view.positions), v["positions"], rtol=1e-12, atol=1e-12)
    ctile = rng.choice(np.array(active + [777], dtype=np.int64), size=(N, K))
    assoc = dict(responsibilities=rng.random((N, K)) / K, candidate_tile_ids=ctile,
                 candidate_slots=rng.integers(0, m, size=(N, K)), row_masses=rng.random(N) * 2.0 / N)
    nxt_ref, st_ref = opm.map_update_step(tiles, 10 * m, batch, assoc, R, t, active, m, 4.0, 31, k_insert_tile=64,
                                          h_tile=2.0)
    st = gpm.primitive_map_update(am, SimpleNamespace(**batch), SimpleNamespace(**assoc), z, active, 4.0, 31)
    assert am.next_global_id == nxt_ref
    for k in ("fused_count", "insert_count_total", "evicted_count", "merged_count"):
        assert st[k] == st_ref[k], k
    for k in ("fused_mass_total", "insert_mass_total", "insert_mass_p95", "evicted_mass_total"):
        assert st[k] == pytest.approx(st_ref[k], rel=1e-12, abs=1e-300), k
    for tid in active:
        _same_tile(am.read_tile(tid), tiles[tid], rtol=1e-11, what=f"tile {tid}")
        assert am.counts[tid] == int(tiles[tid]["valid_mask"].sum())
    assert st_ref["insert_count_total"] > 0
    am.close()


def _full_sort_check():
    """Run in a subprocess with GCSLAM_PM_FULLSORT=1 (the knob is read once per process): the view's
    and the insert's rocPRIM full-sort path against the oracle."""
    rng = np.random.default_rng(3)
    tiles = {5: _rand_tile(rng), 6: _rand_tile(rng, frac=0.1)}
    am = _map(tiles)
    from gcslam import primitive_map as gpm
    v = opm.extract_atlas_map_view(tiles, [5, 6], 1024, M)
    g = gpm.extract_atlas_map_view(am, [5, 6], 1024)
    for f in ("candidate_slots", "candidate_tile_ids", "valid_mask", "primitive_ids", "weights"):
        assert np.array_equal(getattr(g, f).cpu().numpy(), v[f]), f
    K = 64
    P = dict(L=rng.normal(size=(1, K, 3, 3)), th=rng.normal(size=(1, K, 3)), e=rng.normal(size=(1, K, NL, 3)),
             w=rng.random((1, K)), v=rng.random((1, K)) < 0.7)
    am.next_global_id = 500
    res = gpm.primitive_map_insert_masked_tiles(am, [5], P["L"], P["th"], P["e"], P["w"], 2.5, P["v"], scan_seq=40)
    n, ids, _, _ = opm.insert_masked(tiles[5], 500, P["L"][0], P["th"][0], P["e"][0], P["w"][0], 2.5, P["v"][0],
                                     scan_seq=40)
    assert res[0][0].n_inserted == n and np.array_equal(res[0][0].new_ids.cpu().numpy(), ids)
    _same_tile(am.read_tile(5), tiles[5], what="full-sort insert")
    am.close()


def test_radix_select_path_matches_oracle():
    """The register select (M <= 8,192) and the tree top-k (k_pm_topk, larger tiles: the 50,000-slot test
    above) are the defaults; the one-workgroup radix select (GCSLAM_PM_SELECT=radix) keeps its own
    parity check."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_gpu_primitive_map as t; t._full_sort_check()"
            % (here, root, os.path.join(root, "gc-slam_amd")))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, GCSLAM_PM_SELECT="radix"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]


def test_full_sort_path_matches_oracle():
    """The select is the default for k <= 1024; the rocPRIM full sort (GCSLAM_PM_FULLSORT=1, or k above
    the select's capacity) keeps its own parity check."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_gpu_primitive_map as t; t._full_sort_check()"
            % (here, root, os.path.join(root, "gc-slam_amd")))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, GCSLAM_PM_FULLSORT="1"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]


def test_topk_tree_handoff_stress():
    """The tree top-k's run hand-off between workgroups (k_pm_topk, GCS_TOPK_SC1: write-through stores,
    a relaxed ticket and one acquire by the second arrival; cdna_hip_programming.md Guideline 16) under
    repetition: 24 views of seven dense 50,000-slot tiles with fresh weights each time (ties included),
    every candidate slot against the oracle's stable top-k (primitive_map.py:303-322).  A stale run
    handed to the next merge level would show as a wrong or duplicated slot."""
    from gcslam import primitive_map as gpm
    rng = np.random.default_rng(77)
    m, kv, n_t = 50_000, 1024, 7
    am = gpm.AtlasMap(m_tile=m, max_tiles=8, n_lobes=NL, max_merge=0)
    tids = [1000 + 3 * k for k in range(n_t)]
    base = {t: _rand_tile(rng, m=m, frac=0.8, seq_hi=30) for t in tids}
    for t in tids:
        am.write_tile(t, base[t])
    try:
        for rep in range(24):
            w = {}
            for t in tids:
                ww = rng.random(m)
                if rep % 3 == 0:
                    ww = np.round(ww * 64) / 64.0  # many exact ties: the slot order decides
                w[t] = ww
                am.write_tile(t, {"weights": ww})
            view = gpm.extract_atlas_map_view(am, tids, kv)
            got = view.candidate_slots.detach().cpu().numpy().reshape(n_t, kv)
            for i, t in enumerate(tids):
                ref = opm.select_topk_slots(w[t], base[t]["valid_mask"], kv)
                assert np.array_equal(got[i], ref), (rep, t, np.flatnonzero(got[i] != ref)[:8])
    finally:
        am.close()


@pytest.mark.parametrize("env", [{"GCSLAM_FUSE_SMALLSORT": "0"}, {"GCSLAM_PM_TOPK_SPARSE": "0"}],
                         ids=["fuse_rocprim_sort", "topk_tree_only"])
def test_reference_size_map_update_knob_paths(env):
    """Step 12b's defaults are the two-launch LDS sort of the fuse keys (k_ss_block + k_ss_merge) and the
    empty-slot shortcut of the eviction order on dense tiles (k_pm_topk_sparse); rocPRIM's radix sort
    and the tree of sorted runs for every tile stay selectable (A/B) and keep their own parity check on
    the reference-size dense scene."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_gpu_primitive_map as t; "
            "t.test_reference_size_view_and_map_update((0.999, 0.8, 0.8, 0.8, 0.8, 0.0)); "
            "t.test_twice_reference_rows_map_update()"
            % (here, root, os.path.join(root, "gc-slam_amd")))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
