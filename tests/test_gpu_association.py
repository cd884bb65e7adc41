"""OT association on the GPU (gcs_associate_primitives_ot through gcslam.association) against the
numpy oracle (oracle/association.py, primitive_association.py:105-553).

Bars: candidate pool indices, candidate tile ids and slots bit-exact (cost order with stable ties,
the reference's lax.sort num_keys=1); the selected costs at rtol 1e-12 (every term is an
elementwise chain in numpy's operation order; the 3x3 solve and libm transcendentals differ by
ulps); responsibilities and row masses at rtol 1e-9 + atol 1e-12 x the largest entry (50 unbalanced
Sinkhorn iterations of pow, fixed-order reductions on both sides but different orders); OTCert /
Support / Influence scalars at rtol 1e-9; the p95 order statistics at rtol 1e-12 (selected values).
Scenes: tests/assoc_util.py (seeded MA-hex tile atlas, reference sizes N_total = 512 + 1024,
k_assoc = 8, 7 stencil tiles x m_tile_view = 1024)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from assoc_util import budget_scene, make_scene
from oracle import association as OA
from gcslam import association as GA
from gcslam.surfels import MeasurementBatch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _batch(b):
    t = lambda x, dt=torch.float64: torch.as_tensor(np.asarray(x), device=DEV).to(dt)  # noqa: E731
    nf, ns = int(b["n_feat"]), int(b["n_surfel"])
    N = nf + ns
    return MeasurementBatch(Lambdas=t(b["Lambdas"]), thetas=t(b["thetas"]), etas=t(b["etas"]), weights=t(b["weights"]),
                            sources=torch.zeros(N, dtype=torch.int32, device=DEV),
                            source_indices=torch.zeros(N, dtype=torch.int32, device=DEV),
                            valid_mask=t(b["valid_mask"], torch.bool), timestamps=torch.zeros(N, dtype=torch.float64,
                                                                                              device=DEV),
                            colors=torch.zeros((N, 3), dtype=torch.float64, device=DEV), n_feat=nf, n_surfel=ns,
                            n_camera_valid=int(b["n_valid"]), n_lidar_valid=0)


def _view(v):
    t = lambda x, dt: torch.as_tensor(np.asarray(x), device=DEV).to(dt)  # noqa: E731
    return GA.AtlasMapView(candidate_tile_ids=t(v["candidate_tile_ids"], torch.int64),
                           candidate_slots=t(v["candidate_slots"], torch.int32), valid_mask=t(v["valid_mask"], torch.bool),
                           tile_ids=t(v["tile_ids"], torch.int64), m_tile_view=int(v["m_tile_view"]),
                           positions=t(v["positions"], torch.float64), directions=t(v["directions"], torch.float64),
                           kappas=t(v["kappas"], torch.float64),
                           last_supported_scan_seq=t(v["last_supported_scan_seq"], torch.int64))


def _gcfg(c: OA.AssociationConfig) -> GA.AssociationConfig:
    d = {k: getattr(c, k) for k in c.__dataclass_fields__}
    d["a_policy"] = GA.MeasurementMassPolicy(d["a_policy"])
    d["b_policy"] = GA.MapMassPolicy(d["b_policy"])
    return GA.AssociationConfig(**d)


_VIEW_VALID = [None]


def _run_both(batch, view, cfg):
    _VIEW_VALID[0] = np.asarray(view["valid_mask"]).astype(bool)
    ref, rc = OA.associate_primitives_ot(batch, view, cfg)
    res, cert, eff = GA.associate_primitives_ot(_batch(batch), _view(view), _gcfg(cfg))
    torch.cuda.synchronize()
    return ref, rc, res, cert, eff


def _check(ref, rc, res, cert, eff, valid):
    g = lambda x: x.cpu().numpy()  # noqa: E731
    for k in ("candidate_pool_indices", "candidate_tile_ids", "candidate_slots"):
        assert np.array_equal(g(getattr(res, k)), ref[k]), k
    C, Cr = g(res.cost_matrix), ref["cost_matrix"]
    np.testing.assert_allclose(C, Cr, rtol=1e-12, atol=1e-12 * max(np.abs(Cr).max(), 1e-300))
    R, Rr = g(res.responsibilities), ref["responsibilities"]
    np.testing.assert_allclose(R, Rr, rtol=1e-9, atol=1e-12 * max(np.abs(Rr).max(), 1e-300))
    np.testing.assert_allclose(g(res.row_masses), ref["row_masses"], rtol=1e-9,
                               atol=1e-12 * max(np.abs(ref["row_masses"]).max(), 1e-300))
    assert np.all(R[~valid] == 0.0)
    # the MapUpdateCert's candidate statistics (pipeline.py:879-905), computed by the library beside the
    # Sinkhorn, against the restatement on the device's own candidate outputs: exact (integer sums)
    cs = OA.candidate_stats(valid, _VIEW_VALID[0], g(res.candidate_pool_indices), g(res.candidate_tile_ids))
    assert tuple(res.candidate_stats) == cs, (res.candidate_stats, cs)
    if rc["exact"]:
        assert cert.exact and eff.predicted == 0.0
        return
    ot = cert.ot
    for k in ("marginal_defect_a", "marginal_defect_b", "transport_mass_total", "sum_a", "sum_b", "sum_m",
              "sum_novel"):
        np.testing.assert_allclose(getattr(ot, k), rc[k], rtol=1e-9, atol=1e-15, err_msg=k)
    for k in ("p95_a", "p95_b", "b_recency_p95"):
        np.testing.assert_allclose(getattr(ot, k), rc[k], rtol=1e-12, err_msg=k)
    assert ot.nonzero_a == rc["nonzero_a"] and ot.nonzero_b == rc["nonzero_b"]
    np.testing.assert_allclose(cert.support.ess_total, rc["ess_total"], rtol=1e-9)
    np.testing.assert_allclose(cert.support.support_frac, rc["support_frac"], rtol=1e-15)
    np.testing.assert_allclose(cert.influence.mass_epsilon_ratio, rc["mass_epsilon_ratio"], rtol=1e-9)
    np.testing.assert_allclose(eff.predicted, rc["total_cost"], rtol=1e-9, atol=1e-15)
    assert cert.compute.alloc_bytes_est == rc["alloc_bytes_est"]
    assert tuple(cert.compute.largest_tensor_shape) == tuple(rc["largest_tensor_shape"])
    assert cert.approximation_triggers == ["sinkhorn_fixed_iter", "sinkhorn_unbalanced_kl_relax"]


@pytest.mark.parametrize("seed", [0, 1])
def test_association_matches_oracle_reference_sizes(seed):
    batch, view, _ = make_scene(seed=seed)
    cfg = OA.AssociationConfig(scan_seq=10)
    _check(*_run_both(batch, view, cfg), batch["valid_mask"])


@pytest.mark.parametrize("variant", ["weight_proportional", "median_no_rowmin", "k16_r2", "dup_tile"])
def test_association_config_variants(variant):
    kw = dict(seed=7, n_feat=128, n_surfel=256, n_valid_cam=60, n_valid_lidar=200, m_tile=256, m_tile_view=256)
    cfg = OA.AssociationConfig(scan_seq=4)
    if variant == "weight_proportional":
        cfg.a_policy = "weight_proportional"
    elif variant == "median_no_rowmin":
        cfg.cost_subtract_row_min, cfg.cost_scale_by_median = False, True
    elif variant == "k16_r2":
        cfg.k_assoc, cfg.r_stencil_tiles_xy, cfg.r_stencil_tiles_z = 16, 2, 1
    elif variant == "dup_tile":
        kw["dup_tile"] = True
    batch, view, _ = make_scene(**kw)
    _check(*_run_both(batch, view, cfg), batch["valid_mask"])


def test_budget_assertions_association_gpu():
    """test_budget_assertions.py:91-118 on the device: the cert budgets and the closed forms of
    tests/test_association.py (candidates 0..K-1, zero costs, pi = 64^(-2/7))."""
    batch, view = budget_scene()
    K = OA.GC_K_ASSOC
    res, cert, _ = GA.associate_primitives_ot(_batch(batch), _view(view), GA.AssociationConfig(k_assoc=K))
    N = batch["Lambdas"].shape[0]
    assert cert.compute.largest_tensor_shape[0] <= N and cert.compute.largest_tensor_shape[1] <= K
    assert cert.compute.segment_sum_k == K and cert.compute.alloc_bytes_est <= N * K * 8 * 4
    assert np.array_equal(res.candidate_pool_indices.cpu().numpy(), np.tile(np.arange(K, dtype=np.int32), (N, 1)))
    assert np.all(res.cost_matrix.cpu().numpy() == 0.0)
    np.testing.assert_allclose(res.responsibilities.cpu().numpy(), 64.0 ** (-2.0 / 7.0), rtol=1e-12)


def test_empty_map_and_no_valid_rows_are_exact():
    for kw in (dict(fill=(0, 0)), dict(n_valid_cam=0, n_valid_lidar=0)):
        batch, view, _ = make_scene(seed=3, n_feat=32, n_surfel=64, n_valid_cam=kw.get("n_valid_cam", 10),
                                    n_valid_lidar=kw.get("n_valid_lidar", 30), m_tile=64, m_tile_view=64,
                                    fill=kw.get("fill", (0, 64)))
        _check(*_run_both(batch, view, OA.AssociationConfig()), batch["valid_mask"])


def test_unsupported_policy_raises_unless_empty():
    batch, view, _ = make_scene(seed=4, n_feat=32, n_surfel=64, n_valid_cam=10, n_valid_lidar=30, m_tile=64,
                                m_tile_view=64)
    bad = GA.AssociationConfig(b_policy=GA.MapMassPolicy.PRIMITIVE_MASS)
    with pytest.raises(ValueError):
        GA.associate_primitives_ot(_batch(batch), _view(view), bad)
    batch, view, _ = make_scene(seed=4, n_feat=32, n_surfel=64, n_valid_cam=10, n_valid_lidar=30, m_tile=64,
                                m_tile_view=64, fill=(0, 0))
    res, cert, _ = GA.associate_primitives_ot(_batch(batch), _view(view), bad)
    assert cert.exact and float(res.responsibilities.abs().sum()) == 0.0


def test_association_deterministic():
    batch, view, _ = make_scene(seed=9, n_feat=128, n_surfel=256, n_valid_cam=60, n_valid_lidar=200, m_tile=256,
                                m_tile_view=256)
    b, v = _batch(batch), _view(view)
    r1, _, _ = GA.associate_primitives_ot(b, v)
    r2, _, _ = GA.associate_primitives_ot(b, v)
    for k in ("responsibilities", "cost_matrix", "row_masses", "candidate_pool_indices"):
        assert torch.equal(getattr(r1, k), getattr(r2, k)), k


def _knob_paths_check():
    """Run in a subprocess with one of the association's A/B knobs set (they are read once per context
    creation / process): the reference-size scene and two config variants against the oracle."""
    for seed in (0, 1):
        batch, view, _ = make_scene(seed=seed)
        _check(*_run_both(batch, view, OA.AssociationConfig(scan_seq=10)), batch["valid_mask"])
    kw = dict(seed=7, n_feat=128, n_surfel=256, n_valid_cam=60, n_valid_lidar=200, m_tile=256, m_tile_view=256)
    batch, view, _ = make_scene(**kw)
    for extra in (dict(cost_scale_by_median=True, cost_subtract_row_min=False), dict(k_sinkhorn=0)):
        _check(*_run_both(batch, view, OA.AssociationConfig(scan_seq=10, **extra)), batch["valid_mask"])


@pytest.mark.parametrize("env", [{"GCSLAM_POOL_LDS": "0"}, {"GCSLAM_SH_FINSPLIT": "0"}, {"GCSLAM_SH_FINSPLIT": "2"},
                                 {"GCSLAM_PREP_FUSED": "1"}],
                         ids=["pool_l2", "finish_in_wg0", "finish_own_launch", "prep_stage_one_launch"])
def test_association_knob_paths_match_oracle(env):
    """The defaults are the bucketed LDS pool (k_as_prep, k_as_stage, k_as_pool_lds) and the finish in
    extra workgroups of the Sinkhorn launch; the one-workgroup-per-row pool from L2, the prep and staging
    as one launch (k_as_prep_fused) and the two other finish forms stay selectable (A/B) and keep their
    own parity check."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_gpu_association as t; t._knob_paths_check()"
            % (here, root, os.path.join(root, "gc-slam_amd")))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
