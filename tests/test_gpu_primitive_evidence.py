"""GPU parity of visual_pose_evidence (gcs_visual_pose_evidence through gcslam.association) against the
numpy restatement (oracle/primitive_evidence.py) on the association test scenes: the device's
association result feeds both, so the check isolates the evidence stage."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from assoc_util import make_scene
from oracle import primitive_evidence as OE
from gcslam import association as GA
from test_gpu_association import _batch, _view

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,z", [(0, [0.1, -0.2, 0.05, 0.01, -0.02, 0.15]), (3, [0.0] * 6),
                                    (5, [2.0, 1.0, -0.3, 0.3, 0.2, -1.1])])
def test_visual_pose_evidence_matches_oracle(seed, z):
    batch, view, _ = make_scene(seed=seed)
    gb, gv = _batch(batch), _view(view)
    res, _, _ = GA.associate_primitives_ot(gb, gv, GA.AssociationConfig(scan_seq=10))
    out, cert, eff = GA.visual_pose_evidence(res, gb, gv, z_lin_pose=np.array(z))
    g = lambda x: x.detach().cpu().numpy()  # noqa: E731
    ref = OE.visual_pose_evidence(batch, view, dict(responsibilities=g(res.responsibilities),
                                                    candidate_pool_indices=g(res.candidate_pool_indices),
                                                    row_masses=g(res.row_masses)), np.array(z))
    assert not ref["exact"] and not cert.exact and cert.frobenius_applied
    # fixed-order sums vs numpy einsum; Jacobi SVD vs LAPACK (U V^T and s agree to rounding)
    np.testing.assert_allclose(out.L_trans, ref["L_trans"], rtol=1e-11, atol=1e-11 * np.abs(ref["L_trans"]).max())
    np.testing.assert_allclose(out.h_trans, ref["h_trans"], rtol=1e-10, atol=1e-10 * np.abs(ref["h_trans"]).max())
    np.testing.assert_allclose(out.L_rot, ref["L_rot"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(out.h_rot, ref["h_rot"], rtol=1e-8, atol=1e-8 * np.abs(ref["L_rot"]).max())
    np.testing.assert_allclose(out.L_pose, ref["L_pose"], rtol=1e-10, atol=1e-11 * np.abs(ref["L_pose"]).max())
    assert out.total_weighted_cost == pytest.approx(ref["total_weighted_cost"], rel=1e-10)
    assert out.n_associations == ref["n_associations"]
    assert out.mean_transported_mass == pytest.approx(ref["mean_transported_mass"], rel=1e-12)
    assert cert.support.ess_total == pytest.approx(ref["ess_total"], rel=1e-12)
    assert cert.support.support_frac == ref["support_frac"] and eff.realized == out.total_weighted_cost
    L22, h22 = GA.build_visual_pose_evidence_22d(out)
    assert L22.shape == (22, 22) and h22.shape == (22,)


def test_visual_pose_evidence_empty_case():
    batch, view, _ = make_scene(seed=1)
    gb, gv = _batch(batch), _view(view)
    res, _, _ = GA.associate_primitives_ot(gb, gv, GA.AssociationConfig(scan_seq=10))
    gv.valid_mask = torch.zeros_like(gv.valid_mask)
    out, cert, eff = GA.visual_pose_evidence(res, gb, gv, z_lin_pose=np.zeros(6))
    assert cert.exact and eff.predicted == 0.0 and out.n_associations == 0
    assert np.array_equal(out.L_pose, 1e-9 * np.eye(22)) and not out.h_pose.any()


@pytest.mark.parametrize("seed", [0, 5])
def test_split_pose_evidence_bitwise(monkeypatch, seed):
    """k_as_vpe_rows + the ordered fold (default) against the one-workgroup kernel (GCSLAM_VPE_SPLIT=0):
    the same additions on the same values, so every output bit for bit."""
    batch, view, _ = make_scene(seed=seed)
    gb, gv = _batch(batch), _view(view)
    res, _, _ = GA.associate_primitives_ot(gb, gv, GA.AssociationConfig(scan_seq=10))
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("GCSLAM_VPE_SPLIT", flag)
        a = GA.Associator(max_meas=1536, max_pool=7 * 1024, max_k=8)
        try:
            o = a.pose_evidence(gb, gv, res, 8, np.array([0.3, -0.1, 0.2, 0.05, -0.1, 0.4]))
            outs.append(bytes(o))
        finally:
            a.close()
    assert outs[0] == outs[1]
