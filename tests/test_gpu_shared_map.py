"""One map for all hypotheses (gcslam_hip.h GCS_MAP_LEAD / GCS_MAP_FOLLOW): the reference node keeps a
single map and stores hypothesis 0's update (backend_node.py:2036-2083).  Two contexts on one GPU
stand in for two ranks: the lead (hypothesis 0) scans and updates its map; the follower (a perturbed
prior, so its deskew twist and z_t differ) scans against its copy of the lead's map, skips its own
map update and replays the lead's (gcs_map_follow with the lead's record).  Checked over three scans:
the follower's map is bitwise the lead's after every scan, and the follower's z_t / belief match the
oracle run against the lead's map of the previous scan (the declared one-update lag)."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from gpu_util import assert_close, device_scan, map_fields
from oracle import ops, pipeline as opipe
from gcslam.synthetic import scan_kwargs

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)


def _ctx(**kw):
    from gcslam.context import HypothesisContext
    base = dict(lidar_origin=ORIGIN, max_raw_points=1 << 20)
    base.update(kw)
    return HypothesisContext(**base)


@pytest.mark.parametrize("mode,B,cap,n_raw", [("scale", 20000, 8192, 8192), ("dense", 48, 2048, 4096)])
def test_follower_map_is_the_leads_bitwise(mode, B, cap, n_raw):
    from gcslam import synthetic as syn
    lead, fol = _ctx(n_bins=B, n_points_cap=cap, mode=mode), _ctx(n_bins=B, n_points_cap=cap, mode=mode)
    lead.set_map_mode("lead")
    fol.set_map_mode("follow")
    X1 = np.array([0.04, -0.03, 0.0, 0.002, -0.004, 0.006])
    fol.set_belief(X1, 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
    dirs, knn = lead.atlas()
    cfg = opipe.BinPathConfig(n_points_cap=cap, n_bins=B, mode=mode, lidar_origin=ORIGIN, tau=lead.cfg.tau)
    Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
    b0 = ops.Belief.identity_prior()
    b1 = ops.Belief(X1.copy(), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
    ms = opipe.MapState.empty(B)  # the lead's map (the node's map)
    xi_diff = 0.0
    for k in range(3):
        sc = syn.make_scan(n_raw, 5 + k)
        ref0 = opipe.process_scan_bin_path(b0, sc, Q, cfg, dirs, knn, ms)
        ref1 = opipe.process_scan_bin_path(b1, sc, Q, cfg, dirs, knn, ms)  # reads the lead's map of scan k-1
        rec, t, w = device_scan(sc)
        kw = dict(scan_kwargs(sc), Q=Q)
        lead.scan(rec, 16, t, w, n_raw, **kw)
        o1 = fol.scan(rec, 16, t, w, n_raw, **kw)
        r = lead.map_record()
        xi_diff = max(xi_diff, float(np.abs(r[:6] - fol.map_record()[:6]).max()))
        fol.map_follow(fol.prepare_scan(rec, 16, t, w, n_raw, **kw), r)
        lead.synchronize()
        fol.synchronize()
        m0, d0 = lead.get_map()
        m1, d1 = fol.get_map()
        assert np.array_equal(m0, m1) and np.array_equal(d0, d1), f"scan {k}: follower map != lead map"
        assert_close(f"scan{k} follower z_t", np.array(o1.z_t[:]), ref1["z_t"], rtol=1e-7, atol=1e-9)
        _, _, _, L1, _ = fol.get_belief()
        assert_close(f"scan{k} follower L", L1, ref1["belief"].L, rtol=1e-7, atol=1e-7 * np.abs(ref1["belief"].L).max())
        mref = map_fields(ref0["map"].stats)
        assert_close(f"scan{k} shared map", m0, mref, rtol=1e-7, atol=1e-9 * max(np.abs(mref).max(), 1.0))
        b0, b1, ms = ref0["belief"], ref1["belief"], ref0["map"]
    assert xi_diff > 1e-9  # the follower's own twist differs: the replay is not its own stage
    with pytest.raises(RuntimeError, match="FOLLOW"):
        lead.map_follow(lead.prepare_scan(rec, 16, t, w, n_raw, **kw), r)
    lead.close()
    fol.close()
