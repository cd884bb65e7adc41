"""BASELINE.json configs[3] (C4) on one GPU: eight hypotheses at the C2 size (65,536 points x 100,000
bins, scale mode), one gcs_ctx each, through the library's exchange -- gcs_scan per hypothesis, the
library-packed payload (gcs_hypothesis_payload), their sum, and gcs_hypothesis_combine on every
context (the summed payload -> barycenter, process / measurement IW applies, Q) -- over two scans,
against the oracle's eight-hypothesis node loop (backend_node.py:2036-2119, hypothesis.py:51-117).

On the 8-GPU node each context is one rank and the sum is gcs_combine_allreduce's ncclAllReduce; here
the eight payloads are summed in rank order on the host (the all-reduce's order may differ, so the
oracle comparison carries tolerances, while every context must hold bitwise the same combined state).
The second test runs the exchange's device send-buffer path (GCS_DEBUG_SENDBUF: the world > 1 form)
through a world-1 RCCL communicator and requires the host-buffer path's state bit for bit.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from gpu_util import assert_close
from oracle import ops, pipeline as opipe

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)
N, B, K_HYP = 65536, 100000, 8


def _prior(rank):
    rng = np.random.default_rng(1000 + rank)
    return np.concatenate([rng.normal(0, 0.05, 3) * (rank > 0), rng.normal(0, np.deg2rad(0.5), 3) * (rank > 0)])


def test_c4_eight_hypotheses_c2_size_match_oracle_node_loop():
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import hypothesis_weights
    from gcslam.synthetic import scan_kwargs
    ctxs = [HypothesisContext(n_bins=B, n_points_cap=N, max_raw_points=N, mode="scale", k_cand=16,
                              lidar_origin=ORIGIN) for _ in range(K_HYP)]
    try:
        dirs, knn = ctxs[0].atlas()
        w, wn = hypothesis_weights(K_HYP)
        for r, c in enumerate(ctxs):
            c.set_belief(_prior(r), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
        cfg = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", lidar_origin=ORIGIN, tau=ctxs[0].cfg.tau)
        hyps = []
        for r in range(K_HYP):
            b = ops.Belief.identity_prior()
            b.X_anchor = _prior(r)
            b.L = 1e-6 * np.eye(22)
            hyps.append(b)
        maps = [opipe.MapState.empty(B) for _ in range(K_HYP)]
        iw, meas = ops.datasheet_process_noise_state(), ops.datasheet_measurement_noise_state()
        Q = ops.process_noise_Q(*iw)
        for s in range(2):
            sc = synthetic.make_scan(N, 200 + s)
            rec = torch.from_numpy(np.ascontiguousarray(sc["xyz_record"])).cuda()
            t = torch.from_numpy(np.ascontiguousarray(sc["timestamps"])).cuda()
            wt = torch.from_numpy(np.ascontiguousarray(sc["weights"])).cuda()
            zt, pay = [], []
            for r, c in enumerate(ctxs):
                o = c.scan(rec, 16, t, wt, N, **scan_kwargs(sc))
                zt.append(np.array(o.z_t[:]))
                pay.append(c.hypothesis_payload(float(w[r]), float(wn[r])))
            total = pay[0].copy()
            for p in pay[1:]:
                total = total + p
            got = []
            for c in ctxs:
                (X, _, z, Lm, h), cert = c.hypothesis_combine(total, s)
                nu, Psi, Qd = c.iw_state()
                mnu, mPsi, _ = c.meas_iw_state()
                got.append(dict(L=Lm, h=h, z=z, nu=nu, Psi=Psi, Q=Qd, mnu=mnu, mPsi=mPsi))
            for g in got[1:]:  # one summed payload -> the same combine and IW update in every context
                for k in got[0]:
                    assert np.array_equal(g[k], got[0][k]), k
            res = [opipe.process_scan_bin_path(hyps[r], sc, Q, cfg, dirs, knn, maps[r], meas_state=meas)
                   for r in range(K_HYP)]
            for r in range(K_HYP):
                assert_close(f"C4 scan{s} hyp{r} z_t", zt[r], res[r]["z_t"], rtol=1e-7, atol=1e-9)
            c4 = opipe.combine_and_update_noise(res, np.full(K_HYP, 1.0 / K_HYP), iw, s, meas)
            a = got[0]
            Lr = c4["combined"]["L"]
            assert_close(f"C4 scan{s} combined L", a["L"], Lr, rtol=1e-6, atol=1e-9 * np.abs(Lr).max())
            assert_close(f"C4 scan{s} combined z_lin", a["z"], c4["combined"]["z_lin"], rtol=1e-6, atol=1e-9)
            assert_close(f"C4 scan{s} IW nu", a["nu"], c4["iw_state"][0], rtol=1e-12, atol=0.0)
            assert_close(f"C4 scan{s} Q", a["Q"], c4["Q"], rtol=1e-6, atol=1e-9 * np.abs(c4["Q"]).max())
            assert_close(f"C4 scan{s} meas Psi", a["mPsi"], c4["meas_state"][1], rtol=1e-6, atol=1e-18)
            Q, iw, meas = c4["Q"], c4["iw_state"], c4["meas_state"]
            hyps = [res[r]["belief"] for r in range(K_HYP)]
            maps = [res[r]["map"] for r in range(K_HYP)]
    finally:
        for c in ctxs:
            c.close()


def test_device_sendbuf_allreduce_matches_host_buffer():
    """gcs_combine_allreduce with the send buffer in device memory (the copy-engine stage-in that ranks
    > 1 take, forced at world size 1 by GCS_DEBUG_SENDBUF) over four scans: bitwise the state of the
    pinned-host-buffer form, every sum accepted by the host poll."""
    from gcslam import _lib as L, synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import HypothesisComm, combine_allreduce
    comm = HypothesisComm(0, 1, 0)
    outs = []
    try:
        for mode in (0, 1):
            ctx = HypothesisContext(n_bins=48, n_points_cap=2048, max_raw_points=4096, mode="dense",
                                    lidar_origin=ORIGIN)
            ctx.set_debug(L.DEBUG_SENDBUF, mode)
            for s in range(4):
                sc = synthetic.make_scan(4096, 90 + s)
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                ctx.scan(rec, 16, t, w, 4096, **synthetic.scan_kwargs(sc))
                (X, _, z, Lm, h), cert = combine_allreduce(ctx, 0, 1, s, comm=comm)
            st = ctx.mirror_stats()
            assert st[3] == 4 and st[5] == 0, st
            outs.append((Lm, h, z, *ctx.iw_state(), *ctx.meas_iw_state()[:2]))
            ctx.close()
    finally:
        comm.close()
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
    with pytest.raises(ValueError):
        ctx2 = HypothesisContext(n_bins=48, n_points_cap=2048, max_raw_points=4096, mode="dense", lidar_origin=ORIGIN)
        try:
            ctx2.set_debug(L.DEBUG_SENDBUF, 2)
        finally:
            ctx2.close()


def test_straggling_peer_takes_the_synchronize_path_same_state():
    """A peer that reaches the all-reduce late (GCS_DEBUG_COMBINE_DELAY: a 30 ms wait queued on the combine
    stream ahead of ncclAllReduce, the world-1 stand-in for a straggling rank) outlasts the host poll's
    20 ms: the wait falls to its stream synchronize, which returns once the collective is done, and the
    sum is checked as on the poll path.  Over four scans with the delay on scans 1 and 3: bitwise the
    undelayed state, exactly two payload syncs, and each delayed combine takes at least the delay."""
    import time
    from gcslam import _lib as L, synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import HypothesisComm, combine_allreduce
    comm = HypothesisComm(0, 1, 0)
    outs, waits = [], []
    try:
        for delayed in (False, True):
            ctx = HypothesisContext(n_bins=48, n_points_cap=2048, max_raw_points=4096, mode="dense",
                                    lidar_origin=ORIGIN)
            ctx.set_debug(L.DEBUG_SENDBUF, 1)  # the world > 1 form of the exchange
            for s in range(4):
                sc = synthetic.make_scan(4096, 90 + s)
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                ctx.scan(rec, 16, t, w, 4096, **synthetic.scan_kwargs(sc))
                ctx.set_debug(L.DEBUG_COMBINE_DELAY, 30000 if delayed and s % 2 else 0)
                t0 = time.perf_counter()
                (X, _, z, Lm, h), cert = combine_allreduce(ctx, 0, 1, s, comm=comm)
                if delayed and s % 2:
                    waits.append(time.perf_counter() - t0)
            st = ctx.mirror_stats()
            assert st[3] == 4 and st[5] == (2 if delayed else 0), st
            outs.append((Lm, h, z, *ctx.iw_state(), *ctx.meas_iw_state()[:2]))
            ctx.close()
    finally:
        comm.close()
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
    assert min(waits) >= 0.030, waits
    print("straggler combine s:", [round(x, 4) for x in waits])
