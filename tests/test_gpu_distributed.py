"""The multi-hypothesis exchange through the library on the GPU (SURVEY.md 8(e), C4 in miniature).

* Two ranks (processes, gloo transport) each hold a gcs_ctx on device 0 and run gcs_scan ->
  gcs_hypothesis_payload -> sum all-reduce -> gcs_hypothesis_combine for three scans with
  distinct priors.  Both ranks must end with bitwise-identical Q, process / measurement IW states
  and combined belief, and agree with the oracle's two-hypothesis node loop
  (backend_node.py:2036-2119, hypothesis.py:51-117).
* The RCCL path (gcs_rccl_comm_init + gcs_combine_allreduce) at world size 1 on the one GPU of the
  box: the communicator initialises, the all-reduce runs on the context stream, and the result
  equals the library's single-rank combine bitwise.  (RCCL refuses two ranks on one device; the
  8-GPU run is the driver's.)
"""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

WORLD = 2
ORIGIN = (0.0, 0.0, 0.5)
B, CAP, N_RAW = 48, 2048, 4096


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _prior(rank):
    rng = np.random.default_rng(1000 + rank)
    return np.concatenate([rng.normal(0, 0.05, 3) * (rank > 0), rng.normal(0, np.deg2rad(0.5), 3) * (rank > 0)])


def _rank(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gc-slam_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch as th
    import torch.distributed as dist
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    out = []
    try:
        ctx = HypothesisContext(n_bins=B, n_points_cap=CAP, max_raw_points=N_RAW, mode="dense", lidar_origin=ORIGIN)
        ctx.set_belief(_prior(rank), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
        for s in range(3):
            sc = synthetic.make_scan(N_RAW, 80 + s)
            rec = th.from_numpy(sc["xyz_record"]).cuda()
            t = th.from_numpy(sc["timestamps"]).cuda()
            w = th.from_numpy(sc["weights"]).cuda()
            o = ctx.scan(rec, 16, t, w, N_RAW, **synthetic.scan_kwargs(sc))
            (X, _, z, Lm, h), cert = combine_allreduce(ctx, rank, WORLD, s)
            nu, Psi, Q = ctx.iw_state()
            mnu, mPsi, _ = ctx.meas_iw_state()
            out.append(dict(z_t=np.array(o.z_t[:]), L=Lm, h=h, z=z, nu=nu, Psi=Psi, Q=Q, mnu=mnu, mPsi=mPsi))
        ctx.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_library_combine_matches_oracle():
    import torch.multiprocessing as mp
    from gcslam import synthetic
    from oracle import ops, pipeline as opipe
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the oracle's node loop with two hypotheses (per-hypothesis maps, declared)
    bins = ops.fibonacci_atlas(B)
    cfg = opipe.BinPathConfig(n_points_cap=CAP, n_bins=B, mode="dense", lidar_origin=ORIGIN, tau=ops.tau_for_bins(B))
    hyps = []
    for r in range(WORLD):
        b = ops.Belief.identity_prior()
        b.X_anchor = _prior(r)
        hyps.append(b)
    maps = [opipe.MapState.empty(B) for _ in range(WORLD)]
    iw, meas = ops.datasheet_process_noise_state(), ops.datasheet_measurement_noise_state()
    Q = ops.process_noise_Q(*iw)
    for s in range(3):
        a, b = got[0][s], got[1][s]
        for k in ("L", "h", "z", "nu", "Psi", "Q", "mnu", "mPsi"):
            assert np.array_equal(a[k], b[k]), k            # identical combine + IW update on every rank
        sc = synthetic.make_scan(N_RAW, 80 + s)
        res = [opipe.process_scan_bin_path(hyps[r], sc, Q, cfg, bins, None, maps[r], meas_state=meas)
               for r in range(WORLD)]
        for r in range(WORLD):
            np.testing.assert_allclose(got[r][s]["z_t"], res[r]["z_t"], rtol=1e-7, atol=1e-9)
        c = opipe.combine_and_update_noise(res, np.full(WORLD, 1.0 / WORLD), iw, s, meas)
        Lr = c["combined"]["L"]
        np.testing.assert_allclose(a["L"], Lr, rtol=1e-6, atol=1e-9 * np.abs(Lr).max())
        np.testing.assert_allclose(a["z"], c["combined"]["z_lin"], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(a["nu"], c["iw_state"][0], rtol=1e-12)
        np.testing.assert_allclose(a["Q"], c["Q"], rtol=1e-6, atol=1e-9 * np.abs(c["Q"]).max())
        np.testing.assert_allclose(a["mPsi"], c["meas_state"][1], rtol=1e-6, atol=1e-18)
        Q, iw, meas = c["Q"], c["iw_state"], c["meas_state"]
        hyps = [res[r]["belief"] for r in range(WORLD)]
        maps = [res[r]["map"] for r in range(WORLD)]


def test_rccl_combine_world1_matches_single_rank():
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import HypothesisComm, combine_allreduce
    comm = HypothesisComm(0, 1, 0)
    outs = []
    try:
        for use_comm in (True, False):
            ctx = HypothesisContext(n_bins=B, n_points_cap=CAP, max_raw_points=N_RAW, mode="dense",
                                    lidar_origin=ORIGIN)
            for s in range(2):
                sc = synthetic.make_scan(N_RAW, 90 + s)
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                ctx.scan(rec, 16, t, w, N_RAW, **synthetic.scan_kwargs(sc))
                (X, _, z, Lm, h), cert = combine_allreduce(ctx, 0, 1, s, comm=comm if use_comm else None)
            outs.append((Lm, h, z, *ctx.iw_state(), *ctx.meas_iw_state()[:2]))
            ctx.close()
    finally:
        comm.close()
    for x, y in zip(*outs):
        assert np.array_equal(x, y)



def _rccl_sequence(n_scans, comm=None):
    """n_scans dense scans with the combine after each (through `comm` when given), the final state."""
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    ctx = HypothesisContext(n_bins=B, n_points_cap=CAP, max_raw_points=N_RAW, mode="dense", lidar_origin=ORIGIN)
    try:
        for s in range(n_scans):
            sc = synthetic.make_scan(N_RAW, 90 + s)
            rec = torch.from_numpy(sc["xyz_record"]).cuda()
            t = torch.from_numpy(sc["timestamps"]).cuda()
            w = torch.from_numpy(sc["weights"]).cuda()
            ctx.scan(rec, 16, t, w, N_RAW, **synthetic.scan_kwargs(sc))
            (X, _, z, Lm, h), cert = combine_allreduce(ctx, 0, 1, s, comm=comm)
        return (Lm, h, z, *ctx.iw_state(), *ctx.meas_iw_state()[:2]), ctx.mirror_stats()
    finally:
        ctx.close()


def test_rccl_stamped_sum_over_a_sequence():
    """Five scans with the combine through a world-1 RCCL communicator (ncclAllReduce from the pinned
    payload on the combine stream, the sum stamped back with sequence + checksum) give the host-only
    combine's state bit for bit; every all-reduce's sum is accepted by the host poll (none through the
    stream-synchronize fallback)."""
    from gcslam.distributed import HypothesisComm
    ref, _ = _rccl_sequence(5)
    comm = HypothesisComm(0, 1, 0)
    try:
        got, st = _rccl_sequence(5, comm=comm)
    finally:
        comm.close()
    for x, y in zip(ref, got):
        assert np.array_equal(x, y)
    assert st[3] == 5 and st[5] == 0, st
