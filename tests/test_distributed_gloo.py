"""World-size-2 rehearsal (gloo, CPU) of the per-scan hypothesis all-reduce (gcslam.distributed).

The multi-GPU path shards one hypothesis per rank and exchanges one packed 840-f64 payload per
scan: process-noise IW sufficient statistics weighted by the raw
hypothesis weights (backend_node.py:1999-2002, 2085-2090) and the barycenter sums of
hypothesis_barycenter_projection weighted by the floor-renormalised weights (hypothesis.py:83-99,
spread :103-115).  Here two gloo ranks build the payload of their own hypothesis, all-reduce it
through gcslam.distributed.allreduce_payload (the function bench.py calls over RCCL), and the
decoded sums are checked against the oracle's barycenter on the same beliefs (the payload packing
below restates gcs_hypothesis_payload; the GPU suite checks the C packing against it).  A second
test runs the library's own context-free pack / apply (gcs_payload_pack / gcs_payload_apply) on
both ranks for three scans.  tests/test_gpu_distributed.py runs the same exchange between two
gcs_ctx on one GPU.
"""

import os
import socket

import numpy as np
import pytest

WORLD = 2
PAYLOAD_LEN = 840


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _beliefs(n):
    from oracle import ops
    rng = np.random.default_rng(7)
    out = []
    for k in range(n):
        A = rng.normal(size=(22, 22))
        L = A @ A.T + 22.0 * np.eye(22)
        out.append(ops.Belief(rng.normal(0, 0.05, 6), 1.0, rng.normal(0, 1e-3, 22), L, rng.normal(size=22)))
    return out


def _iw_stats(k):
    rng = np.random.default_rng(100 + k)
    return rng.normal(size=252), np.ones(7)


def pack_payload(b, dPsi, dnu, w_iw, w_bary, meas_dPsi=None, meas_dnu=None):
    """Layout of gcs_hypothesis_payload: [dPsi 252 | dnu 7 | meas dPsi 27 | meas dnu 3 | L 484 | h 22 |
    z_lin 22 | mu 22 | |mu|^2 1]."""
    p = np.zeros(PAYLOAD_LEN)
    p[0:252] = w_iw * dPsi
    p[252:259] = w_iw * dnu
    if meas_dPsi is not None:
        p[259:286] = w_iw * np.asarray(meas_dPsi).reshape(27)
        p[286:289] = w_iw * np.asarray(meas_dnu)
    mu = b.mean_increment()
    p[289:773] = w_bary * b.L.ravel()
    p[773:795] = w_bary * b.h
    p[795:817] = w_bary * b.z_lin
    p[817:839] = w_bary * mu
    p[839] = w_bary * float(mu @ mu)
    return p


def _worker(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gc-slam_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from gcslam.distributed import allreduce_payload, hypothesis_weights
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        w, wn = hypothesis_weights(WORLD)
        b = _beliefs(WORLD)[rank]
        dPsi, dnu = _iw_stats(rank)
        total = allreduce_payload(pack_payload(b, dPsi, dnu, float(w[rank]), float(wn[rank])))
        q.put((rank, total))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_payload_allreduce_matches_oracle_barycenter():
    import torch.multiprocessing as mp
    from oracle import ops
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank holds the same sums (bitwise): the combine that follows is identical on all ranks
    assert np.array_equal(got[0], got[1])
    tot = got[0]
    bs = _beliefs(WORLD)
    bary = ops.hypothesis_barycenter(np.stack([b.L for b in bs]), np.stack([b.h for b in bs]),
                                     np.stack([b.z_lin for b in bs]), np.full(WORLD, 1.0 / WORLD))
    np.testing.assert_allclose(tot[289:773].reshape(22, 22), bary["L_raw"], rtol=1e-14, atol=0)
    np.testing.assert_allclose(tot[773:795], bary["h"], rtol=1e-14, atol=1e-300)
    np.testing.assert_allclose(tot[795:817], bary["z_lin"], rtol=1e-14, atol=1e-300)
    mom = tot[817:839]
    spread = tot[839] - float(mom @ mom)   # sum w |mu|^2 - |sum w mu|^2 (hypothesis.py:110-115)
    assert spread == pytest.approx(bary["spread"], rel=1e-9, abs=1e-15)
    exp_dPsi = sum(_iw_stats(k)[0] for k in range(WORLD)) / WORLD
    np.testing.assert_allclose(tot[0:252], exp_dPsi, rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(tot[252:259], np.ones(7), rtol=1e-14)


def _lib_worker(rank, port, q):
    """One rank of the library-level exchange on CPU: gcs_payload_pack of this rank's hypothesis
    (belief, process and measurement IW statistics), gloo sum, gcs_payload_apply on the summed
    payload, three scans in a row with the IW states carried over (backend_node.py:2085-2119)."""
    import ctypes as C
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gc-slam_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from gcslam import _lib as L
    from gcslam.distributed import allreduce_payload, hypothesis_weights
    from oracle import ops
    lib = L.load()
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        w, wn = hypothesis_weights(WORLD)
        nu, Psi = (np.ascontiguousarray(a) for a in ops.datasheet_process_noise_state())
        mnu, mPsi = (np.ascontiguousarray(a) for a in ops.datasheet_measurement_noise_state())
        outs = []
        for s in range(3):
            b = _beliefs(WORLD + s)[rank + s]
            dPsi, dnu = _iw_stats(10 * s + rank)
            mdPsi = np.ascontiguousarray(np.stack([np.outer(v, v) for v in np.random.default_rng(s + 7 * rank)
                                                   .normal(0, 1e-3, (3, 3))]))
            mdnu = np.array([1.0, 1.0, 0.0])
            bs = L.belief_to_struct(b.X_anchor, b.stamp_sec, b.z_lin, b.L, b.h)
            p = np.zeros(840)
            assert lib.gcs_payload_pack(C.byref(bs), dPsi.ctypes.data, dnu.ctypes.data, mdPsi.ctypes.data,
                                        mdnu.ctypes.data, float(w[rank]), float(wn[rank]), p.ctypes.data) == 0
            tot = np.ascontiguousarray(allreduce_payload(p))
            comb = L.GcsBelief()
            nu2, Psi2, Q2, mnu2, mPsi2, c4 = (np.zeros(7), np.zeros(252), np.zeros(484), np.zeros(3), np.zeros(27),
                                              np.zeros(4))
            X0 = np.zeros(6)
            assert lib.gcs_payload_apply(tot.ctypes.data, s, X0.ctypes.data, 0.0, nu.ctypes.data, Psi.ctypes.data,
                                         mnu.ctypes.data, mPsi.ctypes.data, C.byref(comb), nu2.ctypes.data,
                                         Psi2.ctypes.data, Q2.ctypes.data, mnu2.ctypes.data, mPsi2.ctypes.data,
                                         c4.ctypes.data) == 0
            nu, Psi, mnu, mPsi = nu2, Psi2.reshape(7, 6, 6), mnu2, mPsi2.reshape(3, 3, 3)
            X, _, z, Lm, h = L.struct_to_arrays(comb)
            outs.append(dict(L=Lm, h=h, z=z, nu=nu.copy(), Psi=Psi.copy(), Q=Q2.reshape(22, 22), mnu=mnu.copy(),
                             mPsi=mPsi.copy(), dPsi=dPsi, mdPsi=mdPsi))
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_library_combine_matches_oracle():
    """The library's own payload pack / apply meet a second rank (gloo, CPU): both ranks end with
    bitwise-identical combined belief, process and measurement IW states and Q, equal to the
    oracle's 2-hypothesis node update (hypothesis.py:51-117; backend_node.py:2085-2119)."""
    import torch.multiprocessing as mp
    from oracle import ops, pipeline as opipe
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lib_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    iw = ops.datasheet_process_noise_state()
    meas = ops.datasheet_measurement_noise_state()
    for s in range(3):
        a, b = got[0][s], got[1][s]
        for k in a:
            assert np.array_equal(a[k], b[k]) or k in ("dPsi", "mdPsi"), k
        bs = _beliefs(WORLD + s)
        results = []
        for r in range(WORLD):
            dPsi, dnu = _iw_stats(10 * s + r)
            results.append(dict(belief=bs[r + s], iw_process_dPsi=dPsi.reshape(7, 6, 6), iw_process_dnu=dnu,
                                iw_meas_dPsi=got[r][s]["mdPsi"], iw_meas_dnu=np.array([1.0, 1.0, 0.0])))
        ref = opipe.combine_and_update_noise(results, np.full(WORLD, 1.0 / WORLD), iw, s, meas)
        iw, meas = ref["iw_state"], ref["meas_state"]
        Lr = ref["combined"]["L"]
        np.testing.assert_allclose(a["L"], Lr, rtol=1e-12, atol=1e-12 * np.abs(Lr).max())
        np.testing.assert_allclose(a["h"], ref["combined"]["h"], rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(a["nu"], iw[0], rtol=1e-14)
        np.testing.assert_allclose(a["Psi"], iw[1], rtol=1e-9, atol=1e-20)
        np.testing.assert_allclose(a["Q"], ref["Q"], rtol=1e-9, atol=1e-12 * np.abs(ref["Q"]).max())
        np.testing.assert_allclose(a["mPsi"], meas[1], rtol=1e-9, atol=1e-20)


def test_hypothesis_weights_floor():
    from gcslam.distributed import hypothesis_weights
    w, wn = hypothesis_weights(8)
    assert np.allclose(w, 1 / 8) and np.isclose(wn.sum(), 1.0)


def _record(rng, N, lobes, K):
    from types import SimpleNamespace
    import torch
    b = SimpleNamespace(Lambdas=torch.from_numpy(rng.normal(size=(N, 3, 3))), thetas=torch.from_numpy(rng.normal(size=(N, 3))),
                        etas=torch.from_numpy(rng.normal(size=(N, lobes, 3))), weights=torch.from_numpy(rng.random(N)),
                        valid_mask=torch.from_numpy(rng.random(N) < 0.7), colors=torch.from_numpy(rng.random((N, 3))),
                        sources=torch.from_numpy(rng.integers(0, 2, N).astype(np.int32)))
    a = SimpleNamespace(responsibilities=torch.from_numpy(rng.random((N, K))),
                        candidate_tile_ids=torch.from_numpy(rng.integers(-5, 10**12, (N, K))),
                        candidate_slots=torch.from_numpy(rng.integers(0, 50000, (N, K))),
                        row_masses=torch.from_numpy(rng.random(N)))
    return dict(active=[int(x) for x in rng.integers(-10**9, 10**9, 7)], scan_seq=int(rng.integers(0, 10**6)),
                t=float(rng.random() * 1e9), z_t=rng.normal(size=6), batch=b, association=a)


def _rec_worker(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gc-slam_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from gcslam.distributed import MapRecordChannel
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    N, lobes, K = 1536, 3, 8  # GC_VMF_N_LOBES = 3 (constants.py:463)
    ch = MapRecordChannel(N, lobes, K, device=-1)
    out = []
    for s in range(3):  # three scans: rank 0 (the lead) packs, everyone receives the same bytes
        rec = _record(np.random.default_rng(50 + s), N, lobes, K)
        if rank == 0:
            ch.pack(rec)
        ch.broadcast(root=0)
        got = ch.unpack()
        ok = (got["active"] == rec["active"] and got["scan_seq"] == rec["scan_seq"] and got["t"] == rec["t"]
              and np.array_equal(got["z_t"], rec["z_t"]))
        for grp in ("batch", "association"):
            for name, v in vars(rec[grp]).items():
                g = getattr(got[grp], name).numpy()
                ok = ok and np.array_equal(g.reshape(-1), v.numpy().reshape(-1)) and g.dtype == v.numpy().dtype
        out.append(bool(ok))
    q.put((rank, out, ch.nbytes))
    dist.destroy_process_group()


def test_gloo_world2_map_record_channel_bitwise():
    """gcslam.distributed.MapRecordChannel over gloo (the transport of ranks without an RCCL
    communicator of their own): the lead's live-map update record -- active tiles, scan seq / time,
    z_t, the MeasurementBatch and association fields step 12b reads -- reaches the other rank bit for
    bit, three scans in a row (backend_node.py:2079-2083); ~0.5 MB at the reference sizes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rec_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict((r, (o, n)) for r, o, n in (q.get(timeout=120) for _ in range(WORLD)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == [True] * 3 and got[1][0] == [True] * 3
    assert 0.4e6 < got[0][1] < 0.7e6
