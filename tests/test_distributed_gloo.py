"""World-size-2 rehearsal (gloo, CPU) of the per-scan hypothesis all-reduce (gcslam.distributed).

The multi-GPU path shards one hypothesis per rank and exchanges one packed 840-f64 payload per
scan: process-noise IW sufficient statistics weighted by the raw
hypothesis weights (backend_node.py:1999-2002, 2085-2090) and the barycenter sums of
hypothesis_barycenter_projection weighted by the floor-renormalised weights (hypothesis.py:83-99,
spread :103-115).  Here two gloo ranks build the payload of their own hypothesis, all-reduce it
through gcslam.distributed.allreduce_payload (the function bench.py calls over RCCL), and the
decoded sums are checked against the oracle's barycenter on the same beliefs.  The payload packing
below restates gcs_hypothesis_payload (gcs_capi.cpp); the GPU suite checks the C packing against it.
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
    # IW statistics: raw weights 1/H (backend_node.py:2086-2090)
    exp_dPsi = sum(_iw_stats(k)[0] for k in range(WORLD)) / WORLD
    np.testing.assert_allclose(tot[0:252], exp_dPsi, rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(tot[252:259], np.ones(7), rtol=1e-14)
    assert not np.any(tot[259:289])   # measurement-noise IW slots (out of scope this round)


def test_hypothesis_weights_floor():
    from gcslam.distributed import hypothesis_weights
    w, wn = hypothesis_weights(8)
    assert np.allclose(w, 1 / 8) and np.isclose(wn.sum(), 1.0)
