#!/usr/bin/env python3
"""World-2 RCCL exchange on one GPU: two ranks, both on device 0, each one hypothesis context, run a
3-scan sequence twice, with the library's combine over a world-2 RCCL communicator (the device send
buffer, ncclAllReduce across ranks, the stamped return) and over gloo (the library-packed payload
summed by torch.distributed). Each rank checks that the two give the same state, bit for bit, and
that every RCCL sum was taken by the host poll. Two addends sum the same in either order, so the
results must match exactly. This is the N > 1 path the driver's 8-GPU run takes, minus the xGMI
links. If RCCL refuses two ranks on one device, the probe says so and exits 3.

    python tools/rccl_world2.py
"""

import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD, B, CAP, N_RAW = 2, 48, 2048, 4096
ORIGIN = (0.0, 0.0, 0.5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _prior(rank):
    rng = np.random.default_rng(1000 + rank)
    return np.concatenate([rng.normal(0, 0.05, 3) * (rank > 0), rng.normal(0, np.deg2rad(0.5), 3) * (rank > 0)])


def _sequence(rank, comm):
    import torch
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    ctx = HypothesisContext(n_bins=B, n_points_cap=CAP, max_raw_points=N_RAW, mode="dense", lidar_origin=ORIGIN)
    try:
        ctx.set_belief(_prior(rank), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
        out = []
        for s in range(3):
            sc = synthetic.make_scan(N_RAW, 80 + s)
            rec = torch.from_numpy(sc["xyz_record"]).cuda()
            t = torch.from_numpy(sc["timestamps"]).cuda()
            w = torch.from_numpy(sc["weights"]).cuda()
            ctx.scan(rec, 16, t, w, N_RAW, **synthetic.scan_kwargs(sc))
            (X, _, z, Lm, h), _ = combine_allreduce(ctx, rank, WORLD, s, comm=comm)
            nu, Psi, Q = ctx.iw_state()
            out.append((Lm, h, z, nu, Psi, Q))
        return out, ctx.mirror_stats()
    finally:
        ctx.close()


def _rank(rank, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from gcslam.distributed import HypothesisComm
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ref, _ = _sequence(rank, None)
        try:
            comm = HypothesisComm(rank, WORLD, 0)
        except Exception as e:  # noqa: BLE001 -- reported, not raised: the probe's answer
            q.put((rank, "refused", repr(e)))
            return
        try:
            n, r = comm.count()
            got, st = _sequence(rank, comm)
        finally:
            comm.close()
        same = all(all(np.array_equal(a, b) for a, b in zip(x, y)) for x, y in zip(ref, got))
        q.put((rank, "ok", dict(comm_count=n, comm_rank=r, bitwise_equal=bool(same), payloads=int(st[3]),
                                payload_syncs=int(st[5]), payload_rereads=int(st[4]))))
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
    for r in res:
        print(r, flush=True)
    if any(r[1] == "refused" for r in res):
        sys.exit(3)
    ok = all(r[1] == "ok" and r[2]["bitwise_equal"] and r[2]["comm_count"] == WORLD and r[2]["payloads"] == 3
             for r in res)
    print("world-2 RCCL vs gloo:", "bitwise equal" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
