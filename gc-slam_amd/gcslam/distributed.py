"""Hypothesis sharding: one hypothesis per GPU (one process per GPU), one all-reduce per scan.

The node-side accumulation of IW sufficient statistics (FS/backend/backend_node.py:1999-2002,
2085-2090) and the barycenter sums of hypothesis_barycenter_projection (hypothesis.py:92-115)
are both weighted sums over hypotheses, so they travel in one packed f64 payload
(GCS_PAYLOAD_LEN = 840, 6,720 B).  On GPUs the exchange lives in the library:
gcs_combine_allreduce packs the payload, runs ncclAllReduce (RCCL over xGMI) on the context stream
and applies the identical combine and IW update on every rank, so Q is bitwise identical
everywhere.  torch.distributed is only the launcher: it broadcasts the RCCL unique id.  A
torch.distributed transport (gloo) remains for ranks that share one device or have none (CPU
rehearsal, the two-ranks-on-one-GPU test); it moves the same library-packed payload.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

HYP_WEIGHT_FLOOR = 0.0025  # constants.py:63


_WEIGHTS = {}


def hypothesis_weights(n_hyp: int):
    """Uniform weights (backend_node.py:821-831) and their floor-renormalised form (hypothesis.py:83-87)."""
    if n_hyp not in _WEIGHTS:
        w = np.full(n_hyp, 1.0 / n_hyp)
        wf = np.maximum(w, HYP_WEIGHT_FLOOR)
        _WEIGHTS[n_hyp] = (w, wf / wf.sum())
    return _WEIGHTS[n_hyp]


class HypothesisComm:
    """RCCL communicator of the per-scan hypothesis exchange, one rank per GPU.  Rank 0 draws the
    unique id (gcs_rccl_get_unique_id); torch.distributed broadcasts it (the launcher's only job)."""

    def __init__(self, rank: int, world: int, device: int):
        import torch
        import torch.distributed as dist
        self.lib = L.load()
        uid = np.zeros(L.RCCL_ID_BYTES, np.uint8)
        if rank == 0:
            L.check(self.lib.gcs_rccl_get_unique_id(uid.ctypes.data), None, "gcs_rccl_get_unique_id")
        if world > 1:
            t = torch.from_numpy(uid.astype(np.int64))
            if dist.get_backend() == "nccl":
                t = t.to(f"cuda:{device}")
            dist.broadcast(t, src=0)
            uid = t.cpu().numpy().astype(np.uint8)
        h = C.c_void_p()
        L.check(self.lib.gcs_rccl_comm_init(int(device), int(world), int(rank), uid.ctypes.data, C.byref(h)), None,
                "gcs_rccl_comm_init")
        self.h = h
        self.rank, self.world = rank, world

    def count(self):
        """(ranks in the RCCL communicator, this rank's index in it): ncclCommCount / ncclCommUserRank."""
        n, r = C.c_int32(0), C.c_int32(0)
        L.check(self.lib.gcs_rccl_comm_count(self.h, C.byref(n), C.byref(r)), None, "gcs_rccl_comm_count")
        return int(n.value), int(r.value)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gcs_rccl_comm_destroy(self.h)
            self.h = None


def allreduce_payload(payload: np.ndarray, device=None) -> np.ndarray:
    """torch.distributed transport of a packed payload (gloo rehearsal / shared-device ranks).
    With a single rank the sum is the payload itself."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return payload
    import torch
    backend = dist.get_backend()
    dev = device if (device is not None and backend == "nccl") else "cpu"
    t = torch.from_numpy(np.ascontiguousarray(payload)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def combine_allreduce(ctx, rank: int, n_hyp: int, scan_count: int, comm: HypothesisComm | None = None, device=None,
                      want_belief=True):
    """The per-scan exchange of this rank's hypothesis.  With an RCCL communicator (or a single
    rank) everything runs in the library (gcs_combine_allreduce); otherwise the library-packed
    payload travels over torch.distributed and the library applies the sum."""
    w, wn = hypothesis_weights(n_hyp)
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if comm is not None or not distributed:
        return ctx.combine_allreduce(comm.h if comm is not None else None, float(w[rank]), float(wn[rank]),
                                     scan_count, want_belief=want_belief)
    payload = ctx.hypothesis_payload(float(w[rank]), float(wn[rank]))
    total = allreduce_payload(payload, device)
    return ctx.hypothesis_combine(total, scan_count, want_belief=want_belief)
