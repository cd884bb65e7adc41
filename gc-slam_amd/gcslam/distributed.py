"""Hypothesis sharding: one hypothesis per GPU (one process per GPU), one RCCL all-reduce per scan.

The node-side accumulation of IW sufficient statistics (FS/backend/backend_node.py:1999-2002,
2085-2090) and the barycenter sums of hypothesis_barycenter_projection (hypothesis.py:92-115)
are both weighted sums over hypotheses, so they travel in one packed f64 payload
(GCS_PAYLOAD_LEN = 840, 6,720 B) reduced with torch.distributed (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" for the CPU tests).  Every rank then applies the identical combine and
IW update, so Q is bitwise identical on every rank for the next scan.
"""

from __future__ import annotations

import numpy as np

HYP_WEIGHT_FLOOR = 0.0025  # constants.py:63


_WEIGHTS = {}


def hypothesis_weights(n_hyp: int):
    """Uniform weights (backend_node.py:821-831) and their floor-renormalised form (hypothesis.py:83-87)."""
    if n_hyp not in _WEIGHTS:
        w = np.full(n_hyp, 1.0 / n_hyp)
        wf = np.maximum(w, HYP_WEIGHT_FLOOR)
        _WEIGHTS[n_hyp] = (w, wf / wf.sum())
    return _WEIGHTS[n_hyp]


def allreduce_payload(payload: np.ndarray, device=None) -> np.ndarray:
    """Sum-all-reduce the packed payload across ranks (RCCL on GPU, gloo on CPU).  With a single
    rank the sum is the payload itself (returned as is)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return payload
    import torch
    backend = dist.get_backend()
    dev = device if (device is not None and backend == "nccl") else "cpu"
    t = torch.from_numpy(np.ascontiguousarray(payload)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def combine_allreduce(ctx, rank: int, n_hyp: int, scan_count: int, device=None, want_belief=True):
    """Pack this rank's hypothesis, all-reduce, apply the combine + IW update on every rank."""
    w, wn = hypothesis_weights(n_hyp)
    payload = ctx.hypothesis_payload(float(w[rank]), float(wn[rank]))
    total = allreduce_payload(payload, device)
    return ctx.hypothesis_combine(total, scan_count, want_belief=want_belief)
