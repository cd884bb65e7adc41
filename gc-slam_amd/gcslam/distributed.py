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


class MapRecordChannel:
    """The live primitive map across ranks: the lead's per-scan update record (result.map_record --
    active tiles, scan seq / time, z_t, the MeasurementBatch and the association result, the inputs of
    its recency inflation and step 12b) packed into one device buffer and broadcast to the other ranks,
    which replay it on their copy of the node map (gcslam.pipeline.primitive_map_follow): the
    reference's one map over all hypotheses, hypothesis 0's (backend_node.py:2036-2083), with no map
    rows crossing xGMI.  ~0.5 MB at the reference sizes (1,536 rows, k_assoc 8).

    Transport: RCCL (gcs_rccl_broadcast on the current stream) with a HypothesisComm, else
    torch.distributed (gloo: the CPU-staged copy, for ranks sharing one device or the rehearsal)."""

    _B = (("Lambdas", "f8", (9,)), ("thetas", "f8", (3,)), ("etas", "f8", None), ("weights", "f8", ()),
          ("valid_mask", "u1", ()), ("colors", "f8", (3,)), ("sources", "i4", ()))
    _A = (("responsibilities", "f8", "K"), ("candidate_tile_ids", "i8", "K"), ("candidate_slots", "i8", "K"),
          ("row_masses", "f8", ()))
    HDR = 96          # int64 header words
    MAX_ACTIVE = 64
    MAGIC = 0x6763736d72656331

    def __init__(self, n_total: int, n_lobes: int, k_assoc: int, device: int, comm: "HypothesisComm | None" = None):
        import torch
        self.N, self.lobes, self.K, self.device, self.comm = int(n_total), int(n_lobes), int(k_assoc), int(device), comm
        self.layout, off = [], self.HDR * 8
        for group, fields in (("batch", self._B), ("association", self._A)):
            for name, dt, tail in fields:
                shape = (self.N,) + ((self.lobes, 3) if tail is None else ((self.K,) if tail == "K" else tuple(tail)))
                n = int(np.prod(shape)) * np.dtype(dt).itemsize
                self.layout.append((group, name, dt, shape, off, n))
                off += (n + 7) // 8 * 8
        self.nbytes = off
        # device < 0: a host buffer (the CPU rehearsal of the transport)
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=f"cuda:{self.device}" if self.device >= 0 else "cpu")
        self._torch = {"f8": torch.float64, "i8": torch.int64, "i4": torch.int32, "u1": torch.uint8}

    def pack(self, record: dict):
        """Fill the buffer with `record` (the lead's result.map_record)."""
        import torch
        act = [int(x) for x in record["active"]]
        if len(act) > self.MAX_ACTIVE:
            raise ValueError(f"map record: {len(act)} active tiles > {self.MAX_ACTIVE}")
        hdr = np.zeros(self.HDR, np.int64)
        hdr[:6] = [self.MAGIC, self.N, self.K, self.lobes, len(act), int(record["scan_seq"])]
        hdr[6] = np.float64(record["t"]).view(np.int64)
        hdr[7:13] = np.asarray(record["z_t"], np.float64).reshape(6).view(np.int64)
        hdr[16:16 + len(act)] = act
        self.buf[:self.HDR * 8].copy_(torch.from_numpy(hdr.view(np.uint8)), non_blocking=False)
        for group, name, dt, shape, off, n in self.layout:
            src = getattr(record[group], name)
            t = torch.as_tensor(src, device=self.buf.device).to(self._torch[dt]).reshape(shape)
            self.buf[off:off + n].copy_(t.contiguous().view(torch.uint8).reshape(-1))

    def broadcast(self, root: int = 0):
        import torch
        if self.comm is not None:
            from . import _lib as L
            s = torch.cuda.current_stream(self.buf.device).cuda_stream
            L.check(L.load().gcs_rccl_broadcast(self.comm.h, self.buf.data_ptr(), self.nbytes, int(root), s), None,
                    "gcs_rccl_broadcast")
            return
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            host = self.buf.cpu() if self.buf.is_cuda else self.buf
            dist.broadcast(host, src=root)
            if host is not self.buf:
                self.buf.copy_(host)

    def unpack(self) -> dict:
        """The record in the buffer, in the form primitive_map_follow takes (device tensor views)."""
        from types import SimpleNamespace
        hdr = self.buf[:self.HDR * 8].cpu().numpy().view(np.int64)
        if int(hdr[0]) != self.MAGIC or int(hdr[1]) != self.N or int(hdr[2]) != self.K:
            raise RuntimeError("map record: bad header (no record packed, or a layout mismatch between ranks)")
        groups = {"batch": {}, "association": {}}
        for group, name, dt, shape, off, n in self.layout:
            groups[group][name] = self.buf[off:off + n].view(self._torch[dt]).reshape(shape)
        groups["batch"]["valid_mask"] = groups["batch"]["valid_mask"].to(bool)
        n_act = int(hdr[4])
        return dict(active=[int(x) for x in hdr[16:16 + n_act]], scan_seq=int(hdr[5]),
                    t=float(hdr[6:7].view(np.float64)[0]), z_t=hdr[7:13].view(np.float64).copy(),
                    batch=SimpleNamespace(**groups["batch"]), association=SimpleNamespace(**groups["association"]))
