"""PointCloud2 parse on the GPU: parse_pointcloud2_vlp16
(FS/backend/backend_node.py:377-468) plus the no-TF base transform (:1677-1680), through
gcs_parse_pointcloud2.  The message bytes go to the device once; points, times, weights and ring
come back as device tensors ready for HypothesisContext.scan(..., xyz_f64=True, point_step=24)."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L

POINTFIELD = dict(INT8=1, UINT8=2, INT16=3, UINT16=4, INT32=5, UINT32=6, FLOAT32=7, FLOAT64=8)


@dataclass
class PointFieldLike:
    name: str
    offset: int
    datatype: int
    count: int = 1


@dataclass
class PointCloud2Like:
    """The sensor_msgs/PointCloud2 members the parse reads (a ROS message works as is)."""
    data: object                 # bytes / np.uint8 array / torch uint8 tensor (host or device)
    fields: list
    point_step: int
    width: int
    height: int = 1
    stamp_sec: float = 0.0
    header: Optional[object] = None


def _stamp(msg):
    h = getattr(msg, "header", None)
    if h is not None and hasattr(h, "stamp"):
        return h.stamp.sec + h.stamp.nanosec * 1e-9
    return float(getattr(msg, "stamp_sec", 0.0))


def parse_pointcloud2_vlp16(msg, ctx, R_base_lidar=None, t_base_lidar=None):
    """Returns (points (n,3) f64 base frame, t (n,), w (n,), ring (n,) u8, tag (n,) u8) as device
    tensors on the context's GPU.  Raises RuntimeError on a missing x/y/z/ring field, like the
    reference."""
    import torch
    dev = f"cuda:{ctx.device}"
    n = int(msg.width) * int(msg.height)
    fmap = {f.name: (int(f.offset), int(f.datatype)) for f in msg.fields}
    missing = [k for k in ("x", "y", "z", "ring") if k not in fmap]
    if missing:
        raise RuntimeError(f"PointCloud2 (VLP-16 layout) missing required fields: {missing}. "
                           f"Present fields: {sorted(fmap)}")
    tf = "t" if "t" in fmap else ("time" if "time" in fmap else None)
    lay = L.GcsPointCloud2Layout()
    lay.n_points, lay.point_step = n, int(msg.point_step)
    lay.off_x, lay.off_y, lay.off_z = fmap["x"][0], fmap["y"][0], fmap["z"][0]
    lay.off_ring, lay.ring_datatype = fmap["ring"]
    lay.off_t, lay.t_datatype = fmap[tf] if tf else (-1, 0)
    lay.header_stamp_sec = _stamp(msg)
    R = np.eye(3) if R_base_lidar is None else np.asarray(R_base_lidar, np.float64)
    tb = np.zeros(3) if t_base_lidar is None else np.asarray(t_base_lidar, np.float64)
    lay.R_base_lidar[:] = R.reshape(9).tolist()
    lay.t_base_lidar[:] = tb.reshape(3).tolist()
    data = msg.data
    if not isinstance(data, torch.Tensor):
        data = torch.from_numpy(np.frombuffer(bytes(data) if not isinstance(data, np.ndarray) else data.tobytes(),
                                              np.uint8).copy())
    data = data.to(dev).contiguous()
    pts = torch.empty((n, 3), dtype=torch.float64, device=dev)
    t = torch.empty(n, dtype=torch.float64, device=dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    ring = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.current_stream(dev).synchronize()  # the copy above ran on torch's stream
    ctx._chk(ctx.lib.gcs_parse_pointcloud2(ctx.h, data.data_ptr(), C.byref(lay), pts.data_ptr(), t.data_ptr(),
                                          w.data_ptr(), ring.data_ptr()), "parse_pointcloud2")
    ctx.synchronize()
    return pts, t, w, ring, torch.zeros(n, dtype=torch.uint8, device=dev)
