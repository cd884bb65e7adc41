"""The live primitive path's LiDAR surfel extraction on the MI355X:
extract_lidar_surfels with the reference's calling convention
(FS/backend/operators/lidar_surfel_extraction.py:339-431 -> (MeasurementBatch, CertBundle,
ExpectedEffect)), running gcs_extract_lidar_surfels (libgcslam_hip.so).  The MeasurementBatch mirrors
FS/backend/structures/measurement_batch.py:68-135 with device (torch) arrays; the camera slice of a
lidar-only batch is empty, a camera base_batch keeps its slice."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, fields, replace
from typing import Optional

import numpy as np

from . import _lib as L
from .certificates import CertBundle, ExpectedEffect, InfluenceCert, SupportCert

CHART_ID = "GC-RIGHT-01"
GC_N_SURFEL = 1024   # constants.py:353
GC_N_FEAT = 512      # constants.py:350
GC_VMF_N_LOBES = 3   # constants.py:463


@dataclass
class SurfelExtractionConfig:
    """lidar_surfel_extraction.py:43-62 (same fields and defaults)."""
    n_surfel: int = GC_N_SURFEL
    n_feat: int = GC_N_FEAT
    voxel_size_m: float = 0.1
    hex3d_num_cells_1: int = 32
    hex3d_num_cells_2: int = 32
    hex3d_num_cells_z: int = 8
    hex3d_max_occupants: int = 32
    min_points_per_voxel: int = 3
    sensor_noise_var_per_axis: float = 1e-6
    wishart_nu: float = 5.0
    wishart_psi_scale: float = 0.1
    kappa_main_scale: float = 10.0
    kappa_min: float = 0.1
    kappa_max: float = 100.0
    eig_min: float = 1e-12
    eps_lift: float = 1e-9

    @property
    def n_cells(self):
        return int(self.hex3d_num_cells_1 * self.hex3d_num_cells_2 * self.hex3d_num_cells_z)


@dataclass
class MeasurementBatch:
    """measurement_batch.py:68-135: camera splats at [0, n_feat), LiDAR surfels at [n_feat, n_total)."""
    Lambdas: object        # (n_total, 3, 3)
    thetas: object         # (n_total, 3)
    etas: object           # (n_total, B, 3)
    weights: object        # (n_total,)
    sources: object        # (n_total,) 0 camera, 1 lidar
    source_indices: object
    valid_mask: object
    timestamps: object
    colors: object         # (n_total, 3)
    n_feat: int
    n_surfel: int
    n_camera_valid: int
    n_lidar_valid: int

    @property
    def n_total(self) -> int:
        return self.n_feat + self.n_surfel

    @property
    def n_valid(self) -> int:
        return self.n_camera_valid + self.n_lidar_valid

    @property
    def camera_slice(self) -> slice:
        return slice(0, self.n_feat)

    @property
    def lidar_slice(self) -> slice:
        return slice(self.n_feat, self.n_total)


def _torch():
    import torch
    return torch


def create_empty_measurement_batch(n_feat=GC_N_FEAT, n_surfel=GC_N_SURFEL, device="cuda:0"):
    """measurement_batch.py:137-157 (device arrays): one zeroed allocation carved into the nine arrays
    (one fill kernel, not nine)."""
    torch = _torch()
    nt = n_feat + n_surfel
    spec = (("Lambdas", torch.float64, (nt, 3, 3)), ("thetas", torch.float64, (nt, 3)),
            ("etas", torch.float64, (nt, GC_VMF_N_LOBES, 3)), ("weights", torch.float64, (nt,)),
            ("timestamps", torch.float64, (nt,)), ("colors", torch.float64, (nt, 3)),
            ("sources", torch.int32, (nt,)), ("source_indices", torch.int32, (nt,)), ("valid_mask", torch.bool, (nt,)))
    size = {torch.float64: 8, torch.int32: 4, torch.bool: 1}
    nbytes = [int(np.prod(sh)) * size[dt] for _, dt, sh in spec]
    buf = torch.zeros(sum((z + 7) // 8 * 8 for z in nbytes), dtype=torch.uint8, device=device)
    t, off = {}, 0
    for (name, dt, sh), z in zip(spec, nbytes):
        t[name] = buf[off:off + z].view(dt).view(sh)
        off += (z + 7) // 8 * 8
    return MeasurementBatch(**t, n_feat=n_feat, n_surfel=n_surfel, n_camera_valid=0, n_lidar_valid=0)


class SurfelExtractor:
    """A gcs_surfel_ctx: workspace for up to max_points points on one GPU."""

    def __init__(self, config: Optional[SurfelExtractionConfig] = None, max_points: int = 65536, device: int = 0):
        self.config = config or SurfelExtractionConfig()
        self.lib = L.load()
        c = L.GcsSurfelConfig()
        L.check(self.lib.gcs_surfel_config_defaults(C.byref(c)), None, "gcs_surfel_config_defaults")
        cf = self.config
        c.n_surfel, c.n_feat, c.voxel_size_m = int(cf.n_surfel), int(cf.n_feat), float(cf.voxel_size_m)
        c.num_cells_1, c.num_cells_2, c.num_cells_z = cf.hex3d_num_cells_1, cf.hex3d_num_cells_2, cf.hex3d_num_cells_z
        c.max_occupants, c.min_points_per_voxel = cf.hex3d_max_occupants, cf.min_points_per_voxel
        c.sensor_noise_var_per_axis, c.wishart_nu = cf.sensor_noise_var_per_axis, cf.wishart_nu
        c.wishart_psi_scale, c.kappa_main_scale = cf.wishart_psi_scale, cf.kappa_main_scale
        c.kappa_min, c.kappa_max, c.eig_min, c.eps_lift = cf.kappa_min, cf.kappa_max, cf.eig_min, cf.eps_lift
        c.max_points, c.device = int(max_points), int(device)
        h = C.c_void_p()
        rc = self.lib.gcs_surfel_ctx_create(C.byref(c), C.byref(h))
        if rc != 0:
            raise (ValueError if rc == -1 else RuntimeError)(f"gcs_surfel_ctx_create failed ({rc})")
        self.h = h
        self.device = int(device)
        self.max_points = int(max_points)
        self._bufs = {}

    def close(self):
        if getattr(self, "h", None):
            self.lib.gcs_surfel_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.gcs_surfel_last_error(self.h).decode(errors="replace")
            raise (ValueError if rc in (-1, -3) else RuntimeError)(f"{what} failed ({rc}): {msg}")

    def extract(self, points, timestamps, weights, want_intermediates=False, into=None):
        """Surfel arrays (device tensors) + n_valid + centre; points (N,3) / timestamps / weights f64.
        The output tensors belong to the extractor and are overwritten by its next call.  into: a dict of
        the batch-slice tensors (Lambdas, thetas, etas, weights, timestamps, colors, valid_mask as uint8,
        source_indices; n_surfel rows each) the kernel writes instead of the extractor's own arrays."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        cf = self.config
        p = torch.as_tensor(points, dtype=torch.float64, device=dev).reshape(-1, 3).contiguous()
        t = torch.as_tensor(timestamps, dtype=torch.float64, device=dev).reshape(-1).contiguous()
        w = torch.as_tensor(weights, dtype=torch.float64, device=dev).reshape(-1).contiguous()
        n = int(p.shape[0])
        if t.shape[0] != n or w.shape[0] != n:
            raise ValueError("points, timestamps and weights must have the same length")
        o, out = self.outputs(want_intermediates, into)
        self._chk(self.lib.gcs_surfel_ctx_set_stream(self.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                  "gcs_surfel_ctx_set_stream")
        self._chk(self.lib.gcs_extract_lidar_surfels(self.h, C.c_void_p(p.data_ptr()), C.c_void_p(t.data_ptr()),
                                                     C.c_void_p(w.data_ptr()), n, C.byref(o)),
                  "gcs_extract_lidar_surfels")
        out["n_valid"] = int(o.n_valid)
        out["center"] = np.array(o.center[:])
        out["cert"] = np.array(o.cert[:])
        return out

    def outputs(self, want_intermediates=False, into=None):
        """(gcs_surfel_outputs, tensors) of one call: the extractor's arrays, with the batch-slice
        tensors of `into` (extract's argument) in place of its own."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        cf = self.config
        key = bool(want_intermediates)
        if key not in self._bufs:  # allocated once per extractor (and per intermediates flag)
            ns = cf.n_surfel
            f = lambda *sh, dt=torch.float64: torch.empty(sh, dtype=dt, device=dev)  # noqa: E731
            out = dict(positions=f(ns, 3), covariances=f(ns, 3, 3), normals=f(ns, 3), kappas=f(ns), weights=f(ns),
                       timestamps=f(ns), Lambdas=f(ns, 3, 3), thetas=f(ns, 3), etas=f(ns, GC_VMF_N_LOBES, 3),
                       colors=f(ns, 3), valid_mask=f(ns, dt=torch.uint8), source_indices=f(ns, dt=torch.int32),
                       cell_ids=f(ns, dt=torch.int32))
            if want_intermediates:
                out["bucket"] = f(cf.n_cells, cf.hex3d_max_occupants, dt=torch.int32)
                out["count"] = f(cf.n_cells, dt=torch.int32)
            o = L.GcsSurfelOutputs()
            for k, v in out.items():
                setattr(o, k, v.data_ptr())
            self._bufs[key] = (out, o)
        out, o = self._bufs[key]
        out = dict(out)
        if into is not None:  # write the MeasurementBatch's LiDAR slice in place (padding rows: zeros)
            o2 = L.GcsSurfelOutputs()
            for k in ("positions", "covariances", "normals", "kappas", "cell_ids", "bucket", "count"):
                setattr(o2, k, getattr(o, k))
            for k, v in into.items():
                setattr(o2, k, v.data_ptr())
                out[k] = v
            o = o2
        return o, out


_extractors = {}


def _extractor_for(config, n, device):
    key = (tuple((f.name, getattr(config, f.name)) for f in fields(config)), device)
    ex = _extractors.get(key)
    if ex is None or ex.max_points < n:
        if ex is not None:
            ex.close()
        ex = SurfelExtractor(config, max_points=max(n, 8192), device=device)
        _extractors[key] = ex
    return ex


def extract_lidar_surfels(points, timestamps, weights, config: Optional[SurfelExtractionConfig] = None,
                          base_batch: Optional[MeasurementBatch] = None, chart_id: str = CHART_ID,
                          anchor_id: str = "surfel_extraction", device: int = 0, extractor: SurfelExtractor = None):
    """lidar_surfel_extraction.py:339-431.  Fixed-cost operator: n_surfel LiDAR slots; a camera
    base_batch keeps its camera slice and receives the LiDAR slice
    (measurement_batch_add_lidar_surfels), otherwise a lidar-only batch."""
    torch = _torch()
    config = config or SurfelExtractionConfig()
    n = int(np.asarray(points.shape)[0]) if hasattr(points, "shape") else len(points)
    ex = extractor or _extractor_for(config, n, device)
    dev = f"cuda:{ex.device}"
    if base_batch is None:
        # the kernel writes the LiDAR slice of a fresh zeroed batch directly: its padding rows are the
        # empty batch's zeros, so only the sources of the valid rows remain to set
        batch = create_empty_measurement_batch(config.n_feat, config.n_surfel, dev)
        s = batch.n_feat
        sl = slice(s, s + config.n_surfel)
        into = dict(Lambdas=batch.Lambdas[sl], thetas=batch.thetas[sl], etas=batch.etas[sl], weights=batch.weights[sl],
                    timestamps=batch.timestamps[sl], colors=batch.colors[sl],
                    valid_mask=batch.valid_mask[sl].view(torch.uint8), source_indices=batch.source_indices[sl])
        nv = ex.extract(points, timestamps, weights, into=into)["n_valid"]
        batch.sources[s:s + nv] = 1
    else:
        if base_batch.n_surfel != config.n_surfel:
            raise ValueError("base_batch.n_surfel differs from config.n_surfel")
        r = ex.extract(points, timestamps, weights)
        nv = r["n_valid"]
        batch = replace(base_batch, **{k: getattr(base_batch, k).clone() for k in
                                       ("Lambdas", "thetas", "etas", "weights", "sources", "source_indices",
                                        "valid_mask", "timestamps", "colors")})
        s, e = batch.n_feat, batch.n_feat + nv
        batch.Lambdas[s:e] = r["Lambdas"][:nv]
        batch.thetas[s:e] = r["thetas"][:nv]
        batch.etas[s:e] = r["etas"][:nv]
        batch.weights[s:e] = r["weights"][:nv]
        batch.sources[s:e] = 1
        batch.source_indices[s:e] = r["source_indices"][:nv]
        batch.valid_mask[s:e] = True
        batch.timestamps[s:e] = r["timestamps"][:nv]
        batch.colors[s:e] = r["colors"][:nv]
    batch.n_lidar_valid = nv
    cert, effect = surfel_cert(nv, config.n_surfel, chart_id, anchor_id)
    del torch
    return batch, cert, effect


def surfel_cert(nv: int, n_surfel: int, chart_id: str = CHART_ID, anchor_id: str = "surfel_extraction"):
    """(CertBundle, ExpectedEffect) of a surfel extraction with nv valid surfels (:420-431)."""
    support = float(nv) / float(max(n_surfel, 1))
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id,
                                    triggers=["ma_hex3d_binning", "plane_fit_batched", "wishart_regularization"],
                                    support=SupportCert(ess_total=float(nv), support_frac=support),
                                    influence=InfluenceCert.identity())
    return cert, ExpectedEffect(objective_name="surfel_extraction", predicted=float(nv), realized=float(nv))
