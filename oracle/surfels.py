"""numpy restatement of the live primitive path's LiDAR surfel extraction -- TEST INFRASTRUCTURE ONLY.

FS = fl_ws/src/fl_slam_poc/fl_slam_poc.  Follows
  * MA-hex 3D bucketing          FS/common/ma_hex_web.py:182-303 (hex_cell_3d_batch, bin_points_3d)
  * per-cell weighted plane fit  FS/backend/operators/lidar_surfel_extraction.py:69-163
  * extraction core + selection  lidar_surfel_extraction.py:227-331
  * operator + MeasurementBatch   lidar_surfel_extraction.py:339-431,
                                 FS/backend/structures/measurement_batch.py:137-381
The product path (gc-slam_amd/) never imports this; it is the checker of tests/test_surfels.py and
tests/test_gpu_surfels.py.

Pinning: the reference holds no golden vectors for this operator and JAX is absent here, so the
restatement is pinned by the reference's own smoke test (test_lidar_surfel_extraction_mahex3d.py:
16-61, restated in tests/test_surfels.py) and closed-form cases (planar patches with known normal,
centroid and in-plane spread); bit-level parity with JAX is parity unpinned (Surfels).
Reduction orders follow numpy (the reference's are XLA's); numpy.linalg.eigh is LAPACK syevd as
JAX's CPU eigh.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GC_NONFINITE_SENTINEL = 1e6   # FS/common/constants.py:257
GC_N_SURFEL = 1024            # constants.py:353
GC_N_FEAT = 512               # constants.py:350
GC_EPS_LIFT = 1e-9            # constants.py:71
GC_VMF_N_LOBES = 3            # constants.py:463
SQRT3_HALF = float(np.sqrt(np.float64(3.0)) * 0.5)


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
    eps_lift: float = GC_EPS_LIFT

    @property
    def n_cells(self):
        return int(self.hex3d_num_cells_1 * self.hex3d_num_cells_2 * self.hex3d_num_cells_z)


def hex_cell_3d(points, h):
    """ma_hex_web.py:221-240: s1 = x, s2 = x/2 + (sqrt 3 / 2) y, cell_k = floor(s_k / h), z linear."""
    p = np.asarray(points, np.float64).reshape(-1, 3)
    h = max(float(h), 1e-12)
    s1 = p[:, 0]
    s2 = p[:, 0] * 0.5 + p[:, 1] * SQRT3_HALF
    sz = p[:, 2]
    return np.stack([np.floor(s1 / h), np.floor(s2 / h), np.floor(sz / h)], axis=1).astype(np.int64)


def point_mask_and_center(points, weights, eig_min=1e-12):
    """lidar_surfel_extraction.py:259-267: sentinel mask, masked weights, weighted centre."""
    p = np.asarray(points, np.float64).reshape(-1, 3)
    mask = np.all(np.abs(p) < 0.1 * GC_NONFINITE_SENTINEL, axis=1)
    w_eff = np.asarray(weights, np.float64) * mask.astype(np.float64)
    w_sum = np.sum(w_eff) + eig_min
    center = np.sum(p * w_eff[:, None], axis=0) / w_sum
    return mask, w_eff, center


def bin_points_3d(points_c, mask, cfg: SurfelExtractionConfig):
    """ma_hex_web.py:243-303: linear cell of every point (mod-wrapped hash grid), stable argsort by
    (masked, cell), the first max_occupants points of each cell in index order, counts clipped.
    Returns (bucket (n_cells, max_occ) int32 with -1 padding, count_clipped (n_cells,), linear)."""
    n1, n2, nz = cfg.hex3d_num_cells_1, cfg.hex3d_num_cells_2, cfg.hex3d_num_cells_z
    n_cells, max_occ = cfg.n_cells, cfg.hex3d_max_occupants
    cells = hex_cell_3d(points_c, cfg.voxel_size_m)
    cells = np.mod(cells, np.array([n1, n2, nz]))
    linear = cells[:, 0] * (n2 * nz) + cells[:, 1] * nz + cells[:, 2]
    m = np.asarray(mask).astype(np.int64)
    linear = np.where(m > 0, linear, 0)
    key = linear + (1 - m) * n_cells
    order = np.argsort(key, kind="stable")
    bucket = np.full((n_cells, max_occ), -1, np.int32)
    count = np.zeros(n_cells, np.int64)
    for i in order:
        if not m[i]:
            continue
        c = linear[i]
        if count[c] < max_occ:
            bucket[c, count[c]] = i
        count[c] += 1
    return bucket, np.minimum(count, max_occ).astype(np.int32), linear.astype(np.int32)


def _normalize(v, eps=1e-12):
    return v / (np.linalg.norm(v) + eps)


def orthonormal_basis_from_normal(n, eps=1e-12):
    """lidar_surfel_extraction.py:72-81."""
    n = _normalize(n, eps)
    e1 = np.array([-n[1], n[0], 0.0]) if abs(n[2]) < 0.9 else np.array([-n[2], 0.0, n[0]])
    e1 = _normalize(e1, eps)
    e2 = _normalize(np.cross(n, e1), eps)
    return e1, e2


def fit_one_cell(points_c, timestamps, weights, idx_vec, count_used, cfg: SurfelExtractionConfig, eps=1e-12):
    """lidar_surfel_extraction.py:84-163 -> (centroid_c, Sigma_reg, normal, kappa, w_surfel,
    t_surfel, valid, sigma_perp_sq)."""
    idx_vec = np.asarray(idx_vec, np.int64)
    idx_safe = np.maximum(idx_vec, 0)
    present = (idx_vec >= 0).astype(np.float64)
    pts = points_c[idx_safe]
    w = weights[idx_safe] * present
    t = timestamps[idx_safe] * present
    em = cfg.eig_min
    w_sum = np.sum(w) + eps
    centroid = np.sum(pts * w[:, None], axis=0) / w_sum
    centered = pts - centroid[None, :]
    cov = (centered * w[:, None]).T @ centered / w_sum
    cov = 0.5 * (cov + cov.T) + em * np.eye(3)
    ev, V = np.linalg.eigh(cov)
    normal = V[:, 0]
    normal = normal * (-1.0 if normal[2] < 0.0 else 1.0)
    normal = _normalize(normal, eps)
    e1, e2 = orthonormal_basis_from_normal(normal, eps)
    p1, p2 = centered @ e1, centered @ e2
    var_e1 = np.sum(w * p1 * p1) / w_sum + cfg.sensor_noise_var_per_axis
    var_e2 = np.sum(w * p2 * p2) / w_sum + cfg.sensor_noise_var_per_axis
    sigma_perp_sq = max(ev[0], em)
    var_perp = sigma_perp_sq + cfg.sensor_noise_var_per_axis
    B = np.stack([e1, e2, normal], axis=1)
    D = np.diag([max(var_e1, em), max(var_e2, em), max(var_perp, em)])
    Sigma = B @ D @ B.T
    Sigma = 0.5 * (Sigma + Sigma.T) + em * np.eye(3)
    Lam = np.linalg.inv(Sigma + em * np.eye(3))
    Lam = 0.5 * (Lam + Lam.T)
    psi = max(cfg.wishart_psi_scale, eps)
    Lam_reg = Lam + (cfg.wishart_nu / psi) * np.eye(3)
    Lam_reg = 0.5 * (Lam_reg + Lam_reg.T) + em * np.eye(3)
    Sigma_reg = np.linalg.inv(Lam_reg)
    Sigma_reg = 0.5 * (Sigma_reg + Sigma_reg.T) + em * np.eye(3)
    kappa = cfg.kappa_main_scale / np.sqrt(max(sigma_perp_sq, em))
    kappa = min(max(kappa, cfg.kappa_min), cfg.kappa_max)
    w_surfel = np.sum(w)
    t_surfel = np.sum(t) / w_sum
    valid = bool(count_used >= cfg.min_points_per_voxel and w_surfel > 0.0)
    return centroid, Sigma_reg, normal, kappa, w_surfel, t_surfel, valid, sigma_perp_sq


def extract_surfels_mahex3d(points, timestamps, weights, cfg: SurfelExtractionConfig, center=None):
    """lidar_surfel_extraction.py:227-331.  center: use this centre instead of the weighted mean
    (the parity tests pass the device's, so the cell assignment is checked apart from the order of
    the centre's sum).  Returns a dict with the fixed-size outputs and the intermediates."""
    p = np.asarray(points, np.float64).reshape(-1, 3)
    t = np.asarray(timestamps, np.float64).reshape(-1)
    mask, w_eff, c = point_mask_and_center(p, weights, cfg.eig_min)
    if center is not None:
        c = np.asarray(center, np.float64)
    pc = p - c[None, :]
    bucket, count, linear = bin_points_3d(pc, mask, cfg)
    n_cells = cfg.n_cells
    cent = np.zeros((n_cells, 3))
    covs = np.zeros((n_cells, 3, 3))
    normals = np.zeros((n_cells, 3))
    kappas = np.zeros(n_cells)
    sw = np.zeros(n_cells)
    st = np.zeros(n_cells)
    valid = np.zeros(n_cells, bool)
    spq = np.zeros(n_cells)
    for k in range(n_cells):  # empty cells run the same formulas on zero weights (never valid)
        r = fit_one_cell(pc, t, w_eff, bucket[k], count[k], cfg)
        cent[k], covs[k], normals[k], kappas[k], sw[k], st[k], valid[k], spq[k] = r
    cent = cent + c[None, :]
    key = np.arange(n_cells) + (1 - valid.astype(np.int64)) * n_cells
    order = np.argsort(key, kind="stable")
    take = order[:cfg.n_surfel]
    n_valid = int(np.sum(valid[take]))
    sm = (np.arange(cfg.n_surfel) < n_valid).astype(np.float64)
    out = dict(
        positions=cent[take] * sm[:, None],
        covariances=covs[take] * sm[:, None, None] + (1.0 - sm)[:, None, None] * np.eye(3)[None],
        normals=normals[take] * sm[:, None],
        kappas=kappas[take] * sm,
        weights=sw[take] * sm,
        timestamps=st[take] * sm,
        n_valid=n_valid,
        cell_ids=take[:n_valid].astype(np.int32),
        center=c, bucket=bucket, count=count, linear=linear, mask=mask, cell_valid=valid,
        cell_fit=dict(centroid=cent, cov=covs, normal=normals, kappa=kappas, w=sw, t=st, sigma_perp_sq=spq),
    )
    return out


def lidar_measurement_batch(ext, cfg: SurfelExtractionConfig):
    """measurement_batch_from_lidar_only / measurement_batch_add_lidar_surfels
    (measurement_batch.py:272-381): the LiDAR slice [n_feat, n_feat + n_valid) in info form."""
    n = min(int(ext["n_valid"]), cfg.n_surfel)
    nt = cfg.n_feat + cfg.n_surfel
    Lam = np.zeros((nt, 3, 3))
    th = np.zeros((nt, 3))
    etas = np.zeros((nt, GC_VMF_N_LOBES, 3))
    w = np.zeros(nt)
    src = np.zeros(nt, np.int32)
    sidx = np.zeros(nt, np.int32)
    vm = np.zeros(nt, bool)
    ts = np.zeros(nt)
    col = np.zeros((nt, 3))
    s = cfg.n_feat
    for i in range(n):
        L = np.linalg.inv(ext["covariances"][i] + cfg.eps_lift * np.eye(3))
        Lam[s + i] = L
        th[s + i] = L @ ext["positions"][i]
        etas[s + i, 0] = ext["kappas"][i] * ext["normals"][i]
        nz = min(max(ext["normals"][i][2], -1.0), 1.0)
        col[s + i] = 0.25 + 0.5 * (nz + 1.0) / 2.0
    w[s:s + n] = ext["weights"][:n]
    src[s:s + n] = 1
    sidx[s:s + n] = np.arange(n)
    vm[s:s + n] = True
    ts[s:s + n] = ext["timestamps"][:n]
    return dict(Lambdas=Lam, thetas=th, etas=etas, weights=w, sources=src, source_indices=sidx, valid_mask=vm,
                timestamps=ts, colors=col, n_feat=cfg.n_feat, n_surfel=cfg.n_surfel, n_camera_valid=0,
                n_lidar_valid=n)


def extract_lidar_surfels(points, timestamps, weights, cfg: SurfelExtractionConfig | None = None):
    """lidar_surfel_extraction.py:339-431 (lidar-only batch): (batch dict, cert dict)."""
    cfg = cfg or SurfelExtractionConfig()
    ext = extract_surfels_mahex3d(points, timestamps, weights, cfg)
    batch = lidar_measurement_batch(ext, cfg)
    n_use = ext["n_valid"]
    cert = dict(exact=False, triggers=["ma_hex3d_binning", "plane_fit_batched", "wishart_regularization"],
                ess_total=float(n_use), support_frac=float(n_use) / float(max(cfg.n_surfel, 1)))
    return batch, cert, ext
