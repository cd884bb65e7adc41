"""L2 drop-in: process_scan_single_hypothesis / process_hypotheses with the reference calling
convention (FS/backend/pipeline.py:316-340, :1594-1621) on the MI355X through libgcslam_hip.so, plus
the node-level noise updates the reference's backend node calls after the hypothesis loop
(backend_node.py:2093-2119) and the RuntimeManifest (pipeline.py:1629-1793).

Two LiDAR evidence paths behind the one signature:
  * the 14-step bin path (README.md:105-122): `map_bins`, a HypothesisContext that owns the
    device-resident MapBinStats of this hypothesis (the legacy pipeline took bin_atlas/map_stats,
    CHANGELOG.md:280);
  * the live primitive path (pipeline.py:778-1011, 1232-1492) when `primitive_map` (an AtlasMap) is
    given: surfels, recency inflation, the map view, OT association and visual pose evidence between
    gcs_scan_begin and gcs_scan_finish, then step 12b at z_t; the result carries the updated map
    (`map`, the node's result.map hand-off, backend_node.py:2079-2083) and its MapUpdateCert.
"""

from __future__ import annotations

import json
import os
import time
import warnings
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

import ctypes as C

from . import _lib as L
from .certificates import (CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert, MismatchCert, SupportCert,
                           aggregate_certificates)
from .context import HypothesisContext
from .outputs import tape_from_result

CHART_ID = "GC-RIGHT-01"
D_Z = 22
HYP_WEIGHT_FLOOR = 0.0025   # constants.py:63


@dataclass
class BeliefGaussianInfo:
    """FS/common/belief.py:196-229 (arrays as numpy float64)."""
    chart_id: str
    anchor_id: str
    X_anchor: np.ndarray
    stamp_sec: float
    z_lin: np.ndarray
    L: np.ndarray
    h: np.ndarray
    cert: Optional[CertBundle] = None

    @classmethod
    def create_identity_prior(cls, anchor_id="initial", stamp_sec=0.0, prior_precision=1e-6):
        """belief.py:320-358."""
        return cls(CHART_ID, anchor_id, np.zeros(6), stamp_sec, np.zeros(D_Z), prior_precision * np.eye(D_Z),
                   np.zeros(D_Z), CertBundle.create_exact(CHART_ID, anchor_id))


@dataclass
class PipelineConfig:
    """Bin-path subset of FS/backend/pipeline.py:96-223 plus the declared scale parameters."""
    K_HYP: int = 4
    N_POINTS_CAP: int = 8192
    B_BINS: int = 48
    soft_assign_mode: str = "dense"   # "dense" (reference) | "scale" (K candidates, declared)
    k_cand: int = 16
    tau_soft_assign: Optional[float] = None
    eps_psd: float = 1e-12
    eps_lift: float = 1e-9
    eps_mass: float = 1e-12
    alpha_min: float = 1.0            # constants.py:89-90
    alpha_max: float = 1.0
    c0_cond: float = 1e6              # constants.py:92
    power_beta_min: float = 0.25      # pipeline.py:119-121 (fixed in the library)
    power_beta_exc_c: float = 50.0
    power_beta_z_c: float = 1.0
    c_frob: float = 1.0
    forgetting_factor: float = 0.99
    Sigma_g: Optional[np.ndarray] = None   # node sets these per scan from the IW state (backend_node.py:2020-2023)
    Sigma_a: Optional[np.ndarray] = None   # None: the IW mode of the context's measurement-noise state
    imu_gravity_scale: float = 1.0
    deskew_rotation_only: bool = False
    lidar_origin_base: tuple = (0.0, 0.0, 0.0)
    gravity_W: tuple = (0.0, 0.0, -9.81)
    planar_z_ref: float = 0.0         # constants.py:294-310
    planar_z_sigma: float = 0.1
    planar_vz_sigma: float = 0.01
    enable_imu_odom: bool = True      # False: LiDAR-only ablation (the reference always runs the branch)
    camera_batch_policy: str = "warn"  # camera evidence is out of scope here: "warn" once | "raise" | "ignore"
    max_raw_points: int = 1 << 20
    device: int = 0
    # PipelineConfig.enable_timing (pipeline.py:380-394; default off, backend_node.py:152): the live
    # path's stages are timed with a device sync + perf_counter each, into result.stage_ms and the
    # tape's t_*_ms fields (a diagnostic: the syncs serialise host and device)
    enable_timing: bool = False
    # live primitive path (pipeline.py:179-211; constants.py:350-477)
    n_feat: int = 512
    n_surfel: int = 1024
    surfel_voxel_size_m: float = 0.1
    surfel_min_points_per_voxel: int = 3
    k_assoc: int = 8
    k_sinkhorn: int = 50
    ot_epsilon: float = 0.1
    ot_tau_a: float = 0.5
    ot_tau_b: float = 0.5
    primitive_map_max_size: int = 50000
    k_insert_tile: int = 64
    H_TILE: float = 2.0
    R_ACTIVE_TILES_XY: int = 1
    R_ACTIVE_TILES_Z: int = 0
    M_TILE_VIEW: int = 1024
    R_STENCIL_TILES_XY: int = 1
    R_STENCIL_TILES_Z: int = 0
    N_ACTIVE_TILES: int = 7
    N_STENCIL_TILES: int = 7
    RECENCY_DECAY_LAMBDA: float = 0.02
    RECENCY_MIN_SCALE: float = 0.05

    def context_kwargs(self) -> dict:
        return dict(n_bins=self.B_BINS, n_points_cap=self.N_POINTS_CAP, max_raw_points=self.max_raw_points,
                    mode=self.soft_assign_mode, k_cand=self.k_cand, tau=self.tau_soft_assign,
                    lidar_origin=self.lidar_origin_base, deskew_rotation_only=self.deskew_rotation_only,
                    forgetting_factor=self.forgetting_factor, gravity_W=self.gravity_W, device=self.device,
                    use_imu_odom=self.enable_imu_odom, imu_gravity_scale=self.imu_gravity_scale,
                    planar_z_ref=self.planar_z_ref, planar_z_sigma=self.planar_z_sigma,
                    planar_vz_sigma=self.planar_vz_sigma, alpha_min=self.alpha_min, alpha_max=self.alpha_max,
                    c0_cond=self.c0_cond)

    def make_context(self) -> HypothesisContext:
        return HypothesisContext(**self.context_kwargs())


@dataclass
class MapUpdateCert:
    """FS/common/certificates.py MapUpdateCert, as step 12b fills it (pipeline.py:1454-1487)."""
    n_active_tiles: int = 0
    tile_ids_active: List[int] = field(default_factory=list)
    n_inactive_tiles: int = 0
    staleness_inflation_strength: float = 0.0
    staleness_cov_inflation_trace: float = 0.0
    stale_precision_downscale_total: float = 0.0
    tile_ids_inactive: List[int] = field(default_factory=list)
    tile_cache_hits: int = 0
    tile_cache_misses: int = 0
    candidate_tiles_per_meas_mean: float = 0.0
    candidate_primitives_per_meas_mean: float = 0.0
    candidate_primitives_per_meas_p95: float = 0.0
    insert_count_total: int = 0
    insert_mass_total: float = 0.0
    insert_mass_p95: float = 0.0
    evicted_count: int = 0
    evicted_mass_total: float = 0.0
    fused_count: int = 0
    fused_mass_total: float = 0.0
    merged_count: int = 0


@dataclass
class ScanPipelineResult:
    """FS/backend/pipeline.py:230-254."""
    belief_updated: BeliefGaussianInfo
    iw_process_dPsi: np.ndarray
    iw_process_dnu: np.ndarray
    iw_meas_dPsi: np.ndarray
    iw_meas_dnu: np.ndarray
    iw_lidar_bucket_dPsi: np.ndarray
    iw_lidar_bucket_dnu: np.ndarray
    all_certs: List[CertBundle]
    aggregated_cert: CertBundle
    diagnostics_tape: Optional[object] = None   # gcslam.outputs.MinimalScanTape (diagnostics.py:19-160)
    map_bins_updated: Optional[HypothesisContext] = None
    z_t: Optional[np.ndarray] = None
    raw_cert: Optional[np.ndarray] = None
    L_evidence: Optional[np.ndarray] = None
    h_evidence: Optional[np.ndarray] = None
    L_imu_odom: Optional[np.ndarray] = None
    h_imu_odom: Optional[np.ndarray] = None
    # live primitive path (pipeline.py:230-254): the updated map, the scan's measurement batch, the
    # map-update certificate and the association / view it fused through
    map: Optional[object] = None
    measurement_batch: Optional[object] = None
    map_update_cert: Optional[MapUpdateCert] = None
    association: Optional[object] = None
    map_view: Optional[object] = None
    z_lin_pose: Optional[np.ndarray] = None
    map_record: Optional[dict] = None  # the map update's inputs (primitive_map_follow)
    stage_ms: Optional[dict] = None    # live path, config.enable_timing: wall ms per stage (synced)


IMU_ODOM_CERTS = (("OdomEvidenceGaussian",), ("ImuAccelDirectionTimeResolved", "TransportConsistencyWeighting"),
                  ("ImuDependenceInflation",), ("ImuGyroRotationGaussian",), ("ImuPreintegrationVelPos",),
                  ("PlanarZPrior",), ("VelocityZPrior",), ("OdomVelocityEvidence",), ("OdomYawRateEvidence",),
                  ("PoseTwistKinematicConsistency",), ("OdomDependenceInflation",))


def _certs_from_vector(c, io, chart, anchor, live_certs=None):
    """Rebuild the per-operator certificates in the reference's all_certs order from the scan's
    cert vector and the eleven IMU/odometry certificate rows (DESIGN.md cert slots).  live_certs: the
    live path's map-branch + visual certs, which take the place of the bin path's LiDAR certs."""
    I = InfluenceCert
    c = c.tolist() if hasattr(c, "tolist") else list(c)      # Python floats: no numpy scalar per field
    io = io.tolist() if hasattr(io, "tolist") else list(io)
    certs = [
        CertBundle.create_approx(chart, anchor, ["PointBudgetResample"], support=SupportCert(c[0], c[1]),
                                 influence=I(mass_epsilon_ratio=c[2])),
        CertBundle.create_approx(chart, anchor, ["PredictDiffusion"],
                                 influence=I(lift_strength=c[6], psd_projection_delta=c[7], dt_scale=c[8])),
        CertBundle.create_exact(chart, anchor, support=SupportCert(c[10], c[9])),
    ]
    for k, trig in enumerate(IMU_ODOM_CERTS):
        r = io[7 * k:7 * k + 7]
        if not any(r):
            continue   # branch disabled
        certs.append(CertBundle.create_approx(chart, anchor, list(trig), support=SupportCert(r[0], r[1]),
                                              mismatch=MismatchCert(nll_per_ess=r[2]),
                                              influence=I(lift_strength=r[3], psd_projection_delta=r[4],
                                                          mass_epsilon_ratio=r[5], trust_alpha=r[6])))
    if live_certs is not None:
        certs += list(live_certs)
    else:
        certs += [
            CertBundle.create_exact(chart, anchor, support=SupportCert(c[12], c[13])),
            CertBundle.create_approx(chart, anchor, ["ScanBinMomentMatch"], support=SupportCert(c[14], c[15]),
                                     influence=I(psd_projection_delta=c[16], mass_epsilon_ratio=c[17])),
            CertBundle.create_approx(chart, anchor, ["MatrixFisherRotationEvidence"],
                                     influence=I(psd_projection_delta=c[18], mass_epsilon_ratio=c[19])),
            CertBundle.create_approx(chart, anchor, ["PlanarTranslationEvidence"],
                                     influence=I(psd_projection_delta=c[25], mass_epsilon_ratio=c[26])),
        ]
    certs += [
        CertBundle.create_approx(chart, anchor, ["PowerTempering"], frobenius_applied=abs(1.0 - c[30]) > 0.0,
                                 influence=I(power_beta=c[30])),
        CertBundle.create_approx(chart, anchor, ["ExcitationPriorScaling"],
                                 influence=I(dt_scale=1.0 - c[31], extrinsic_scale=1.0 - c[32])),
        CertBundle.create_exact(chart, anchor, influence=I(trust_alpha=c[33]),
                                conditioning=ConditioningCert(cond=c[49], near_null_count=int(c[50]))),
        CertBundle.create_approx(chart, anchor, ["InfoFusionAdditive"],
                                 influence=I(psd_projection_delta=c[34], trust_alpha=c[33])),
        CertBundle.create_approx(chart, anchor, ["PoseUpdateFrobeniusRecompose"], frobenius_applied=c[36] > 0),
        CertBundle.create_approx(chart, anchor, ["AnchorDriftUpdate"], influence=I(anchor_drift_rho=c[37])),
    ]
    return certs


_pinned = {}


def _to_device(a, dtype, device, role):
    """Host array -> device tensor through one pinned staging buffer per role, grown to the largest
    array seen (not one per shape: scan sizes vary) and reused across scans: one async H2D, and before
    the buffer is refilled the event of its previous copy is waited on (the copy may still read it)."""
    import torch
    if isinstance(a, torch.Tensor):
        return a.to(f"cuda:{device}", dtype=dtype).contiguous()
    a = np.ascontiguousarray(a)
    key = (role, device, dtype)
    ent = _pinned.get(key)
    if ent is not None and ent[0].numel() < a.size:
        if ent[1] is not None:
            ent[1].synchronize()
        ent = None
    if ent is None:
        ent = _pinned[key] = [torch.empty(max(a.size, 4096), dtype=dtype).pin_memory(), None]
    flat, ev = ent
    if ev is not None:
        ev.synchronize()
    buf = flat[:a.size].view(a.shape)
    buf.numpy()[...] = a
    out = buf.to(f"cuda:{device}", non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    ent[1] = ev
    return out


# GCSLAM_LIVE_STAMPS=1: host wall-clock stamps of each call's phases (tools/live_bench.py prints their
# mean differences); off, _stamp is a no-op
LIVE_STAMPS, LIVE_PHASES = [], []
_STAMPS_ON = os.environ.get("GCSLAM_LIVE_STAMPS", "0") == "1"


def _stamp(name):
    if _STAMPS_ON:
        LIVE_STAMPS.append((name, time.perf_counter()))


def _as_device_scan(raw_points, raw_timestamps, raw_weights, device):
    """The node's parsed cloud (backend_node.py:1675-1690) as device inputs: xyz as the float32
    PointCloud2 records the point kernel reads ((x, y, z) from host arrays, (x, y, z, pad) from a
    float32 (N, 4) tensor; point_step 4 x columns), t and w f64."""
    import torch
    if isinstance(raw_points, torch.Tensor) and raw_points.dim() == 2 and raw_points.shape[1] == 4 \
            and raw_points.dtype == torch.float32:
        rec = raw_points.to(f"cuda:{device}").contiguous()
    elif not any(isinstance(x, torch.Tensor) for x in (raw_points, raw_timestamps, raw_weights)):
        # host arrays: the three through one pinned staging buffer and one H2D copy
        p = np.asarray(raw_points, np.float64).reshape(-1, 3)
        n = p.shape[0]
        ts, ws = np.asarray(raw_timestamps).reshape(-1), np.asarray(raw_weights).reshape(-1)
        if ts.shape[0] != n or ws.shape[0] != n:
            raise ValueError("points, timestamps and weights must have the same length")
        # the device copy is reused by the next scan on the same stream (stream order keeps the begin's
        # reads of it ahead of the next copy); the staging buffer waits for its previous copy's event
        stream = torch.cuda.current_stream(device)
        # one staging pair per (device, stream), sized to the largest scan seen: a LiDAR scan's point count
        # changes from scan to scan, so a buffer per count would grow without bound over a long run
        key = ("scan", device, stream.cuda_stream)
        ent = _pinned.get(key)
        if ent is not None and ent[0] < n:
            if ent[5]:
                ent[2].synchronize()  # the last copy out of the old buffer before it is dropped
            ent = None
        if ent is None:
            cap = max(n, 4096)
            cap = -(-max(cap, (_pinned[key][0] * 3) // 2 if key in _pinned else cap) // 4096) * 4096
            hb = torch.empty(32 * cap, dtype=torch.uint8).pin_memory()
            d = torch.empty(32 * cap, dtype=torch.uint8, device=f"cuda:{device}")
            ent = _pinned[key] = [cap, hb, torch.cuda.Event(), hb.numpy(), d, False]
        cap, hb, ev, hn, d, used = ent
        if used:
            ev.synchronize()  # the previous copy out of the staging buffer
        # this scan's first 32 n bytes: xyz as compact float32 triples at [0, 12 n) (point_step 12: one
        # contiguous cast, not a strided one), t at [16 n, 24 n), w at [24 n, 32 n); one H2D copy
        np.copyto(hn[:12 * n].view(np.float32).reshape(n, 3), p, casting="unsafe")  # PointCloud2 x,y,z: float32
        hn[16 * n:24 * n].view(np.float64)[...] = ts
        hn[24 * n:32 * n].view(np.float64)[...] = ws
        d[:32 * n].copy_(hb[:32 * n], non_blocking=True)
        ev.record(stream)
        ent[5] = True
        return (d[:12 * n].view(torch.float32).view(n, 3), d[16 * n:24 * n].view(torch.float64),
                d[24 * n:32 * n].view(torch.float64))
    else:
        p = np.asarray(raw_points.cpu() if isinstance(raw_points, torch.Tensor) else raw_points,
                       np.float64).reshape(-1, 3)
        r = np.zeros((p.shape[0], 4), np.float32)
        r[:, :3] = p   # PointCloud2 x,y,z are float32 (backend_node.py:377-468)
        rec = _to_device(r, torch.float32, device, "xyz")
    t = _to_device(raw_timestamps, torch.float64, device, "t")
    w = _to_device(raw_weights, torch.float64, device, "w")
    return rec, t, w


_camera_warned = False


def _camera_batch_has_content(camera_batch):
    if camera_batch is None:
        return False
    for attr in ("n_valid", "n", "count"):
        v = getattr(camera_batch, attr, None)
        if v is not None:
            return int(v) > 0
    return True


def _process_scan_primitive(ctx: HypothesisContext, primitive_map, belief_prev, rec, t, w, imu_stamps, imu_gyro,
                            imu_accel, odom_pose, odom_cov_se3, scan_start_time, scan_end_time, dt_sec, t_last_scan,
                            t_scan, Q, config: PipelineConfig, odom_twist, odom_twist_cov, scan_seq, L_ext, h_ext,
                            update_map=True):
    """The live pipeline (pipeline.py:316-1591) on the device: gcs_scan_begin (budget, predict, IMU
    preintegration, deskew, IMU/odometry branch, z_lin_pose) -> the map branch (:778-926) -> visual
    pose evidence (:980-1010) -> gcs_scan_finish (tempering, fusion, recompose, anchor drift) ->
    step 12b at z_t (:1232-1492)."""
    import torch
    from . import association as GA, primitive_map as GPM
    from .surfels import SurfelExtractionConfig, extract_lidar_surfels
    if _live_chain_enabled(ctx, config):
        return _process_scan_live_chain(ctx, primitive_map, rec, t, w, imu_stamps, imu_gyro, imu_accel, odom_pose,
                                        odom_cov_se3, scan_start_time, scan_end_time, dt_sec, t_last_scan, t_scan, Q,
                                        config, odom_twist, odom_twist_cov, scan_seq, L_ext, h_ext, update_map)
    cap = ctx.cfg.n_points_cap
    dev = f"cuda:{config.device}"
    bufs = getattr(ctx, "_live_bufs", None)
    if bufs is None:
        bufs = ctx._live_bufs = (torch.empty((cap, 3), dtype=torch.float64, device=dev),
                                 torch.empty(cap, dtype=torch.float64, device=dev),
                                 torch.empty(cap, dtype=torch.float64, device=dev))
    stage_ms = {}
    clock = [time.perf_counter()]

    def tick(name):  # the reference's _record_timing: block until ready, then the wall clock
        if config.enable_timing:
            torch.cuda.synchronize(dev)
            now = time.perf_counter()
            stage_ms[name] = (now - clock[0]) * 1e3
            clock[0] = now

    b = ctx.scan_begin(rec, 4 * rec.shape[1], t, w, rec.shape[0], imu_stamps, imu_gyro, imu_accel, scan_start_time, scan_end_time,
                       dt_sec, Q=Q, L_ext=L_ext, h_ext=h_ext, t_last_scan=t_last_scan, t_scan=t_scan,
                       odom_pose=odom_pose, odom_cov_se3=odom_cov_se3, odom_twist=odom_twist,
                       odom_twist_cov=odom_twist_cov, Sigma_g=config.Sigma_g, Sigma_a=config.Sigma_a, buffers=bufs)
    tick("scan_begin_ms")  # budget, predict, IMU preintegration, deskew, IMU / odometry branch
    # the map branch (pipeline.py:778-926)
    scfg = SurfelExtractionConfig(n_surfel=config.n_surfel, n_feat=config.n_feat,
                                  voxel_size_m=config.surfel_voxel_size_m,
                                  min_points_per_voxel=config.surfel_min_points_per_voxel, eps_lift=config.eps_lift)
    batch, c_surf, _ = extract_lidar_surfels(bufs[0], bufs[1], bufs[2], config=scfg, chart_id=CHART_ID,
                                             device=config.device)
    tick("surfel_extraction_ms")
    centre = np.array(b.pose_pred[:3])
    active = GPM.ma_hex_stencil_tile_ids(centre, config.H_TILE, config.R_ACTIVE_TILES_XY, config.R_ACTIVE_TILES_Z)
    stencil = GPM.ma_hex_stencil_tile_ids(centre, config.H_TILE, config.R_STENCIL_TILES_XY, config.R_STENCIL_TILES_Z)
    if len(active) != int(config.N_ACTIVE_TILES):
        raise ValueError(f"active tile stencil size mismatch: expected N_ACTIVE_TILES={config.N_ACTIVE_TILES}, "
                         f"got {len(active)}")
    if len(stencil) != int(config.N_STENCIL_TILES):
        raise ValueError(f"stencil tile size mismatch: expected N_STENCIL_TILES={config.N_STENCIL_TILES}, "
                         f"got {len(stencil)}")
    if not update_map:
        # a hypothesis k > 0: the node's map is read, never written (the reference stores hypothesis 0's
        # update only, backend_node.py:2079-2083): this scan's recency, view and step 12b run on device
        # copies of the tiles it touches
        primitive_map = ctx._scratch_map = primitive_map.working_copy(list(active) + list(stencil),
                                                                      into=getattr(ctx, "_scratch_map", None))
    am, c_infl, _, infl = GPM.primitive_map_recency_inflate(primitive_map, active, int(scan_seq),
                                                            config.RECENCY_DECAY_LAMBDA, config.RECENCY_MIN_SCALE)
    view = GPM.extract_atlas_map_view(am, stencil, int(config.M_TILE_VIEW), config.eps_lift, config.eps_mass)
    tick("map_view_ms")  # recency inflation + the atlas view over the stencil
    acfg = GA.AssociationConfig(k_assoc=config.k_assoc, k_sinkhorn=config.k_sinkhorn, epsilon=config.ot_epsilon,
                                tau_a=config.ot_tau_a, tau_b=config.ot_tau_b, eps_mass=config.eps_mass,
                                h_tile=config.H_TILE, r_stencil_tiles_xy=config.R_STENCIL_TILES_XY,
                                r_stencil_tiles_z=config.R_STENCIL_TILES_Z, scan_seq=int(scan_seq),
                                recency_decay_lambda=config.RECENCY_DECAY_LAMBDA)
    res, c_assoc, _ = GA.associate_primitives_ot(batch, view, acfg, chart_id=CHART_ID, device=config.device)
    tick("association_ms")
    # the MapUpdateCert's candidate statistics (pipeline.py:879-905) come with the association
    # (computed in the library beside the Sinkhorn: no device round trip here)
    cand = res.candidate_stats
    z_lin_pose = np.array(b.z_lin_pose[:])
    vis, c_vis, _ = GA.visual_pose_evidence(res, batch, view, eps_lift=config.eps_lift, eps_mass=config.eps_mass,
                                            chart_id=CHART_ID, z_lin_pose=z_lin_pose, device=config.device)
    L_lidar, h_lidar = GA.build_visual_pose_evidence_22d(vis)
    tick("visual_pose_ms")
    # the map branch's + visual certs enter all_certs (T, pipeline.py:1211); the LiDAR evidence aggregate
    # is [deskew, surfel, association, visual] (:1049-1056)
    trig = sum(c.total_trigger_magnitude() for c in (c_surf, c_infl, c_assoc, c_vis))
    lid = (c_surf, c_assoc, c_vis)
    out = ctx.scan_finish(L_lidar, h_lidar, trig, sum(c.support.ess_total for c in lid), len(lid),
                          sum(c.mismatch.nll_per_ess for c in lid))
    z_t = np.array(out.z_t[:])
    tick("scan_finish_ms")  # evidence sum, tempering, fusion, recompose, anchor drift
    # step 12b: the primitive map update at z_t (pipeline.py:1232-1492)
    ucfg = GPM.PrimitiveMapUpdateConfig(k_insert_tile=config.k_insert_tile, H_TILE=config.H_TILE,
                                        RECENCY_DECAY_LAMBDA=config.RECENCY_DECAY_LAMBDA, eps_lift=config.eps_lift,
                                        eps_mass=config.eps_mass, eps_psd=config.eps_psd)
    st = GPM.primitive_map_update(am, batch, res, z_t, active, float(scan_end_time), int(scan_seq), config=ucfg)
    tick("map_update_ms")
    act = set(active)
    inactive = [int(x) for x in am.tile_ids if int(x) not in act]
    hits = len([x for x in active if int(x) in set(am.tile_ids)])
    muc = MapUpdateCert(n_active_tiles=len(active), tile_ids_active=[int(x) for x in active],
                        n_inactive_tiles=len(inactive), staleness_inflation_strength=infl.staleness_inflation_strength,
                        staleness_cov_inflation_trace=infl.staleness_cov_inflation_trace,
                        stale_precision_downscale_total=infl.stale_precision_downscale_total,
                        tile_ids_inactive=inactive, tile_cache_hits=hits, tile_cache_misses=len(act) - hits,
                        candidate_tiles_per_meas_mean=cand[0], candidate_primitives_per_meas_mean=cand[1],
                        candidate_primitives_per_meas_p95=cand[2],
                        **{k: st[k] for k in ("insert_count_total", "insert_mass_total", "insert_mass_p95",
                                              "evicted_count", "evicted_mass_total", "fused_count", "fused_mass_total",
                                              "merged_count")})
    # the inputs of this scan's map update: replayed on another copy of the node's map, they give this
    # hypothesis' map bit for bit (primitive_map_follow)
    record = dict(active=[int(x) for x in active], scan_seq=int(scan_seq), t=float(scan_end_time), z_t=z_t,
                  batch=batch, association=res)
    return out, dict(map=am, batch=batch, map_update_cert=muc, certs=[c_surf, c_infl, c_assoc, c_vis],
                     association=res, view=view, z_lin_pose=z_lin_pose, map_record=record, stage_ms=stage_ms)


def _live_chain_enabled(ctx: HypothesisContext, config: "PipelineConfig") -> bool:
    """The one-call live path (gcs_live_scan) unless per-stage wall times are asked for
    (config.enable_timing: the per-operator path syncs between stages), GCSLAM_LIVE_CHAIN=0, or the context
    runs on a stream other than torch's current one (the batch / view / association tensors are
    allocated on torch's stream; the chain queues on the context's)."""
    import os
    import torch
    if config.enable_timing or os.environ.get("GCSLAM_LIVE_CHAIN", "1") == "0":
        return False
    return ctx.stream_ptr is not None and ctx.stream_ptr == torch.cuda.current_stream(config.device).cuda_stream


def _live_chain_state(ctx: HypothesisContext, config: "PipelineConfig"):
    """gcs_live_scan's per-(context, config) arguments: the surfel / association contexts, the config
    structs and the fields of gcs_live_args that do not change between scans (cached on the context)."""
    from . import association as GA, primitive_map as GPM
    from .surfels import GC_VMF_N_LOBES, SurfelExtractionConfig
    key = (config.n_surfel, config.n_feat, config.surfel_voxel_size_m, config.surfel_min_points_per_voxel,
           config.eps_lift, config.eps_mass, config.eps_psd, config.k_assoc, config.k_sinkhorn, config.ot_epsilon,
           config.ot_tau_a, config.ot_tau_b, config.H_TILE, config.R_ACTIVE_TILES_XY, config.R_ACTIVE_TILES_Z,
           config.R_STENCIL_TILES_XY, config.R_STENCIL_TILES_Z, config.N_ACTIVE_TILES, config.N_STENCIL_TILES,
           config.RECENCY_DECAY_LAMBDA, config.RECENCY_MIN_SCALE, config.M_TILE_VIEW, config.k_insert_tile,
           config.device, ctx.cfg.n_points_cap)
    st = getattr(ctx, "_live_chain", None)
    if st is not None and st["key"] == key:
        return st
    cap = ctx.cfg.n_points_cap
    scfg = SurfelExtractionConfig(n_surfel=config.n_surfel, n_feat=config.n_feat,
                                  voxel_size_m=config.surfel_voxel_size_m,
                                  min_points_per_voxel=config.surfel_min_points_per_voxel, eps_lift=config.eps_lift)
    # the association runs with its operator defaults for eps_lift / eps_mass, as the per-operator path
    # calls it (associate_primitives_ot(batch, view, acfg)); the view and the pose evidence take the config's
    acfg = GA.AssociationConfig(k_assoc=config.k_assoc, k_sinkhorn=config.k_sinkhorn, epsilon=config.ot_epsilon,
                                tau_a=config.ot_tau_a, tau_b=config.ot_tau_b, eps_mass=config.eps_mass,
                                h_tile=config.H_TILE, r_stencil_tiles_xy=config.R_STENCIL_TILES_XY,
                                r_stencil_tiles_z=config.R_STENCIL_TILES_Z, scan_seq=0,
                                recency_decay_lambda=config.RECENCY_DECAY_LAMBDA)
    c_as = GA.assoc_config_struct(acfg)
    N, K = config.n_feat + config.n_surfel, int(config.k_assoc)
    ucfg = GPM.PrimitiveMapUpdateConfig(k_insert_tile=config.k_insert_tile, H_TILE=config.H_TILE,
                                        RECENCY_DECAY_LAMBDA=config.RECENCY_DECAY_LAMBDA, eps_lift=config.eps_lift,
                                        eps_mass=config.eps_mass, eps_psd=config.eps_psd)
    c_up = GPM.update_config_struct(ucfg)
    dev = f"cuda:{config.device}"
    import torch
    bufs = getattr(ctx, "_live_bufs", None)
    if bufs is None:
        bufs = ctx._live_bufs = (torch.empty((cap, 3), dtype=torch.float64, device=dev),
                                 torch.empty(cap, dtype=torch.float64, device=dev),
                                 torch.empty(cap, dtype=torch.float64, device=dev))
    a = L.GcsLiveArgs()
    a.h_tile = float(config.H_TILE)
    a.r_active_xy, a.r_active_z = int(config.R_ACTIVE_TILES_XY), int(config.R_ACTIVE_TILES_Z)
    a.r_stencil_xy, a.r_stencil_z = int(config.R_STENCIL_TILES_XY), int(config.R_STENCIL_TILES_Z)
    a.n_active_expected, a.n_stencil_expected = int(config.N_ACTIVE_TILES), int(config.N_STENCIL_TILES)
    a.recency_lambda, a.recency_min_scale = float(config.RECENCY_DECAY_LAMBDA), float(config.RECENCY_MIN_SCALE)
    a.m_tile_view = int(config.M_TILE_VIEW)
    a.eps_lift, a.eps_mass = float(config.eps_lift), float(config.eps_mass)
    a.assoc_cfg, a.update_cfg = C.addressof(c_as), C.addressof(c_up)
    a.points_dev, a.timestamps_dev, a.weights_dev = (x.data_ptr() for x in bufs)
    a.n_points = cap
    vpe = L.GcsVpeOutputs()
    a.vpe_out = C.addressof(vpe)
    lay = _live_arena(config, N, K)
    off, s0 = lay["off"], config.n_feat
    o_sf, o_v, ao = L.GcsSurfelOutputs(), L.GcsPmapView(), L.GcsAssocOutputs()
    row = {"Lambdas": 72, "thetas": 24, "etas": 24 * GC_VMF_N_LOBES, "weights": 8, "timestamps": 8,
           "colors": 24, "valid_mask": 1, "source_indices": 4}
    ptr = [(o_sf, k, off[("batch", k)] + s0 * rb) for k, rb in row.items()]  # the batch's LiDAR slice
    ptr += [(o_v, r[0], off[("view", r[0])]) for r in lay["view"][:-1]]
    ptr += [(ao, r[0], off[("assoc", r[0])]) for r in lay["assoc"]]
    ptr += [(a.meas, k, off[("batch", k)]) for k in ("Lambdas", "thetas", "etas", "weights", "valid_mask")]
    ptr += [(a, "zero_dev", 0), (a, "lidar_sources_dev", off[("batch", "sources")] + 4 * s0),
            (a, "batch_colors", off[("batch", "colors")]), (a, "batch_sources", off[("batch", "sources")]),
            (a, "view_tile_ids_dev", off[("view", "tile_ids")])]
    a.meas.n_total, a.meas.n_lobes, a.meas.n_valid = N, GC_VMF_N_LOBES, 0
    a.zero_bytes = lay["zero_bytes"]
    a.surfel_out, a.view, a.assoc_out = C.addressof(o_sf), C.addressof(o_v), C.addressof(ao)
    st = dict(key=key, scfg=scfg, ex=None, ex_key=None, o_sf=o_sf, o_v=o_v, ao=ao, o_sf_ex=None, ptr_fields=ptr, pool=int(config.N_STENCIL_TILES) * int(config.M_TILE_VIEW), acfg=acfg,
              arena=lay, c_as=c_as, c_up=c_up, args=a, vpe=vpe, bufs=bufs, N=N, K=K,
              lo=L.GcsLiveOutputs())
    ctx._live_chain = st
    return st


def _live_arena(config: "PipelineConfig", N: int, K: int) -> dict:
    """Layout of one scan's result arrays in one device allocation (8-byte aligned segments): the
    MeasurementBatch (create_empty_measurement_batch's arrays; zeroed by gcs_live_scan on its stream),
    the AtlasMapView (view_buffers' arrays), the view's tile ids and the PrimitiveAssociationResult.
    Pointers go to the C call before it; the tensors are views made after it, beside step 12b."""
    import torch
    from .surfels import GC_VMF_N_LOBES
    nt, R = config.n_feat + config.n_surfel, int(config.N_STENCIL_TILES) * int(config.M_TILE_VIEW)
    f64, i64, i32, b8 = torch.float64, torch.int64, torch.int32, torch.bool
    size = {f64: 8, i64: 8, i32: 4, b8: 1}
    parts = {
        "batch": (("Lambdas", f64, (nt, 3, 3)), ("thetas", f64, (nt, 3)), ("etas", f64, (nt, GC_VMF_N_LOBES, 3)),
                  ("weights", f64, (nt,)), ("timestamps", f64, (nt,)), ("colors", f64, (nt, 3)),
                  ("sources", i32, (nt,)), ("source_indices", i32, (nt,)), ("valid_mask", b8, (nt,))),
        "view": (("positions", f64, (R, 3)), ("covariances", f64, (R, 3, 3)), ("directions", f64, (R, 3)),
                 ("kappas", f64, (R,)), ("weights", f64, (R,)), ("primitive_ids", i64, (R,)),
                 ("last_supported_scan_seq", i64, (R,)), ("etas", f64, (R, GC_VMF_N_LOBES, 3)),
                 ("colors", f64, (R, 3)), ("candidate_tile_ids", i64, (R,)), ("candidate_slots", i32, (R,)),
                 ("valid_mask", b8, (R,)), ("tile_ids", i64, (int(config.N_STENCIL_TILES),))),
        "assoc": (("responsibilities", f64, (N, K)), ("candidate_pool_indices", i32, (N, K)),
                  ("candidate_tile_ids", i64, (N, K)), ("candidate_slots", i64, (N, K)), ("row_masses", f64, (N,)),
                  ("cost_matrix", f64, (N, K))),
    }
    lay, off = {}, 0
    for part, spec in parts.items():
        rows = []
        for name, dt, shape in spec:
            shape = tuple(int(x) for x in shape)
            z = int(np.prod(shape)) * size[dt]
            stride = tuple(int(np.prod(shape[k + 1:])) for k in range(len(shape)))
            rows.append((name, dt, shape, stride, off // size[dt], off))
            off += (z + 7) // 8 * 8
        lay[part] = [r[:5] for r in rows]
        lay.setdefault("off", {}).update({(part, r[0]): r[5] for r in rows})
        if part == "batch":
            lay["zero_bytes"] = off
    lay["total"] = off
    return lay


def _arena_tensors(typed, rows) -> dict:
    """The arena's tensors: one as_strided view per array over the arena's typed views."""
    import torch
    st = torch.as_strided
    return {name: st(typed[dt], shape, stride, item_off) for name, dt, shape, stride, item_off in rows}


def _arena_typed(buf) -> dict:
    import torch
    return {dt: buf.view(dt) for dt in (torch.float64, torch.int64, torch.int32, torch.bool)}


def _process_scan_live_chain(ctx: HypothesisContext, primitive_map, rec, t, w, imu_stamps, imu_gyro, imu_accel,
                             odom_pose, odom_cov_se3, scan_start_time, scan_end_time, dt_sec, t_last_scan, t_scan, Q,
                             config: "PipelineConfig", odom_twist, odom_twist_cov, scan_seq, L_ext, h_ext, update_map):
    """_process_scan_primitive through gcs_live_scan: begin -> surfels -> recency -> view -> association ->
    visual pose evidence -> finish -> step 12b in one C call on the context's stream (pipeline.py:316-1591;
    :778-1011, 1232-1492), with this scan's fresh result tensors handed in.  Step 12b is left running:
    live["finish"]() waits for it and fills the MapUpdateCert and the map's bookkeeping."""
    import torch
    from . import association as GA, primitive_map as GPM
    from .association import AtlasMapView
    from .surfels import GC_VMF_N_LOBES, MeasurementBatch, _extractor_for, _extractors
    st = _live_chain_state(ctx, config)
    lib, a, lo = ctx.lib, st["args"], st["lo"]
    # the operator contexts (looked up per scan: another caller may have replaced a cached one)
    ex = st.get("ex")
    if ex is None or ex.h is None or _extractors.get(st["ex_key"]) is not ex:
        ex = st["ex"] = _extractor_for(st["scfg"], ctx.cfg.n_points_cap, config.device)
        st["ex_key"] = next(k for k, v in _extractors.items() if v is ex)
    asc = GA._associator_for(st["N"], st["pool"], st["K"], config.device)
    a.surfels, a.assoc = ex.h.value, asc.h.value
    dev = f"cuda:{config.device}"
    inp, keep = ctx._scan_inputs(rec, 4 * rec.shape[1], t, w, rec.shape[0], imu_stamps, imu_gyro, imu_accel, scan_start_time,
                                 scan_end_time, dt_sec, Q=Q, L_ext=L_ext, h_ext=h_ext, t_last_scan=t_last_scan,
                                 t_scan=t_scan, odom_pose=odom_pose, odom_cov_se3=odom_cov_se3, odom_twist=odom_twist,
                                 odom_twist_cov=odom_twist_cov, Sigma_g=config.Sigma_g, Sigma_a=config.Sigma_a)
    bo = L.GcsScanBeginOutputs()
    bo.points_dev, bo.timestamps_dev, bo.weights_dev = a.points_dev, a.timestamps_dev, a.weights_dev
    in_ref = C.byref(inp)
    if not update_map:
        # a hypothesis k > 0 works on device copies of the tiles it touches (see _process_scan_primitive):
        # the copy needs the tiles around the predicted pose, so the begin runs first here
        ctx._chk(lib.gcs_scan_begin(ctx.h, in_ref, C.byref(bo)), "gcs_scan_begin")
        in_ref = None
        centre = np.array(bo.pose_pred[:3])
        ids = GPM.ma_hex_stencil_tile_ids(centre, config.H_TILE, config.R_ACTIVE_TILES_XY, config.R_ACTIVE_TILES_Z) + \
            GPM.ma_hex_stencil_tile_ids(centre, config.H_TILE, config.R_STENCIL_TILES_XY, config.R_STENCIL_TILES_Z)
        primitive_map = ctx._scratch_map = primitive_map.working_copy(ids, into=getattr(ctx, "_scratch_map", None))
    am = primitive_map
    if am.n_lobes != GC_VMF_N_LOBES:
        raise ValueError(f"live path: the map's n_lobes {am.n_lobes} differs from the batch's {GC_VMF_N_LOBES}")
    # this scan's result arrays (the results keep them) in one allocation: pointers now, tensors after
    lay = st["arena"]
    buf = torch.empty(lay["total"], dtype=torch.uint8, device=dev)
    base = buf.data_ptr()
    o_sf, o_v, ao = st["o_sf"], st["o_v"], st["ao"]
    if st["o_sf_ex"] is not ex:  # the extractor's own arrays (positions, covariances, normals, kappas, cell ids)
        o_ex, _ = ex.outputs(False)
        for k in ("positions", "covariances", "normals", "kappas", "cell_ids"):
            setattr(o_sf, k, getattr(o_ex, k))
        st["o_sf_ex"] = ex
    for obj, name, o in st["ptr_fields"]:  # the arena's arrays in the argument structs
        setattr(obj, name, base + o)
    ids, slots, free, written = am.directory()
    a.map = am.h.value
    a.n_tiles, a.tile_ids, a.tile_slots = len(ids), ids.ctypes.data, slots.ctypes.data
    a.n_free, a.free_slots, a.slot_written = len(free), free.ctypes.data, written.ctypes.data
    a.next_global_id = int(am.next_global_id)
    a.scan_seq = st["c_as"].scan_seq = int(scan_seq)
    a.timestamp = float(scan_end_time)
    out = L.GcsScanOutputs()
    _stamp("args")
    rc = lib.gcs_live_scan(ctx.h, in_ref, C.byref(bo), C.byref(a), C.byref(lo), C.byref(out))
    _stamp("live_scan")
    del keep
    if lo.n_created:  # tiles created (and cleared where written) before the device failed or ran
        am.adopt_created(lo.created_ids[:lo.n_created], lo.created_slots[:lo.n_created])
    ctx._chk(rc, "gcs_live_scan")
    try:
        typed = _arena_typed(buf)
        bt = _arena_tensors(typed, lay["batch"])
        batch = MeasurementBatch(**bt, n_feat=config.n_feat, n_surfel=config.n_surfel, n_camera_valid=0,
                                 n_lidar_valid=0)
        vt = _arena_tensors(typed, lay["view"])
        view_tids = vt.pop("tile_ids")
        a_out = _arena_tensors(typed, lay["assoc"])
        r = _live_chain_results(ctx, am, st, lo, o_sf, bo, out, batch, vt, view_tids, a_out, ao, scan_seq,
                                scan_end_time, config)
        _stamp("live_results")
        return out, r
    except BaseException:
        lib.gcs_live_collect(ctx.h, C.byref(lo))  # step 12b is queued: drain it before the error propagates
        raise


def _live_chain_results(ctx, am, st, lo, o_sf, bo, out, batch, vt, view_tids, a_out, ao, scan_seq, scan_end_time,
                        config):
    """The live dict of _process_scan_primitive from gcs_live_scan's outputs (host work that overlaps
    the queued step 12b); live["finish"]() collects step 12b."""
    from . import association as GA, primitive_map as GPM
    from .association import AtlasMapView
    from .surfels import surfel_cert
    lib = ctx.lib
    N, k_v = st["N"], int(config.M_TILE_VIEW)
    nv = int(o_sf.n_valid)
    batch.n_lidar_valid = nv
    c_surf, _ = surfel_cert(nv, config.n_surfel, CHART_ID)
    down, infl_tr, nrec = (float(x) for x in lo.recency_stats)
    infl = GPM.PrimitiveMapRecencyInflateStats(down / max(nrec, 1.0), infl_tr, down)
    c_infl = CertBundle.create_exact(chart_id=CHART_ID, anchor_id="primitive_map_recency_inflate")
    view = AtlasMapView(tile_ids=view_tids, m_tile_view=k_v, **vt)
    res = GA.association_result(a_out, ao)
    c_assoc, _ = GA.association_cert(ao, st["acfg"], N, CHART_ID)
    vis, c_vis, _ = GA.visual_pose_result(st["vpe"], config.eps_lift, CHART_ID)
    z_t = np.array(out.z_t[:])
    z_lin_pose = np.array(bo.z_lin_pose[:])
    active = [int(x) for x in lo.active_ids[:lo.n_active]]
    cand = res.candidate_stats
    record = dict(active=active, scan_seq=int(scan_seq), t=float(scan_end_time), z_t=z_t, batch=batch,
                  association=res)
    live = dict(map=am, batch=batch, map_update_cert=None, certs=[c_surf, c_infl, c_assoc, c_vis], association=res,
                view=view, z_lin_pose=z_lin_pose, map_record=record, stage_ms={})

    def finish():
        if live["map_update_cert"] is not None:
            return live["map_update_cert"]
        ctx._chk(lib.gcs_live_collect(ctx.h, C.byref(lo)), "gcs_live_collect")
        if _STAMPS_ON:
            LIVE_PHASES.append(list(lo.phase_us))
        u = lo.update
        am.total_count += int(u.insert_count_total) - int(u.evicted_count) - int(u.merged_count)
        am.next_global_id = int(lo.next_global_id)
        for k, tid in enumerate(active):
            am.counts[tid] = int(lo.counts[k])
        act = set(active)
        held = am.tiles
        inactive = [int(x) for x in held if int(x) not in act]
        hits = len([x for x in active if x in held])
        live["map_update_cert"] = MapUpdateCert(
            n_active_tiles=len(active), tile_ids_active=list(active), n_inactive_tiles=len(inactive),
            staleness_inflation_strength=infl.staleness_inflation_strength,
            staleness_cov_inflation_trace=infl.staleness_cov_inflation_trace,
            stale_precision_downscale_total=infl.stale_precision_downscale_total, tile_ids_inactive=inactive,
            tile_cache_hits=hits, tile_cache_misses=len(act) - hits, candidate_tiles_per_meas_mean=cand[0],
            candidate_primitives_per_meas_mean=cand[1], candidate_primitives_per_meas_p95=cand[2],
            insert_count_total=int(u.insert_count_total), insert_mass_total=float(u.insert_mass_total),
            insert_mass_p95=float(u.insert_mass_p95), evicted_count=int(u.evicted_count),
            evicted_mass_total=float(u.evicted_mass_total), fused_count=int(u.fused_count),
            fused_mass_total=float(u.fused_mass_total), merged_count=int(u.merged_count))
        return live["map_update_cert"]

    live["finish"] = finish
    return live


def primitive_map_follow(primitive_map, record: dict, config: "PipelineConfig"):
    """Apply a lead hypothesis' map update (its recency inflation and step 12b, pipeline.py:800-809,
    1232-1492, from `result.map_record`) to another copy of the node's map: every copy stays bitwise the
    lead's (the node's hypothesis-0 map, backend_node.py:2079-2083) without moving map rows.  Returns the
    step-12b statistics."""
    from . import primitive_map as GPM
    GPM.primitive_map_recency_inflate(primitive_map, record["active"], int(record["scan_seq"]),
                                      config.RECENCY_DECAY_LAMBDA, config.RECENCY_MIN_SCALE)
    ucfg = GPM.PrimitiveMapUpdateConfig(k_insert_tile=config.k_insert_tile, H_TILE=config.H_TILE,
                                        RECENCY_DECAY_LAMBDA=config.RECENCY_DECAY_LAMBDA, eps_lift=config.eps_lift,
                                        eps_mass=config.eps_mass, eps_psd=config.eps_psd)
    return GPM.primitive_map_update(primitive_map, record["batch"], record["association"], record["z_t"],
                                    record["active"], record["t"], int(record["scan_seq"]), config=ucfg)


def process_scan_single_hypothesis(belief_prev: BeliefGaussianInfo, raw_points, raw_timestamps, raw_weights,
                                   raw_ring, raw_tag, imu_stamps, imu_gyro, imu_accel, odom_pose, odom_cov_se3,
                                   scan_start_time, scan_end_time, dt_sec, t_last_scan, t_scan, Q,
                                   config: PipelineConfig, odom_twist=None, odom_twist_cov=None, camera_batch=None,
                                   scan_seq=0, primitive_map=None, map_bins: Optional[HypothesisContext] = None,
                                   L_ext=None, h_ext=None, update_map: bool = True) -> ScanPipelineResult:
    """FS/backend/pipeline.py:316-1591 with the bin path of README.md:105-122.

    Every reference input is consumed: the point stream, the IMU window (deskew, scan-to-scan
    preintegration, measurement-noise statistics, IMU evidence), odometry pose / covariance /
    twist (the step-9 odometry factors; None takes the node's "no odometry yet" inputs,
    backend_node.py:939-940,2047-2051).  raw_ring / raw_tag are only gathered by the reference's
    budget step for the primitive path; the bin path does not read them.  camera_batch feeds the
    live primitive path's visual evidence, which this backend does not build (DESIGN.md out of
    scope): config.camera_batch_policy says whether a non-empty batch warns (default), raises or is
    ignored.  L_ext / h_ext add further caller evidence to step 9.

    primitive_map (an AtlasMap): the live primitive path (pipeline.py:778-1011, 1232-1492) replaces the
    bin evidence; map_bins then only carries the hypothesis state (belief, IW), and result.map is the
    updated AtlasMap (the node keeps hypothesis 0's, backend_node.py:2079-2083).  The AtlasMap is updated in
    place; a hypothesis k > 0 passes update_map=False: its scan reads the node's map and works on device
    copies of the tiles it touches (result.map is that scratch), as the reference's immutable maps behave.
    The scratch is cached on the map_bins context and rewritten by its next update_map=False scan: such
    a result.map is valid until then (copy it -- AtlasMap.working_copy -- to keep it longer).
    result.map_record holds the update's inputs for primitive_map_follow (one map over several GPUs)."""
    global _camera_warned
    if _camera_batch_has_content(camera_batch):
        if config.camera_batch_policy == "raise":
            raise NotImplementedError("camera_batch: visual evidence is not part of the bin-path backend")
        if config.camera_batch_policy == "warn" and not _camera_warned:
            warnings.warn("camera_batch ignored: the bin-path backend has no visual evidence (DESIGN.md section 9)")
            _camera_warned = True
    _stamp("enter")
    ctx = map_bins if map_bins is not None else config.make_context()
    ctx.set_belief(belief_prev.X_anchor, belief_prev.stamp_sec, belief_prev.z_lin, belief_prev.L, belief_prev.h)
    rec, t, w = _as_device_scan(raw_points, raw_timestamps, raw_weights, config.device)
    _stamp("h2d")
    live = None
    if primitive_map is not None:
        out, live = _process_scan_primitive(ctx, primitive_map, belief_prev, rec, t, w, imu_stamps, imu_gyro,
                                            imu_accel, odom_pose, odom_cov_se3, scan_start_time, scan_end_time, dt_sec,
                                            t_last_scan, t_scan, Q, config, odom_twist, odom_twist_cov, scan_seq,
                                            L_ext, h_ext, update_map=update_map)
    else:
        out = ctx.scan(rec, 4 * rec.shape[1], t, w, rec.shape[0], imu_stamps, imu_gyro, imu_accel, scan_start_time, scan_end_time,
                       dt_sec, Q=Q, L_ext=L_ext, h_ext=h_ext, t_last_scan=t_last_scan, t_scan=t_scan,
                       odom_pose=odom_pose, odom_cov_se3=odom_cov_se3, odom_twist=odom_twist,
                       odom_twist_cov=odom_twist_cov, Sigma_g=config.Sigma_g, Sigma_a=config.Sigma_a)
    try:
        res = _scan_result(ctx, out, live, belief_prev, scan_seq, scan_end_time, dt_sec, rec.shape[0])
        _stamp("result")
    finally:
        if live is not None and "finish" in live:  # the one-call path's step 12b (queued): its cert
            live["map_update_cert"] = live["finish"]()
    if live is not None:
        res.map_update_cert = live["map_update_cert"]
    _stamp("collect")
    if map_bins is None:
        ctx.close()
        res.map_bins_updated = None
    return res


def _scan_result(ctx, out, live, belief_prev, scan_seq, scan_end_time, dt_sec, n_raw):
    """ScanPipelineResult of a scan's outputs (and the live path's dict)."""
    X, stamp, z, Lm, h = ctx.get_belief()
    cert = np.array(out.cert[:])
    certs = _certs_from_vector(cert, np.array(out.imu_odom_certs[:]), CHART_ID, belief_prev.anchor_id,
                               live["certs"] if live else None)
    agg = aggregate_certificates(certs)
    bel = BeliefGaussianInfo(CHART_ID, belief_prev.anchor_id, X, stamp, z, Lm, h, certs[-1])
    view = np.ctypeslib.as_array
    res = ScanPipelineResult(
        belief_updated=bel,
        iw_process_dPsi=view(out.iw_process_dPsi).copy().reshape(7, 6, 6),
        iw_process_dnu=view(out.iw_process_dnu).copy(),
        iw_meas_dPsi=view(out.iw_meas_dPsi).copy().reshape(3, 3, 3), iw_meas_dnu=view(out.iw_meas_dnu).copy(),
        iw_lidar_bucket_dPsi=np.zeros((64, 3, 3)), iw_lidar_bucket_dnu=np.zeros(64),
        all_certs=certs, aggregated_cert=agg,
        diagnostics_tape=dict(stage_ms=list(out.stage_ms[:4])),
        map_bins_updated=ctx, z_t=view(out.z_t).copy(), raw_cert=cert,
        L_evidence=view(out.L_evidence).copy().reshape(D_Z, D_Z), h_evidence=view(out.h_evidence).copy(),
        L_imu_odom=view(out.L_imu_odom).copy().reshape(D_Z, D_Z), h_imu_odom=view(out.h_imu_odom).copy())
    if live is not None:
        res.map = live["map"]
        res.measurement_batch = live["batch"]
        res.map_update_cert = live["map_update_cert"]
        res.association = live["association"]
        res.map_view = live["view"]
        res.z_lin_pose = live["z_lin_pose"]
        res.map_record = live["map_record"]
        res.stage_ms = live["stage_ms"]
        res.map_bins_updated = None
    # the reference's per-scan MinimalScanTape (pipeline.py:1504-1570)
    res.diagnostics_tape = tape_from_result(res, scan_seq, scan_end_time, dt_sec, n_raw, res.L_evidence)
    sm = getattr(res, "stage_ms", None) or {}
    if sm:  # the reference's live-path timing fields (diagnostics.py:58-67)
        t = res.diagnostics_tape
        t.t_surfel_extraction_ms = sm.get("surfel_extraction_ms", 0.0)
        t.t_association_ms = sm.get("association_ms", 0.0)
        t.t_visual_pose_ms = sm.get("visual_pose_ms", 0.0)
        t.t_map_branch_ms = sum(sm.get(k, 0.0) for k in ("surfel_extraction_ms", "map_view_ms", "association_ms"))
        t.t_map_update_ms = sm.get("map_update_ms", 0.0)
        t.t_total_ms = sum(sm.values())
    return res


def process_hypotheses(hypotheses: List[BeliefGaussianInfo], weights, config: PipelineConfig):
    """FS/backend/pipeline.py:1594-1621 -> hypothesis_barycenter_projection (hypothesis.py:125-236):
    returns (combined BeliefGaussianInfo, CertBundle, ExpectedEffect).  Host numerics through
    gcs_hypothesis_barycenter: no context, no device, no state change (the IW applies are separate
    calls, as in the node).  The multi-GPU form is gcslam.distributed.combine_allreduce."""
    lib = L.load()
    w = np.ascontiguousarray(weights, np.float64).reshape(-1)
    if len(hypotheses) != config.K_HYP:
        raise ValueError(f"Expected {config.K_HYP} hypotheses, got {len(hypotheses)}")
    if w.shape != (config.K_HYP,):
        raise ValueError(f"Expected weights shape ({config.K_HYP},), got {w.shape}")
    Ls = np.ascontiguousarray(np.stack([b.L for b in hypotheses]), np.float64)
    hs = np.ascontiguousarray(np.stack([b.h for b in hypotheses]), np.float64)
    zs = np.ascontiguousarray(np.stack([b.z_lin for b in hypotheses]), np.float64)
    Lo, ho, zo, c = np.zeros((D_Z, D_Z)), np.zeros(D_Z), np.zeros(D_Z), np.zeros(6)
    L.check(lib.gcs_hypothesis_barycenter(len(hypotheses), L.dptr(Ls), L.dptr(hs), L.dptr(zs), L.dptr(w),
                                          L.dptr(Lo), L.dptr(ho), L.dptr(zo), L.dptr(c)), None,
            "gcs_hypothesis_barycenter")
    t = hypotheses[0]
    wf = np.maximum(w, HYP_WEIGHT_FLOOR)
    wn = wf / wf.sum()
    cert = CertBundle.create_approx(
        CHART_ID, t.anchor_id, ["HypothesisProjection", "I-projection-info-barycenter"],
        conditioning=ConditioningCert(cond=float(c[5])),
        support=SupportCert(ess_total=float(c[2]), support_frac=float(c[3])),
        influence=InfluenceCert(psd_projection_delta=float(c[0]), mass_epsilon_ratio=float(c[1]) / config.K_HYP))
    belief = BeliefGaussianInfo(CHART_ID, t.anchor_id, t.X_anchor, t.stamp_sec, zo, Lo, ho, cert)
    effect = ExpectedEffect("predicted_projection_spread_proxy", float(c[4]), None)
    assert np.isclose(wn.sum(), 1.0)
    return belief, cert, effect


# ---------------------------------------------------------------- node-level noise updates
@dataclass
class ProcessNoiseIWState:
    """FS/backend/structures/inverse_wishart_jax.py:28-39 (7 blocks, dims [3,3,3,3,3,1,6])."""
    nu: np.ndarray
    Psi_blocks: np.ndarray   # (7, 6, 6)


@dataclass
class MeasurementNoiseIWState:
    """FS/backend/structures/measurement_noise_iw_jax.py:29-34 (blocks gyro, accel, lidar)."""
    nu: np.ndarray
    Psi_blocks: np.ndarray   # (3, 3, 3)


def process_noise_iw_apply_suffstats(state: ProcessNoiseIWState, dPsi, dnu):
    """process_noise_iw_apply_suffstats_jax (inverse_wishart_jax.py:126-185) -> (state, cert2)."""
    lib = L.load()
    nu, Psi = np.ascontiguousarray(state.nu, np.float64), np.ascontiguousarray(state.Psi_blocks, np.float64)
    dP, dn = np.ascontiguousarray(dPsi, np.float64), np.ascontiguousarray(dnu, np.float64)
    nu2, Psi2, c = np.zeros(7), np.zeros((7, 6, 6)), np.zeros(2)
    L.check(lib.gcs_process_iw_apply(L.dptr(nu), L.dptr(Psi), L.dptr(dP), L.dptr(dn), L.dptr(nu2), L.dptr(Psi2),
                                     L.dptr(c)), None, "gcs_process_iw_apply")
    return ProcessNoiseIWState(nu2, Psi2), c


def process_noise_state_to_Q(state: ProcessNoiseIWState):
    """process_noise_state_to_Q_jax (inverse_wishart_jax.py:35-68)."""
    lib = L.load()
    nu, Psi = np.ascontiguousarray(state.nu, np.float64), np.ascontiguousarray(state.Psi_blocks, np.float64)
    Q = np.zeros((D_Z, D_Z))
    L.check(lib.gcs_process_noise_Q(L.dptr(nu), L.dptr(Psi), L.dptr(Q)), None, "gcs_process_noise_Q")
    return Q


def measurement_noise_apply_suffstats(state: MeasurementNoiseIWState, dPsi_blocks, dnu):
    """measurement_noise_apply_suffstats_jax (measurement_noise_iw_jax.py:59-100) -> (state, cert2)."""
    lib = L.load()
    nu, Psi = np.ascontiguousarray(state.nu, np.float64), np.ascontiguousarray(state.Psi_blocks, np.float64)
    dP, dn = np.ascontiguousarray(dPsi_blocks, np.float64), np.ascontiguousarray(dnu, np.float64)
    nu2, Psi2, c = np.zeros(3), np.zeros((3, 3, 3)), np.zeros(2)
    L.check(lib.gcs_meas_iw_apply(L.dptr(nu), L.dptr(Psi), L.dptr(dP), L.dptr(dn), L.dptr(nu2), L.dptr(Psi2),
                                  L.dptr(c)), None, "gcs_meas_iw_apply")
    return MeasurementNoiseIWState(nu2, Psi2), c


def measurement_noise_mean(state: MeasurementNoiseIWState, idx: int):
    """measurement_noise_mean_jax (measurement_noise_iw_jax.py:38-56): the IW mode of block idx."""
    lib = L.load()
    nu, Psi = np.ascontiguousarray(state.nu, np.float64), np.ascontiguousarray(state.Psi_blocks, np.float64)
    S = np.zeros((3, 3))
    L.check(lib.gcs_meas_iw_mode(L.dptr(nu), L.dptr(Psi), int(idx), L.dptr(S)), None, "gcs_meas_iw_mode")
    return S


def datasheet_process_noise_state() -> ProcessNoiseIWState:
    """create_datasheet_process_noise_state (structures/inverse_wishart_jax.py:42-80)."""
    dims = (3, 3, 3, 3, 3, 1, 6)
    sig = (1e-4, 8.7e-7, 9.5e-5, 1e-8, 1e-6, 1e-6, 1e-8)   # constants.py:225-237
    Psi = np.zeros((7, 6, 6))
    for i, d in enumerate(dims):
        Psi[i, :d, :d] = np.eye(d) * sig[i] * 0.5
    return ProcessNoiseIWState(np.array(dims, np.float64) + 1.5, Psi)


def datasheet_measurement_noise_state() -> MeasurementNoiseIWState:
    """create_datasheet_measurement_noise_state (structures/measurement_noise_iw_jax.py:37-68)."""
    return MeasurementNoiseIWState(np.full(3, 4.5), np.stack([np.eye(3) * s * 0.5 for s in (8.7e-7, 9.5e-5, 0.01)]))


# ---------------------------------------------------------------- RuntimeManifest
@dataclass
class RuntimeManifest:
    """RuntimeManifest (FS/backend/pipeline.py:1629-1793) for the bin-path backend: the reference's
    constants plus every declared item (tau rule, candidate rule, K, N_POINTS_CAP, map mode,
    pushforward form) and the library's own description of a live context (gcs_ctx_describe)."""
    config: PipelineConfig = field(default_factory=PipelineConfig)
    chart_id: str = CHART_ID
    D_Z: int = D_Z
    D_DESKEW: int = 22
    HYP_WEIGHT_FLOOR: float = HYP_WEIGHT_FLOOR
    eps_r: float = 1e-6
    eps_den: float = 1e-12
    kappa_scale: float = 1.0
    c_dt: float = 1.0
    c_ex: float = 1.0
    MAX_IMU_PREINT_LEN: int = 512
    pose_evidence_backend: str = "bins"       # legacy bin path (README.md:105-122), not primitives
    map_backend: str = "map_bin_stats"
    topics: Dict[str, str] = field(default_factory=dict)
    context_description: Optional[dict] = None

    @classmethod
    def from_context(cls, config: PipelineConfig, ctx: HypothesisContext):
        return cls(config=config, context_description=ctx.describe())

    def to_dict(self) -> dict:
        c = self.config
        d = dict(chart_id=self.chart_id, pose_evidence_backend=self.pose_evidence_backend,
                 map_backend=self.map_backend, topics=dict(self.topics), D_Z=self.D_Z, D_DESKEW=self.D_DESKEW,
                 K_HYP=c.K_HYP, HYP_WEIGHT_FLOOR=self.HYP_WEIGHT_FLOOR, N_POINTS_CAP=c.N_POINTS_CAP,
                 B_BINS=c.B_BINS, soft_assign_mode=c.soft_assign_mode, k_cand=c.k_cand,
                 tau_soft_assign=(c.tau_soft_assign if c.tau_soft_assign is not None else 0.1 * 48.0 / c.B_BINS),
                 tau_rule="tau_B = 0.1 * 48 / B (declared; GC_TAU_SOFT_ASSIGN is undefined in the reference)",
                 candidate_rule=("dense N x B softmax (reference)" if c.soft_assign_mode == "dense" else
                                 "K nearest atlas bins of the exact nearest bin, ties -> lower id (declared)"),
                 map_mode="per-hypothesis MapBinStats (declared)",
                 pushforward_form="declared (DESIGN.md section 3 item 3)",
                 eps_psd=c.eps_psd, eps_lift=c.eps_lift, eps_mass=c.eps_mass, eps_r=self.eps_r, eps_den=self.eps_den,
                 alpha_min=c.alpha_min, alpha_max=c.alpha_max, kappa_scale=self.kappa_scale, c0_cond=c.c0_cond,
                 c_dt=self.c_dt, c_ex=self.c_ex, c_frob=c.c_frob, imu_gravity_scale=c.imu_gravity_scale,
                 deskew_rotation_only=c.deskew_rotation_only, power_beta_min=c.power_beta_min,
                 power_beta_exc_c=c.power_beta_exc_c, power_beta_z_c=c.power_beta_z_c,
                 enable_parallel_stages=False, MAX_IMU_PREINT_LEN=self.MAX_IMU_PREINT_LEN,
                 backends={"core_array": "HIP (gfx950) + host C++", "library": L.load().gcs_version().decode()})
        if self.context_description is not None:
            d["context"] = self.context_description
        return d

    def to_json(self) -> str:
        return json.dumps(self.to_dict())
