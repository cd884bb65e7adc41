"""L2 drop-in: process_scan_single_hypothesis / process_hypotheses with the reference calling
convention (FS/backend/pipeline.py:316-340, :1594-1621), running the 14-step bin path
(README.md:105-122) on the MI355X through libgcslam_hip.so.

`primitive_map` is replaced by `map_bins`, a HypothesisContext that owns the device-resident
MapBinStats of this hypothesis (the legacy pipeline took bin_atlas/map_stats, CHANGELOG.md:280).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .certificates import CertBundle, InfluenceCert, SupportCert, aggregate_certificates
from .context import HypothesisContext
from .outputs import tape_from_result

CHART_ID = "GC-RIGHT-01"
D_Z = 22


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
    c_frob: float = 1.0
    forgetting_factor: float = 0.99
    deskew_rotation_only: bool = False
    lidar_origin_base: tuple = (0.0, 0.0, 0.0)
    gravity_W: tuple = (0.0, 0.0, -9.81)
    max_raw_points: int = 1 << 20
    device: int = 0

    def make_context(self) -> HypothesisContext:
        return HypothesisContext(n_bins=self.B_BINS, n_points_cap=self.N_POINTS_CAP,
                                 max_raw_points=self.max_raw_points, mode=self.soft_assign_mode, k_cand=self.k_cand,
                                 tau=self.tau_soft_assign, lidar_origin=self.lidar_origin_base,
                                 deskew_rotation_only=self.deskew_rotation_only,
                                 forgetting_factor=self.forgetting_factor, gravity_W=self.gravity_W,
                                 device=self.device)


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


def _certs_from_vector(c, chart, anchor):
    """Rebuild the per-operator certificates from the scan's cert vector (DESIGN.md cert slots)."""
    I = InfluenceCert
    return [
        CertBundle.create_approx(chart, anchor, ["PointBudgetResample"], support=SupportCert(c[0], c[1]),
                                 influence=I(mass_epsilon_ratio=c[2])),
        CertBundle.create_approx(chart, anchor, ["PredictDiffusion"],
                                 influence=I(lift_strength=c[6], psd_projection_delta=c[7], dt_scale=c[8])),
        CertBundle.create_exact(chart, anchor, support=SupportCert(c[10], c[9])),
        CertBundle.create_exact(chart, anchor, support=SupportCert(c[12], c[13])),
        CertBundle.create_approx(chart, anchor, ["ScanBinMomentMatch"], support=SupportCert(c[14], c[15]),
                                 influence=I(psd_projection_delta=c[16], mass_epsilon_ratio=c[17])),
        CertBundle.create_approx(chart, anchor, ["MatrixFisherRotationEvidence"],
                                 influence=I(psd_projection_delta=c[18], mass_epsilon_ratio=c[19])),
        CertBundle.create_approx(chart, anchor, ["PlanarTranslationEvidence"],
                                 influence=I(psd_projection_delta=c[25], mass_epsilon_ratio=c[26])),
        CertBundle.create_approx(chart, anchor, ["PowerTempering"], influence=I(power_beta=c[30])),
        CertBundle.create_approx(chart, anchor, ["ExcitationPriorScaling"],
                                 influence=I(dt_scale=1.0 - c[31], extrinsic_scale=1.0 - c[32])),
        CertBundle.create_exact(chart, anchor, influence=I(trust_alpha=c[33])),
        CertBundle.create_approx(chart, anchor, ["InfoFusionAdditive"],
                                 influence=I(psd_projection_delta=c[34], trust_alpha=c[33])),
        CertBundle.create_approx(chart, anchor, ["PoseUpdateFrobeniusRecompose"], frobenius_applied=c[36] > 0),
        CertBundle.create_approx(chart, anchor, ["AnchorDriftUpdate"], influence=I(anchor_drift_rho=c[37])),
    ]


def _as_device_scan(raw_points, raw_timestamps, raw_weights, device):
    import torch
    dev = f"cuda:{device}"
    if isinstance(raw_points, torch.Tensor) and raw_points.dim() == 2 and raw_points.shape[1] == 4 \
            and raw_points.dtype == torch.float32:
        rec = raw_points.to(dev)
    else:
        p = torch.as_tensor(np.asarray(raw_points), dtype=torch.float64).reshape(-1, 3)
        rec = torch.zeros((p.shape[0], 4), dtype=torch.float32)
        rec[:, :3] = p.to(torch.float32)   # PointCloud2 x,y,z are float32 (backend_node.py:377-468)
        rec = rec.to(dev)
    t = torch.as_tensor(np.asarray(raw_timestamps, np.float64) if not isinstance(raw_timestamps, torch.Tensor)
                        else raw_timestamps, dtype=torch.float64).to(dev).contiguous()
    w = torch.as_tensor(np.asarray(raw_weights, np.float64) if not isinstance(raw_weights, torch.Tensor)
                        else raw_weights, dtype=torch.float64).to(dev).contiguous()
    return rec.contiguous(), t, w


def process_scan_single_hypothesis(belief_prev: BeliefGaussianInfo, raw_points, raw_timestamps, raw_weights,
                                   raw_ring, raw_tag, imu_stamps, imu_gyro, imu_accel, odom_pose, odom_cov_se3,
                                   scan_start_time, scan_end_time, dt_sec, t_last_scan, t_scan, Q,
                                   config: PipelineConfig, odom_twist=None, odom_twist_cov=None, camera_batch=None,
                                   scan_seq=0, map_bins: Optional[HypothesisContext] = None,
                                   L_ext=None, h_ext=None) -> ScanPipelineResult:
    """FS/backend/pipeline.py:316-1591 with the bin path of README.md:105-122.

    odom/IMU evidence factors (pipeline.py:595-776) are not computed this round; callers may pass
    their summed information as L_ext/h_ext (DESIGN.md "out of scope")."""
    ctx = map_bins if map_bins is not None else config.make_context()
    ctx.set_belief(belief_prev.X_anchor, belief_prev.stamp_sec, belief_prev.z_lin, belief_prev.L, belief_prev.h)
    rec, t, w = _as_device_scan(raw_points, raw_timestamps, raw_weights, config.device)
    out = ctx.scan(rec, 16, t, w, rec.shape[0], imu_stamps, imu_gyro, imu_accel, scan_start_time, scan_end_time,
                   dt_sec, Q=Q, L_ext=L_ext, h_ext=h_ext, t_last_scan=t_last_scan, t_scan=t_scan)
    X, stamp, z, Lm, h = ctx.get_belief()
    cert = np.array(out.cert[:])
    certs = _certs_from_vector(cert, CHART_ID, belief_prev.anchor_id)
    agg = aggregate_certificates(certs)
    bel = BeliefGaussianInfo(CHART_ID, belief_prev.anchor_id, X, stamp, z, Lm, h, certs[-1])
    res = ScanPipelineResult(
        belief_updated=bel,
        iw_process_dPsi=np.array(out.iw_process_dPsi[:]).reshape(7, 6, 6),
        iw_process_dnu=np.array(out.iw_process_dnu[:]),
        iw_meas_dPsi=np.array(out.iw_meas_dPsi[:]).reshape(3, 3, 3), iw_meas_dnu=np.array(out.iw_meas_dnu[:]),
        iw_lidar_bucket_dPsi=np.zeros((64, 3, 3)), iw_lidar_bucket_dnu=np.zeros(64),
        all_certs=certs, aggregated_cert=agg,
        diagnostics_tape=dict(stage_ms=list(out.stage_ms[:4])),
        map_bins_updated=ctx, z_t=np.array(out.z_t[:]), raw_cert=cert)
    # the reference's per-scan MinimalScanTape (pipeline.py:1504-1570)
    res.diagnostics_tape = tape_from_result(res, scan_seq, scan_end_time, dt_sec, rec.shape[0],
                                            np.array(out.L_evidence[:]))
    return res


def process_hypotheses(hypotheses: List[BeliefGaussianInfo], weights, config: PipelineConfig,
                       ctx: Optional[HypothesisContext] = None):
    """FS/backend/pipeline.py:1594-1621 -> hypothesis_barycenter_projection (hypothesis.py:51-117),
    single-process form: sum the per-hypothesis payloads on the host (the multi-GPU form is
    gcslam.distributed.combine_allreduce)."""
    from . import _lib as L
    w = np.maximum(np.asarray(weights, np.float64), 0.0025)
    wn = w / w.sum()
    total = np.zeros(L.PAYLOAD_LEN)
    own = ctx is None
    ctx = ctx or config.make_context()
    for k, b in enumerate(hypotheses):
        ctx.set_belief(b.X_anchor, b.stamp_sec, b.z_lin, b.L, b.h)
        total += ctx.hypothesis_payload(float(weights[k]), float(wn[k]))
    (X, stamp, z, Lm, h), cert = ctx.hypothesis_combine(total, 0)
    if own:
        ctx.close()
    return BeliefGaussianInfo(CHART_ID, hypotheses[0].anchor_id, hypotheses[0].X_anchor, hypotheses[0].stamp_sec,
                              z, Lm, h), cert
