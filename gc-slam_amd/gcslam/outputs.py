"""Output formats after the path: the TUM trajectory line the node writes
(FS/backend/backend_node.py:2212-2221 pose export, :2287-2293 line format) and the minimal
per-scan diagnostics tape (FS/backend/diagnostics.py:19-160 MinimalScanTape, :163-267
DiagnosticsLog.save_npz / save_jsonl), filled from a ScanPipelineResult of this build.  Host
formatting only; the poses and certificates come from the device pipeline."""

from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field, fields
from typing import List, Optional

import numpy as np

EPS_PSD = 1e-12


def _so3_exp(w):
    th = math.sqrt(float(w @ w))
    K = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + math.sin(th) / th * K + (1.0 - math.cos(th)) / (th * th) * (K @ K)


def se3_compose(a, b):
    """[t, rotvec] composition a ∘ b (se3_jax.py se3_compose): R = Ra Rb, t = ta + Ra tb."""
    Ra, Rb = _so3_exp(np.asarray(a[3:], float)), _so3_exp(np.asarray(b[3:], float))
    R = Ra @ Rb
    t = np.asarray(a[:3], float) + Ra @ np.asarray(b[:3], float)
    return np.concatenate([t, rotvec_from_R(R)])


def rotvec_from_R(R):
    c = min(1.0, max(-1.0, (np.trace(R) - 1.0) * 0.5))
    th = math.acos(c)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    if th < 1e-12:
        return 0.5 * v
    if math.pi - th < 1e-6:  # near pi: axis from the symmetric part
        A = (R + np.eye(3)) * 0.5
        k = int(np.argmax(np.diag(A)))
        axis = A[:, k] / math.sqrt(max(A[k, k], 1e-300))
        if axis @ v < 0:
            axis = -axis
        return axis * th
    return v * (th / (2.0 * math.sin(th)))


def quat_xyzw_from_rotvec(rv):
    """scipy Rotation.from_rotvec(rv).as_quat(): (x, y, z, w), w = cos(theta/2) >= 0."""
    rv = np.asarray(rv, float)
    th = math.sqrt(float(rv @ rv))
    s = 0.5 - th * th / 48.0 if th < 1e-6 else math.sin(0.5 * th) / th
    return np.array([rv[0] * s, rv[1] * s, rv[2] * s, math.cos(0.5 * th)])


def tum_line(stamp_sec, pose6, anchor_correction=None):
    """One TUM line for the exported pose anchor_correction ∘ pose (backend_node.py:2212-2221,2287-2293)."""
    pose = np.asarray(pose6, float)
    if anchor_correction is not None:
        pose = se3_compose(np.asarray(anchor_correction, float), pose)
    t, q = pose[:3], quat_xyzw_from_rotvec(pose[3:])
    return (f"{stamp_sec:.9f} {t[0]:.6f} {t[1]:.6f} {t[2]:.6f} "
            f"{q[0]:.6f} {q[1]:.6f} {q[2]:.6f} {q[3]:.6f}\n")


class TumTrajectoryWriter:
    """The node's trajectory_file: one flushed TUM line per exported pose."""

    def __init__(self, path):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "w")

    def write(self, stamp_sec, pose6, anchor_correction=None):
        self._f.write(tum_line(stamp_sec, pose6, anchor_correction))
        self._f.flush()

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


@dataclass
class MinimalScanTape:
    """diagnostics.py:19-160 (same fields and order)."""
    scan_number: int
    timestamp: float
    dt_sec: float
    n_points_raw: int
    n_points_budget: int
    fusion_alpha: float
    cond_pose6: float
    conditioning_number: float
    eigmin_pose6: float
    L_pose6: np.ndarray
    total_trigger_magnitude: float
    cert_exact: bool
    cert_frobenius_applied: bool
    cert_n_triggers: int
    support_ess_total: float
    support_frac: float
    mismatch_nll_per_ess: float
    mismatch_directional_score: float
    excitation_dt_effect: float
    excitation_extrinsic_effect: float
    influence_psd_projection_delta: float
    influence_mass_epsilon_ratio: float
    influence_anchor_drift_rho: float
    influence_dt_scale: float
    influence_extrinsic_scale: float
    influence_trust_alpha: float
    influence_power_beta: float
    overconfidence_excitation_total: float
    overconfidence_ess_to_excitation: float
    overconfidence_cond_to_support: float
    overconfidence_dt_asymmetry: float
    overconfidence_z_to_xy_ratio: float
    t_total_ms: float = 0.0
    t_point_budget_ms: float = 0.0
    t_deskew_ms: float = 0.0
    t_imu_preint_scan_ms: float = 0.0
    t_imu_preint_int_ms: float = 0.0
    t_surfel_extraction_ms: float = 0.0
    t_association_ms: float = 0.0
    t_visual_pose_ms: float = 0.0
    t_map_branch_ms: float = 0.0
    t_map_update_ms: float = 0.0

    def to_dict(self):
        d = asdict(self)
        d["L_pose6"] = np.asarray(self.L_pose6).tolist()
        return d

    @classmethod
    def from_dict(cls, d):
        d = dict(d)
        d["L_pose6"] = np.asarray(d["L_pose6"], float)
        return cls(**{f.name: d[f.name] for f in fields(cls) if f.name in d})


def pose_conditioning(L_evidence):
    """Pose-block conditioning (pipeline.py:1155-1168): eigvalsh of sym(L[0:6, 0:6]) clipped at eps."""
    Lp = np.nan_to_num(0.5 * (L_evidence[:6, :6] + L_evidence[:6, :6].T), nan=0.0, posinf=0.0, neginf=0.0)
    ev = np.maximum(np.nan_to_num(np.linalg.eigvalsh(Lp), nan=EPS_PSD, posinf=EPS_PSD, neginf=EPS_PSD), EPS_PSD)
    return float(ev[0]), float(ev[-1]), float(ev[-1] / ev[0])


def tape_from_result(result, scan_number, scan_end_time, dt_sec, n_points_raw, L_evidence):
    """A MinimalScanTape from gcslam.pipeline.ScanPipelineResult (pipeline.py:1504-1570).  Fields
    with no producer on the bin path (mismatch, excitation totals, surfel/association timings)
    keep the reference's neutral values."""
    c = np.asarray(result.raw_cert)
    agg = result.aggregated_cert
    eig_min, _, cond = pose_conditioning(np.asarray(L_evidence).reshape(22, 22))
    inf = agg.influence
    stage = (result.diagnostics_tape or {}).get("stage_ms", [0.0] * 4)
    return MinimalScanTape(
        scan_number=int(scan_number), timestamp=float(scan_end_time), dt_sec=float(dt_sec),
        n_points_raw=int(n_points_raw), n_points_budget=int(c[4]), fusion_alpha=float(c[33]),
        cond_pose6=cond, conditioning_number=float(agg.conditioning.cond if agg.conditioning else 1.0),
        eigmin_pose6=eig_min, L_pose6=np.asarray(L_evidence).reshape(22, 22)[:6, :6].copy(),
        total_trigger_magnitude=float(c[35]), cert_exact=bool(agg.exact),
        cert_frobenius_applied=bool(agg.frobenius_applied), cert_n_triggers=len(agg.approximation_triggers),
        support_ess_total=float(agg.support.ess_total), support_frac=float(agg.support.support_frac),
        mismatch_nll_per_ess=float(agg.mismatch.nll_per_ess),
        mismatch_directional_score=float(agg.mismatch.directional_score),
        excitation_dt_effect=float(c[31]), excitation_extrinsic_effect=float(c[32]),
        influence_psd_projection_delta=float(inf.psd_projection_delta),
        influence_mass_epsilon_ratio=float(inf.mass_epsilon_ratio),
        influence_anchor_drift_rho=float(inf.anchor_drift_rho), influence_dt_scale=float(inf.dt_scale),
        influence_extrinsic_scale=float(inf.extrinsic_scale), influence_trust_alpha=float(inf.trust_alpha),
        influence_power_beta=float(inf.power_beta), overconfidence_excitation_total=0.0,
        overconfidence_ess_to_excitation=0.0, overconfidence_cond_to_support=0.0,
        overconfidence_dt_asymmetry=float(c[39]), overconfidence_z_to_xy_ratio=float(c[40]),
        t_total_ms=float(stage[3]), t_point_budget_ms=float(stage[1]), t_deskew_ms=0.0,
        t_imu_preint_scan_ms=float(stage[0]))


_NPZ_KEYS = [("scan_numbers", "scan_number"), ("timestamps", "timestamp"), ("dt_secs", "dt_sec")]


@dataclass
class DiagnosticsLog:
    """diagnostics.py:163-267: the minimal tape, saved as npz ("minimal_tape") or JSON lines."""
    tape: List[MinimalScanTape] = field(default_factory=list)
    run_id: str = ""
    start_time: float = 0.0
    end_time: float = 0.0
    total_scans: int = 0

    def append_tape(self, entry: MinimalScanTape) -> None:
        self.tape.append(entry)
        self.total_scans = len(self.tape)

    def save_jsonl(self, path: str) -> None:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            f.write(json.dumps({"_type": "header", "run_id": self.run_id, "start_time": self.start_time,
                                "total_scans": self.total_scans}) + "\n")
            for e in self.tape:
                f.write(json.dumps(e.to_dict()) + "\n")

    @classmethod
    def load_jsonl(cls, path: str) -> "DiagnosticsLog":
        log = cls()
        with open(path) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                d = json.loads(line)
                if d.get("_type") == "header":
                    log.run_id, log.start_time = d.get("run_id", ""), d.get("start_time", 0.0)
                else:
                    log.tape.append(MinimalScanTape.from_dict(d))
        log.total_scans = len(log.tape)
        return log

    def save_npz(self, path: str) -> None:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        n = len(self.tape)
        if n == 0:
            np.savez_compressed(path, format="minimal_tape", n_scans=0)
            return
        data = {"format": "minimal_tape", "n_scans": n, "run_id": self.run_id, "start_time": self.start_time}
        for key, attr in _NPZ_KEYS:
            data[key] = np.array([getattr(t, attr) for t in self.tape])
        for f in fields(MinimalScanTape):
            if f.name in ("scan_number", "timestamp", "dt_sec"):
                continue
            vals = [getattr(t, f.name) for t in self.tape]
            data[f.name] = np.stack(vals) if f.name == "L_pose6" else np.array(vals)
        np.savez_compressed(path, **data)


# ---------------------------------------------------------------- trajectory error (evaluation side)
def pose6_to_matrix(pose6):
    """[t, rotvec] -> 4x4 homogeneous transform."""
    p = np.asarray(pose6, float)
    T = np.eye(4)
    T[:3, :3] = _so3_exp(p[3:])
    T[:3, 3] = p[:3]
    return T


def associate_stamps(t_ref, t_est, max_diff=0.01):
    """Index pairs (i_ref, i_est) of stamps within max_diff, each est stamp used once, in ref order
    (evo sync.associate_trajectories, as called by tools/evaluate_slam.py:254)."""
    t_ref, t_est = np.asarray(t_ref, float), np.asarray(t_est, float)
    pairs, used = [], set()
    for i, t in enumerate(t_ref):
        if t_est.size == 0:
            break
        j = int(np.argmin(np.abs(t_est - t)))
        if abs(t_est[j] - t) <= max_diff and j not in used:
            used.add(j)
            pairs.append((i, j))
    return pairs


def align_initial(T_gt, T_est):
    """tools/evaluate_slam.py:220-232: GT moved into the estimate frame so that the first associated
    GT pose equals the first estimate (T_gt_i <- T_est0 T_gt0^-1 T_gt_i)."""
    if len(T_gt) == 0 or len(T_est) == 0:
        return [np.array(T) for T in T_gt]
    A = np.asarray(T_est[0], float) @ np.linalg.inv(np.asarray(T_gt[0], float))
    return [A @ np.asarray(T, float) for T in T_gt]


def align_umeyama(T_gt, T_est):
    """SE(3) Umeyama fit of the estimate positions to GT, scale fixed (evo PoseTrajectory3D.align
    with correct_scale=False, tools/evaluate_slam.py:260); returns the aligned estimate poses."""
    X = np.array([np.asarray(T, float)[:3, 3] for T in T_est])
    Y = np.array([np.asarray(T, float)[:3, 3] for T in T_gt])
    mx, my = X.mean(0), Y.mean(0)
    S = (Y - my).T @ (X - mx) / len(X)
    U, _, Vt = np.linalg.svd(S)
    D = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        D[2, 2] = -1.0
    R = U @ D @ Vt
    A = np.eye(4)
    A[:3, :3] = R
    A[:3, 3] = my - R @ mx
    return [A @ np.asarray(T, float) for T in T_est]


def _stats(e):
    e = np.asarray(e, float)
    return dict(rmse=float(np.sqrt(np.mean(e * e))), mean=float(e.mean()), median=float(np.median(e)),
                std=float(e.std()), min=float(e.min()), max=float(e.max()), sse=float(np.sum(e * e)))


def ate(stamps_gt, poses_gt, stamps_est, poses_est, align="initial", max_diff=0.01):
    """Absolute trajectory error as tools/evaluate_slam.py:235-270 computes it with evo: associate
    by stamp, align ("initial": GT into the estimate frame at the first pose; "umeyama": SE(3)
    fit, no scale), then APE of E_i = P_gt_i^-1 P_est_i: translation |t(E_i)| (m) and rotation
    angle |angle(R(E_i))| (deg).  Poses are [t, rotvec] rows or 4x4 matrices."""
    def mats(P):
        P = np.asarray(P, float)
        return [T for T in P] if P.ndim == 3 else [pose6_to_matrix(p) for p in P]
    Tg, Te = mats(poses_gt), mats(poses_est)
    pairs = associate_stamps(stamps_gt, stamps_est, max_diff)
    if not pairs:
        raise ValueError("no associated poses")
    Tg = [Tg[i] for i, _ in pairs]
    Te = [Te[j] for _, j in pairs]
    if align == "initial":
        Tg = align_initial(Tg, Te)
    elif align == "umeyama":
        Te = align_umeyama(Tg, Te)
    elif align != "none":
        raise ValueError(f"align must be 'initial', 'umeyama' or 'none', got {align!r}")
    et, er = [], []
    for A, B in zip(Tg, Te):
        E = np.linalg.inv(A) @ B
        et.append(float(np.linalg.norm(E[:3, 3])))
        c = min(1.0, max(-1.0, (np.trace(E[:3, :3]) - 1.0) * 0.5))
        er.append(math.degrees(math.acos(c)))
    return dict(align=align, n=len(pairs), trans=_stats(et), rot_deg=_stats(er))
