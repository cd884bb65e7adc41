"""The 14-step bin-path per-scan pipeline, one hypothesis (test oracle only).

Step order follows README.md:105-122 with the live calling convention of
process_scan_single_hypothesis (FS/backend/pipeline.py:316-1591); see SURVEY.md
section 3.3 for the reconstruction.  Step 9 sums the LiDAR bin evidence with the IMU/odometry
evidence family (pipeline.py:595-776, oracle/imu_odom.py) and an optional external (L, h) term.
Scans without t_last_scan / t_scan keys use the scan window (scan_start_time, scan_end_time) for
the scan-to-scan IMU window; scans without odometry get the node's "no odometry yet" inputs
(identity pose, 1e12 I covariances; backend_node.py:939-940,2047-2051).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import imu_odom, ops, se3
from .primitives import psd_project, spd_inverse_lifted, spd_solve_lifted


@dataclass
class BinPathConfig:
    n_points_cap: int = 8192
    n_bins: int = 48
    mode: str = "dense"            # "dense" (reference N x B softmax) or "scale" (K candidates)
    k_cand: int = ops.K_CAND
    tau: float | None = None       # None -> ops.tau_for_bins(n_bins)
    lidar_origin: tuple = (0.0, 0.0, 0.0)
    deskew_rotation_only: bool = False
    forgetting_factor: float = ops.FORGETTING_FACTOR
    gravity_W: tuple = ops.GRAVITY_W
    # sensitivity of the declared pushforward inflation form: the pose
    # covariance J Sigma J^T enters scaled by this factor (1.0: the declared form)
    pushforward_inflation_scale: float = 1.0
    # step 9 IMU/odometry family (PipelineConfig, FS/backend/pipeline.py:96-223)
    use_imu_odom: bool = True
    planar_z_ref: float = imu_odom.PLANAR_Z_REF
    planar_z_sigma: float = imu_odom.PLANAR_Z_SIGMA
    planar_vz_sigma: float = imu_odom.PLANAR_VZ_SIGMA
    alpha_min: float = imu_odom.ALPHA_MIN
    alpha_max: float = imu_odom.ALPHA_MAX
    c0_cond: float = imu_odom.C0_COND

    def temperature(self):
        return ops.tau_for_bins(self.n_bins) if self.tau is None else self.tau


@dataclass
class MapState:
    stats: ops.MapBinStats
    mu_dir: np.ndarray
    kappa: np.ndarray
    centroid: np.ndarray
    Sigma_c: np.ndarray

    @classmethod
    def empty(cls, B):
        st = ops.MapBinStats.empty(B)
        return cls(st, *ops.map_derived_stats(st))


def _aggregate_ess(certs):
    return sum(c.get("ess_total", 0.0) for c in certs) / len(certs)


def scan_odometry(scan):
    """Odometry inputs of a scan, or the node's defaults when it carries none."""
    big = imu_odom.ODOM_COV_MISSING * np.eye(6)
    return (np.asarray(scan.get("odom_pose", np.zeros(6)), np.float64),
            np.asarray(scan.get("odom_cov_se3", big), np.float64),
            np.asarray(scan.get("odom_twist", np.zeros(6)), np.float64),
            np.asarray(scan.get("odom_twist_cov", big), np.float64))


def _scan_prologue(belief_prev: ops.Belief, scan: dict, Q, cfg, meas_state=None, Sigma_g=None, Sigma_a=None):
    """Steps 1-3 and the step-9 IMU/odometry branch, shared by the bin path and the live primitive
    path (pipeline.py:399-776).  Returns the state the LiDAR evidence and the tail read."""
    certs = []   # list of dicts: influence fields + ess_total (+ name)
    # 1 PointBudgetResample (pipeline.py:399-418)
    bud = ops.point_budget_resample(scan["points"], scan["timestamps"], scan["weights"],
                                    n_points_cap=cfg.n_points_cap)
    certs.append(dict(name="budget", mass_epsilon_ratio=bud["mass_epsilon_ratio"], ess_total=bud["ess"]))
    # 2 PredictDiffusion (pipeline.py:423-430)
    b_pred, infl = ops.predict_diffusion(belief_prev, Q, scan["dt_sec"])
    certs.append(dict(name="predict", **infl))
    # 3 IMU window, preintegration, deskew (pipeline.py:432-587)
    cov_pred, _ = spd_inverse_lifted(b_pred.L, ops.EPS_LIFT)
    sigma_warp = max(math.sqrt(cov_pred[15, 15]), 0.01)
    w_imu = ops.smooth_window_weights(scan["imu_stamps"], scan["scan_start_time"], scan["scan_end_time"],
                                      sigma_warp)
    mu_inc = b_pred.mean_increment()
    pose0 = belief_prev.mean_world_pose()
    pre = ops.preintegrate_imu(scan["imu_stamps"], scan["imu_gyro"], scan["imu_accel"], w_imu, pose0[3:6],
                               mu_inc[9:12], mu_inc[12:15], np.asarray(cfg.gravity_W))
    xi = se3.se3_log(pre["delta_pose"])
    # measurement-noise IW statistics over the scan-to-scan window (pipeline.py:448-453,522-566)
    t_last, t_scan = scan.get("t_last_scan", scan["scan_start_time"]), scan.get("t_scan", scan["scan_end_time"])
    w_int = ops.smooth_window_weights(scan["imu_stamps"], t_last, t_scan, sigma_warp)
    meas_dPsi, meas_dnu = ops.imu_meas_iw_suffstats(scan["imu_stamps"], scan["imu_gyro"], scan["imu_accel"], w_int,
                                                    mu_inc[9:12], mu_inc[12:15], pose0[3:6],
                                                    np.asarray(cfg.gravity_W))
    if cfg.deskew_rotation_only:
        xi[:3] = 0.0
    dk = ops.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"],
                                   scan["scan_start_time"], scan["scan_end_time"], xi)
    cert_deskew = dict(name="deskew", ess_total=pre["ess"])
    certs.append(cert_deskew)
    # step 9 IMU + odometry evidence (pipeline.py:595-776)
    io = None
    if cfg.use_imu_odom:
        if meas_state is None:
            meas_state = ops.datasheet_measurement_noise_state()
        Sg = imu_odom.measurement_noise_mean(*meas_state, 0) if Sigma_g is None else np.asarray(Sigma_g)
        Sa = imu_odom.measurement_noise_mean(*meas_state, 1) if Sigma_a is None else np.asarray(Sigma_a)
        dt_int = imu_odom.compute_imu_integration_time(scan["imu_stamps"], t_last, t_scan)
        dt_imu, omega_avg = imu_odom.dt_imu_and_omega_avg(scan["imu_stamps"], scan["imu_gyro"], w_int, mu_inc[9:12])
        pre_int = ops.preintegrate_imu(scan["imu_stamps"], scan["imu_gyro"], scan["imu_accel"], w_int, pose0[3:6],
                                       mu_inc[9:12], mu_inc[12:15], np.asarray(cfg.gravity_W))
        op, oc, ot, otc = scan_odometry(scan)
        L_io, h_io, io_certs, io_named, io_info = imu_odom.imu_odom_branch(
            pose0=pose0, pose_pred=b_pred.mean_world_pose(), mu_prev=belief_prev.mean_increment(), mu_inc=mu_inc,
            imu_stamps=scan["imu_stamps"], imu_gyro=scan["imu_gyro"], imu_accel=scan["imu_accel"], w_int=w_int,
            dt_imu=dt_imu, omega_avg=omega_avg, dt_int=dt_int, pre_int=pre_int, gravity_W=np.asarray(cfg.gravity_W),
            Sigma_g=Sg, Sigma_a=Sa, odom_pose=op, odom_cov=oc, odom_twist=ot, odom_twist_cov=otc,
            dt_sec=scan["dt_sec"], planar_z_ref=cfg.planar_z_ref, planar_z_sigma=cfg.planar_z_sigma,
            planar_vz_sigma=cfg.planar_vz_sigma)
        certs.extend(io_certs)
        io = dict(L=L_io, h=h_io, certs=io_certs, named=io_named, info=io_info, dt_int=dt_int, dt_imu=dt_imu,
                  omega_avg=omega_avg, pre_int=pre_int)
    return dict(certs=certs, bud=bud, b_pred=b_pred, pre=pre, xi=xi, dk=dk, cert_deskew=cert_deskew, io=io,
                meas_dPsi=meas_dPsi, meas_dnu=meas_dnu, pose_pred=b_pred.mean_world_pose())


def _scan_tail(st, cfg, L_lidar, h_lidar, ev_ess, ev_nll, L_ext=None, h_ext=None):
    """Steps 9 (evidence sum, power tempering, excitation scaling) to 12 (recompose) and the process
    IW statistics (pipeline.py:1038-1230).  ev_ess / ev_nll: support.ess_total / mismatch.nll_per_ess
    of aggregate(LiDAR certs)."""
    certs, io, b_pred = st["certs"], st["io"], st["b_pred"]
    L_raw = L_lidar + (0.0 if L_ext is None else L_ext) + (0.0 if io is None else io["L"])
    h_raw = h_lidar + (0.0 if h_ext is None else h_ext) + (0.0 if io is None else io["h"])
    eps = ops.EPS_MASS
    dt_pose = np.linalg.norm(L_raw[15, 0:6]) + np.linalg.norm(L_raw[0:6, 15])
    dt_vel = np.linalg.norm(L_raw[15, 6:9]) + np.linalg.norm(L_raw[6:9, 15])
    dt_asym = min(max(abs(dt_vel - dt_pose) / (dt_vel + dt_pose + eps), 0.0), 1.0)
    z_to_xy = abs(L_raw[2, 2]) / (0.5 * (abs(L_raw[0, 0]) + abs(L_raw[1, 1])) + eps)
    # combined evidence cert = aggregate([aggregate(lidar certs), odom, imu, gyro]) (pipeline.py:1057-1067)
    if io is None:
        ess_total, nll_total = ev_ess, ev_nll
    else:
        named = io["named"]
        ess_total = (ev_ess + named["odom"]["ess_total"] + named["imu"]["ess_total"] + named["gyro"]["ess_total"]) / 4.0
        nll_total = ev_nll + named["odom"]["nll_per_ess"] + named["imu"]["nll_per_ess"] + named["gyro"]["nll_per_ess"]
    exc_total = 0.0   # no reference operator fills an ExcitationCert (certificates.py:564-567 aggregates zeros)
    ess_to_exc = ess_total / (exc_total + eps)
    s_z = z_to_xy / (z_to_xy + ops.POWER_BETA_Z_C)
    s_exc = 1.0 / (1.0 + ess_to_exc / ops.POWER_BETA_EXC_C)
    s = min(max(dt_asym * s_z * s_exc, 0.0), 1.0)
    beta = ops.POWER_BETA_MIN + (1.0 - ops.POWER_BETA_MIN) * s
    beta = min(max(beta, ops.POWER_BETA_MIN), 1.0)
    L_ev, h_ev = beta * L_raw, beta * h_raw
    certs.append(dict(name="temper", power_beta=beta))
    s_dt, s_ex = ops.excitation_scales(L_ev, b_pred.L)
    Lp, hp = ops.apply_excitation_scaling(b_pred.L, b_pred.h, s_dt, s_ex)
    certs.append(dict(name="excitation", dt_scale=1.0 - s_dt, extrinsic_scale=1.0 - s_ex))
    b_pred = ops.Belief(b_pred.X_anchor, b_pred.stamp_sec, b_pred.z_lin, Lp, hp)
    # 10 FusionScaleFromCertificates with the pose-6 conditioning of the tempered evidence
    # (pipeline.py:1150-1192, fusion.py:46-142)
    cond6 = imu_odom.pose6_conditioning(L_ev)
    alpha, quality = imu_odom.fusion_scale_from_certificates(
        dict(cond=cond6["cond"], ess_total=ess_total, nll_per_ess=nll_total, power_beta=beta),
        alpha_min=cfg.alpha_min, alpha_max=cfg.alpha_max, c0_cond=cfg.c0_cond, excitation_total=exc_total,
        dt_asymmetry=dt_asym, z_to_xy_ratio=z_to_xy)
    certs.append(dict(name="fusion_scale", trust_alpha=alpha))
    # 11 InfoFusionAdditive
    b_post, infl = ops.info_fusion_additive(b_pred, L_ev, h_ev, alpha)
    certs.append(dict(name="fusion", **infl))
    # 12 PoseUpdateFrobeniusRecompose (T = sum of trigger magnitudes, pipeline.py:1211)
    T = sum(ops.trigger_magnitude(c) for c in certs)
    b_rec, rinfo = ops.frobenius_recompose(b_post, T)
    certs.append(dict(name="recompose"))
    dPsi, dnu = ops.process_noise_iw_suffstats(b_pred.L, b_pred.h, b_rec.L, b_rec.h)
    return dict(b_rec=b_rec, b_post=b_post, L_evidence=L_ev, h_evidence=h_ev, beta=beta, total_trigger=T,
                frobenius_strength=rinfo["frobenius_strength"], z_t=b_rec.mean_world_pose(), alpha=alpha,
                fusion_quality=quality, cond_pose6=cond6, ess_total=ess_total, nll_total=nll_total,
                iw_process_dPsi=dPsi, iw_process_dnu=dnu)


def process_scan_bin_path(belief_prev: ops.Belief, scan: dict, Q, cfg: BinPathConfig, bins, knn,
                          map_state: MapState, L_ext=None, h_ext=None, meas_state=None, Sigma_g=None, Sigma_a=None):
    """One hypothesis, one scan.  `scan` keys: points (N,3), timestamps, weights, imu_stamps,
    imu_gyro, imu_accel, scan_start_time, scan_end_time, dt_sec (+ t_last_scan, t_scan, odom_pose,
    odom_cov_se3, odom_twist, odom_twist_cov).  Sigma_g / Sigma_a default to the IW modes of
    meas_state (datasheet state when None), as the node sets them per scan (backend_node.py:2020-2023)."""
    st = _scan_prologue(belief_prev, scan, Q, cfg, meas_state, Sigma_g, Sigma_a)
    certs, dk, cert_deskew = st["certs"], st["dk"], st["cert_deskew"]
    # 4-6 BinSoftAssign + ScanBinMomentMatch (+Kappa)
    origin = np.asarray(cfg.lidar_origin, np.float64)
    d = ops.point_directions(dk["points"], origin)
    tau = cfg.temperature()
    if cfg.mode == "dense":
        sa = ops.bin_soft_assign_dense(d, bins, tau)
        st_b = ops.scan_bin_moment_match_dense(dk["points"], dk["weights"], sa["responsibilities"], origin)
    else:
        sa = ops.bin_soft_assign_scale(d, bins, knn, tau)
        st_b = ops.scan_bin_moment_match_scale(dk["points"], dk["weights"], sa["indices"],
                                               sa["responsibilities"], origin, bins.shape[0])
    cert_sa = dict(name="soft_assign", ess_total=sa["ess_total"])
    cert_mm = dict(name="moment_match", ess_total=st_b["ess"], psd_projection_delta=st_b["psd_projection_delta"],
                   mass_epsilon_ratio=st_b["mass_epsilon_ratio"])
    # 7 MatrixFisherRotation, 8 PlanarTranslationEvidence
    pose_pred = st["pose_pred"]
    R_pred = se3.so3_exp(pose_pred[3:6])
    m = map_state
    mf = ops.matrix_fisher_rotation(R_pred, st_b["s_dir"], st_b["S_dir_scatter"], st_b["N"], m.stats.S_dir,
                                    m.stats.S_dir_scatter, m.stats.N_dir)
    pt = ops.planar_translation(pose_pred[:3], mf["R_mf"], st_b["p_bar"], st_b["Sigma_p"], st_b["N"], m.centroid,
                                m.Sigma_c, m.stats.N_pos, m.stats.S_dir_scatter, m.stats.N_dir)
    cert_mf = dict(name="mf", psd_projection_delta=mf["psd_projection_delta"],
                   mass_epsilon_ratio=mf["mass_epsilon_ratio"])
    cert_pt = dict(name="planar", psd_projection_delta=pt["psd_projection_delta"],
                   mass_epsilon_ratio=pt["mass_epsilon_ratio"])
    lidar_certs = [cert_deskew, cert_sa, cert_mm, cert_mf, cert_pt]
    certs.extend([cert_sa, cert_mm, cert_mf, cert_pt])
    # 9-12 evidence, tempering, fusion, recompose
    L_lidar, h_lidar = ops.combined_lidar_evidence_22d(mf, pt)
    tl = _scan_tail(st, cfg, L_lidar, h_lidar, _aggregate_ess(lidar_certs), mf["nll_per_ess"] + pt["nll_per_ess"],
                    L_ext, h_ext)
    b_rec = tl["b_rec"]
    # 13 PoseCovInflationPushforward (map update with z_t)
    z_t = tl["z_t"]
    cov_rec, _ = spd_inverse_lifted(b_rec.L, ops.EPS_LIFT)
    new_stats = ops.pose_cov_inflation_pushforward(m.stats, st_b, z_t, cfg.pushforward_inflation_scale * cov_rec[0:6, 0:6],
                                                   cfg.forgetting_factor)
    new_map = MapState(new_stats, *ops.map_derived_stats(new_stats))
    # 14 AnchorDriftUpdate
    b_fin, dinfo = ops.anchor_drift_update(b_rec)
    certs.append(dict(name="anchor_drift", **dinfo))
    return dict(belief=b_fin, map=new_map, iw_process_dPsi=tl["iw_process_dPsi"], iw_process_dnu=tl["iw_process_dnu"],
                iw_meas_dPsi=st["meas_dPsi"], iw_meas_dnu=st["meas_dnu"], budget=st["bud"], deskew=dk, soft_assign=sa,
                scan_bins=st_b, mf=mf, planar=pt, L_evidence=tl["L_evidence"], h_evidence=tl["h_evidence"],
                beta=tl["beta"], total_trigger=tl["total_trigger"], frobenius_strength=tl["frobenius_strength"],
                z_t=z_t, xi_body=st["xi"], certs=certs, belief_post=tl["b_post"], belief_recomposed=b_rec,
                imu_odom=st["io"], alpha=tl["alpha"], fusion_quality=tl["fusion_quality"], cond_pose6=tl["cond_pose6"],
                ess_total=tl["ess_total"], nll_total=tl["nll_total"])


@dataclass
class PrimitivePathConfig(BinPathConfig):
    """The live path's map-branch parameters (PipelineConfig, FS/backend/pipeline.py:179-211, with
    the reference constants, FS/common/constants.py:350-477)."""
    n_surfel: int = 1024
    n_feat: int = 512
    m_tile: int = 50000
    m_tile_view: int = 1024
    h_tile: float = 2.0
    r_active_xy: int = 1
    r_active_z: int = 0
    r_stencil_xy: int = 1
    r_stencil_z: int = 0
    k_assoc: int = 8
    k_sinkhorn: int = 50
    ot_epsilon: float = 0.1
    ot_tau_a: float = 0.5
    ot_tau_b: float = 0.5
    k_insert_tile: int = 64
    recency_decay_lambda: float = 0.02
    recency_min_scale: float = 0.05


def process_scan_primitive_path(belief_prev: ops.Belief, scan: dict, Q, cfg: PrimitivePathConfig, tiles: dict,
                                next_global_id: int, scan_seq: int, meas_state=None, Sigma_g=None, Sigma_a=None,
                                batch=None):
    """One hypothesis, one scan of the live pipeline (FS/backend/pipeline.py:316-1591): the shared
    prologue, the map branch (:778-926: surfels on the deskewed budget points, recency inflation of
    the active tiles, the view over the stencil, OT association), visual pose evidence at z_lin_pose
    (:980-1010) as the LiDAR evidence, the shared tail (:1038-1230), step 12b at z_t (:1232-1492)
    and AnchorDriftUpdate.  `tiles` (dict tile id -> tile) is updated in place; returns the result
    dict with next_global_id.  The camera batch is empty (out of scope).  batch: a MeasurementBatch
    dict to use instead of this oracle's surfel extraction (a plane fit whose two smallest
    eigenvalues coincide -- cells of two or three collinear points -- has no unique normal, and
    lidar_surfel_extraction.py:129-130 then orients it by the sign of a rounding-level z component,
    so a closed-loop check feeds both sides the same batch and checks the extraction on its own)."""
    from . import association as OA, primitive_evidence as OE, primitive_map as OPM, surfels as OS
    st = _scan_prologue(belief_prev, scan, Q, cfg, meas_state, Sigma_g, Sigma_a)
    certs, dk, io, b_pred = st["certs"], st["dk"], st["io"], st["b_pred"]
    # z_lin_pose (pipeline.py:745-755)
    L_f = b_pred.L + (0.0 if io is None else io["L"])
    h_f = b_pred.h + (0.0 if io is None else io["h"])
    z_lin_pose = spd_solve_lifted(psd_project(L_f, ops.EPS_PSD)[0], h_f, ops.EPS_LIFT)[0][0:6]
    # map branch (:778-926)
    scfg = OS.SurfelExtractionConfig(n_surfel=cfg.n_surfel, n_feat=cfg.n_feat)
    if batch is None:
        batch, c_surf, _ = OS.extract_lidar_surfels(dk["points"], st["bud"]["timestamps"], dk["weights"], scfg)
        batch["n_valid"] = batch["n_camera_valid"] + batch["n_lidar_valid"]
    else:
        nv = int(batch["n_valid"])
        c_surf = dict(ess_total=float(nv), support_frac=float(nv) / float(max(cfg.n_surfel, 1)))
    centre = st["pose_pred"][:3]
    active = OPM.ma_hex_stencil_tile_ids(centre, cfg.h_tile, cfg.r_active_xy, cfg.r_active_z)
    stencil = OPM.ma_hex_stencil_tile_ids(centre, cfg.h_tile, cfg.r_stencil_xy, cfg.r_stencil_z)
    infl = OPM.recency_inflate(tiles, active, scan_seq, cfg.recency_decay_lambda, cfg.recency_min_scale)
    view = OPM.extract_atlas_map_view(tiles, stencil, cfg.m_tile_view, cfg.m_tile)
    view.update(m_tile_view=cfg.m_tile_view)
    acfg = OA.AssociationConfig(k_assoc=cfg.k_assoc, k_sinkhorn=cfg.k_sinkhorn, epsilon=cfg.ot_epsilon,
                                tau_a=cfg.ot_tau_a, tau_b=cfg.ot_tau_b, h_tile=cfg.h_tile,
                                r_stencil_tiles_xy=cfg.r_stencil_xy, r_stencil_tiles_z=cfg.r_stencil_z,
                                scan_seq=scan_seq, recency_decay_lambda=cfg.recency_decay_lambda)
    assoc, c_assoc = OA.associate_primitives_ot(batch, view, acfg)
    vis = OE.visual_pose_evidence(batch, view, assoc, z_lin_pose)
    # certificates (surfel: support only; recency inflation: exact; association: mass_epsilon_ratio;
    # visual: lift_strength eps_lift, support = transported mass), in all_certs order
    cert_surf = dict(name="surfel", ess_total=c_surf["ess_total"])
    cert_infl = dict(name="recency_inflate")
    cert_assoc = dict(name="association") if c_assoc.get("exact") else dict(
        name="association", ess_total=c_assoc["ess_total"], mass_epsilon_ratio=c_assoc["mass_epsilon_ratio"])
    cert_vis = dict(name="visual") if vis["exact"] else dict(name="visual", ess_total=vis["ess_total"],
                                                               lift_strength=ops.EPS_LIFT)
    certs.extend([cert_surf, cert_infl, cert_assoc, cert_vis])
    lidar_certs = [st["cert_deskew"], cert_surf, cert_assoc, cert_vis]
    tl = _scan_tail(st, cfg, vis["L_pose"], vis["h_pose"], _aggregate_ess(lidar_certs), 0.0)
    b_rec, z_t = tl["b_rec"], tl["z_t"]
    # 12b the primitive map update at z_t (:1232-1492)
    next_global_id, mstats = OPM.map_update_step(tiles, next_global_id, batch, assoc, se3.so3_exp(z_t[3:6]), z_t[:3],
                                                 active, cfg.m_tile, float(scan["scan_end_time"]), scan_seq,
                                                 k_insert_tile=cfg.k_insert_tile, h_tile=cfg.h_tile,
                                                 recency_decay_lambda=cfg.recency_decay_lambda)
    # 13 AnchorDriftUpdate
    b_fin, dinfo = ops.anchor_drift_update(b_rec)
    certs.append(dict(name="anchor_drift", **dinfo))
    return dict(belief=b_fin, next_global_id=next_global_id, map_update=mstats, active_tile_ids=active,
                stencil_tile_ids=stencil, recency=infl, surfels=batch, view=view, assoc=assoc, assoc_cert=c_assoc,
                visual=vis, z_lin_pose=z_lin_pose, iw_process_dPsi=tl["iw_process_dPsi"],
                iw_process_dnu=tl["iw_process_dnu"], iw_meas_dPsi=st["meas_dPsi"], iw_meas_dnu=st["meas_dnu"],
                L_evidence=tl["L_evidence"], h_evidence=tl["h_evidence"], beta=tl["beta"],
                total_trigger=tl["total_trigger"], z_t=z_t, certs=certs, belief_recomposed=b_rec, deskew=dk,
                budget=st["bud"], imu_odom=io, alpha=tl["alpha"], ess_total=tl["ess_total"])


def combine_and_update_noise(results, weights, iw_state, scan_count, meas_state=None):
    """Node-level post-loop (FS/backend/backend_node.py:1999-2119): IW accumulation with raw
    weights, barycenter with floor-renormalised weights, process IW apply (weight min(1, scan)),
    Q rebuild, measurement-noise IW apply (weight 1, :2105,2114-2119)."""
    nu, Psi = iw_state
    acc = np.zeros((7, 6, 6))
    accn = np.zeros(7)
    accm = np.zeros((3, 3, 3))
    accmn = np.zeros(3)
    for w, r in zip(weights, results):
        acc += w * r["iw_process_dPsi"]
        accn += w * r["iw_process_dnu"]
        accm += w * r["iw_meas_dPsi"]
        accmn += w * r["iw_meas_dnu"]
    if meas_state is None:
        meas_state = ops.datasheet_measurement_noise_state()
    mnu, mPsi, mcert = ops.measurement_noise_iw_apply(meas_state[0], meas_state[1], accm, accmn)
    L = np.stack([r["belief"].L for r in results])
    h = np.stack([r["belief"].h for r in results])
    z = np.stack([r["belief"].z_lin for r in results])
    combo = ops.hypothesis_barycenter(L, h, z, weights)
    wp = min(1, scan_count)
    nu2, Psi2, cert = ops.process_noise_iw_apply(nu, Psi, wp * acc, wp * accn)
    Q = ops.process_noise_Q(nu2, Psi2)
    return dict(combined=combo, iw_state=(nu2, Psi2), Q=Q, iw_cert=cert, acc_dPsi=acc, acc_dnu=accn,
                meas_state=(mnu, mPsi), meas_cert=mcert, acc_meas_dPsi=accm, acc_meas_dnu=accmn)
