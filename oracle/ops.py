"""Per-operator numpy restatement of the GC-SLAM bin-path hot path (test oracle only).

Reference paths are relative to /root/reference; FS = fl_ws/src/fl_slam_poc/fl_slam_poc.
Declared items that the reference does not pin are marked
DECLARED and documented in DESIGN.md.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import se3
from .primitives import (F64_EPS, inv_mass, psd_project, psd_project_batch, sigmoid,
                         softplus, spd_inverse_lifted, spd_solve_lifted)

# ---------------------------------------------------------------- constants (FS/common/constants.py)
EPS_PSD = 1e-12          # :70
EPS_LIFT = 1e-9          # :71
EPS_MASS = 1e-12         # :72
EPS_R = 1e-6             # :73
KAPPA_R0 = 0.8           # :95
KAPPA_TAU = 0.03         # :96
C_FROB = 1.0             # :101
ANCHOR_M0 = 0.5          # :104
ANCHOR_R0 = 0.2          # :105
TIME_WARP_SIGMA_FRAC = 0.1  # :143
WEIGHT_FLOOR = 1e-12     # :256
OU_LAMBDA = 0.1          # :248
HYP_WEIGHT_FLOOR = 0.0025  # :63
GRAVITY_W = (0.0, 0.0, -9.81)  # :80
IW_NU_WEAK_ADD = 0.5     # :164
IW_RHO = (0.99, 0.995, 0.95, 0.999, 0.999, 0.9999, 0.9999)  # trans,rot,vel,bg,ba,dt,ex :265-271
PROCESS_BLOCK_DIMS = (3, 3, 3, 3, 3, 1, 6)     # FS/backend/structures/inverse_wishart_jax.py:20
PROCESS_BLOCK_STARTS = (0, 3, 6, 9, 12, 15, 16)
POWER_BETA_MIN, POWER_BETA_EXC_C, POWER_BETA_Z_C = 0.25, 50.0, 1.0  # FS/backend/pipeline.py:119-121
FORGETTING_FACTOR = 0.99  # FS/backend/pipeline.py:130 (PipelineConfig.forgetting_factor)

# DECLARED: soft-assign temperature and scale-mode candidates.
TAU_48 = 0.1             # temperature at the legacy B=48 atlas (SURVEY 8d suggestion)
K_CAND = 16              # candidate bins per point in scale mode


def tau_for_bins(B: int) -> float:
    """DECLARED: tau scales with the bin solid angle, tau_B = TAU_48 * 48 / B."""
    return TAU_48 * 48.0 / float(B)


def trigger_magnitude(infl: dict) -> float:
    """CertBundle.total_trigger_magnitude, FS/common/certificates.py:439-455."""
    g = lambda k, d: float(infl.get(k, d))  # noqa: E731
    return (g("lift_strength", 0.0) + g("psd_projection_delta", 0.0) + g("nu_projection_delta", 0.0)
            + g("mass_epsilon_ratio", 0.0) + g("anchor_drift_rho", 0.0)
            + abs(1.0 - g("dt_scale", 1.0)) + abs(1.0 - g("extrinsic_scale", 1.0))
            + abs(1.0 - g("trust_alpha", 1.0)) + abs(1.0 - g("power_beta", 1.0)))


def dot3(a, b):
    """Canonical 3-dot (x*x' + y*y') + z*z', no fma: the op order the HIP kernels use."""
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


# ================================================================ before row 1: PointCloud2 parse
NONFINITE_SENTINEL = 1e6                           # constants.py:256-262
RANGE_WEIGHT_SIGMA, RANGE_WEIGHT_MIN_R, RANGE_WEIGHT_MAX_R = 0.25, 0.5, 50.0
PC2_DTYPES = {1: "i1", 2: "u1", 3: "<i2", 4: "<u2", 5: "<i4", 6: "<u4", 7: "<f4", 8: "<f8"}  # PointField codes


def parse_pointcloud2_vlp16(data, fields, point_step, n_points, header_stamp_sec):
    """parse_pointcloud2_vlp16, FS/backend/backend_node.py:377-468.  fields: {name: (offset,
    datatype)}.  Returns points (n,3) f64 (lidar frame), t, w, ring (u8), tag (u8)."""
    if n_points <= 0:
        return (np.zeros((0, 3)), np.zeros(0), np.zeros(0), np.zeros(0, np.uint8), np.zeros(0, np.uint8))
    missing = [k for k in ("x", "y", "z", "ring") if k not in fields]
    if missing:
        raise RuntimeError(f"PointCloud2 (VLP-16 layout) missing required fields: {missing}")
    time_field = "t" if "t" in fields else ("time" if "time" in fields else None)
    names = ["x", "y", "z", "ring"] + ([time_field] if time_field else [])
    dt = np.dtype({"names": names, "formats": [PC2_DTYPES[fields[k][1]] for k in names],
                   "offsets": [fields[k][0] for k in names], "itemsize": point_step})
    arr = np.frombuffer(bytes(data), dtype=dt, count=n_points)
    s = NONFINITE_SENTINEL
    x, y, z = (np.nan_to_num(np.asarray(arr[k], np.float64), nan=s, posinf=s, neginf=-s) for k in "xyz")
    ring = np.asarray(arr["ring"]).astype(np.uint8)
    if time_field is not None:
        t_raw = np.asarray(arr[time_field], np.float64)
        t = t_raw * 1e-9 if np.any(t_raw > 1e6) else t_raw
    else:
        t = np.full(n_points, header_stamp_sec, np.float64)
    dist = np.sqrt(x * x + y * y + z * z)
    a = (dist - RANGE_WEIGHT_MIN_R) / RANGE_WEIGHT_SIGMA
    b = (RANGE_WEIGHT_MAX_R - dist) / RANGE_WEIGHT_SIGMA
    with np.errstate(over="ignore"):  # sentinel ranges: exp overflows to inf, the weight to 0 (as in numpy there)
        w_raw = (1.0 / (1.0 + np.exp(-a))) * (1.0 / (1.0 + np.exp(-b)))
    w = w_raw * (1.0 - WEIGHT_FLOOR) + WEIGHT_FLOOR
    return np.stack([x, y, z], axis=1), t, w, ring, np.zeros(n_points, np.uint8)


def lidar_to_base(points, R_base_lidar, t_base_lidar):
    """No-TF mode transform before inference, backend_node.py:1677-1680."""
    return (np.asarray(R_base_lidar) @ points.T).T + np.asarray(t_base_lidar)[None, :]


# ================================================================ row 1: PointBudgetResample
def point_budget_resample(points, timestamps, weights, ring=None, tag=None, n_points_cap=8192):
    """FS/backend/operators/point_budget.py:50-109 (core) and :117-221 (wrapper)."""
    points = np.asarray(points, dtype=np.float64)
    timestamps = np.asarray(timestamps, dtype=np.float64)
    weights = np.asarray(weights, dtype=np.float64)
    n = points.shape[0]
    ring = np.zeros(n, np.uint8) if ring is None else np.asarray(ring, np.uint8)
    tag = np.zeros(n, np.uint8) if tag is None else np.asarray(tag, np.uint8)
    stride = max(1, int(math.ceil(n / n_points_cap)))          # :160
    idx = np.arange(0, n, stride)                               # :70
    ns = idx.shape[0]
    mass_in = weights.sum()
    w_raw = weights[idx]
    mass_scale = mass_in / (w_raw.sum() + EPS_MASS)             # :80-84
    out = dict(points=np.zeros((n_points_cap, 3)), timestamps=np.zeros(n_points_cap),
               weights=np.zeros(n_points_cap), ring=np.zeros(n_points_cap, np.uint8),
               tag=np.zeros(n_points_cap, np.uint8), indices=idx.astype(np.int64))
    out["points"][:ns] = points[idx]
    out["timestamps"][:ns] = timestamps[idx]
    out["weights"][:ns] = w_raw * mass_scale
    out["ring"][:ns] = ring[idx]
    out["tag"][:ns] = tag[idx]
    wn = out["weights"] / (mass_in + EPS_MASS)
    ess = 1.0 / np.sum(wn ** 2 + EPS_MASS)                      # :95-96
    out.update(n_input=n, n_output=ns, stride=stride, total_mass_in=mass_in, total_mass_out=mass_in,
               ess=ess, support_frac=min(1.0, n_points_cap / (n + EPS_MASS)),
               mass_epsilon_ratio=EPS_MASS / (mass_in + EPS_MASS))
    return out


# ================================================================ row 2: IMU window + preintegration
def smooth_window_weights(t, start, end, sigma):
    """FS/backend/operators/imu_preintegration.py:20-43."""
    t = np.asarray(t, dtype=np.float64)
    sig = max(float(sigma), 1e-6)
    w_raw = sigmoid((t - start) / sig) * sigmoid((end - t) / sig)
    return w_raw * (1.0 - WEIGHT_FLOOR) + WEIGHT_FLOOR


def preintegrate_imu(stamps, gyro, accel, weights, rotvec_start, gyro_bias, accel_bias, gravity_W):
    """preintegrate_imu_relative_pose_jax, imu_preintegration.py:47-147 (sequential lax.scan)."""
    stamps = np.asarray(stamps, np.float64)
    gyro = np.asarray(gyro, np.float64)
    accel = np.asarray(accel, np.float64)
    w = np.asarray(weights, np.float64)
    gb, ab, g = (np.asarray(x, np.float64) for x in (gyro_bias, accel_bias, gravity_W))
    ess = w.sum()
    dt = np.concatenate([stamps[1:] - stamps[:-1], [0.0]])
    dt = np.maximum(dt, 0.0)
    R = se3.so3_exp(rotvec_start)
    v = np.zeros(3)
    p = np.zeros(3)
    s_wdt = 0.0
    s_ab = np.zeros(3)
    s_an = np.zeros(3)
    s_aw = np.zeros(3)
    for i in range(stamps.shape[0]):
        dte = w[i] * dt[i]
        dR = se3.so3_exp((gyro[i] - gb) * dte)
        Rn = R @ dR
        a_body = accel[i] - ab
        a_nog = R @ a_body
        a_w = a_nog + g
        s_wdt += dte
        s_ab = s_ab + a_body * dte
        s_an = s_an + a_nog * dte
        s_aw = s_aw + a_w * dte
        vn = v + a_w * dte
        p = p + v * dte + 0.5 * a_w * (dte * dte)
        v, R = vn, Rn
    R0 = se3.so3_exp(rotvec_start)
    dR = R0.T @ R
    delta_pose = np.concatenate([R0.T @ p, se3.so3_log(dR)])
    den = max(s_wdt, 1e-12)
    return dict(delta_pose=delta_pose, delta_R=dR, delta_p=R0.T @ p, delta_v=R0.T @ v, ess=ess,
                a_body_mean=s_ab / den, a_world_nog_mean=s_an / den, a_world_mean=s_aw / den,
                dt_eff_sum=s_wdt)


# ================================================================ row 3: DeskewConstantTwist
def deskew_constant_twist(points, timestamps, weights, t0, t1, xi_body):
    """deskew_constant_twist.py:31-69 (core) + :72-117 (wrapper cert)."""
    timestamps = np.asarray(timestamps, np.float64)
    weights = np.asarray(weights, np.float64)
    denom = max(t1 - t0, 1e-12)
    alpha = (timestamps - t0) / denom
    p0 = se3.deskew_points(points, alpha, xi_body)
    w_time = smooth_window_weights(timestamps, t0, t1, TIME_WARP_SIGMA_FRAC * denom)
    w_out = weights * w_time
    retained = w_out.sum() / (weights.sum() + EPS_MASS)
    return dict(points=p0, weights=w_out, support_frac=retained)


def point_directions(points, origin, eps_mass=EPS_MASS):
    """FS/backend/pipeline.py:589-593 and binning.py:162-164: d = (p-o)/(|p-o|+eps)."""
    rays = np.asarray(points, np.float64) - np.asarray(origin, np.float64)[None, :]
    nrm = np.sqrt(dot3(rays, rays))
    return rays / (nrm + eps_mass)[:, None]


# ================================================================ atlas (archive/bin_atlas.py)
def fibonacci_atlas(n_bins):
    """_create_fibonacci_atlas_jax, archive/bin_atlas.py:40-61."""
    idx = np.arange(n_bins, dtype=np.float64) + 0.5
    phi = np.arccos(1.0 - 2.0 * idx / n_bins)
    theta = np.pi * (1.0 + np.sqrt(5.0)) * idx
    d = np.stack([np.sin(phi) * np.cos(theta), np.sin(phi) * np.sin(theta), np.cos(phi)], axis=1)
    n = np.sqrt(dot3(d, d))
    return d / (n + EPS_MASS)[:, None]


def knn_shortlist(queries, bins, k, extra=8, brute=False):
    """DECLARED candidate rule helper: exact K-nearest atlas bins by canonical dot, ties by lower id.

    brute=True scans all bins (small cases); otherwise a cKDTree shortlist of k+extra
    Euclidean neighbours is re-ranked exactly (distance^2 = 2-2dot on the unit sphere).
    """
    queries = np.asarray(queries, np.float64)
    if brute or bins.shape[0] <= k + extra:
        sims = dot3(queries[:, None, :], bins[None, :, :])
        ids = np.broadcast_to(np.arange(bins.shape[0]), sims.shape)
        out = np.empty((queries.shape[0], k), np.int64)
        for i in range(queries.shape[0]):
            o = np.lexsort((ids[i], -sims[i]))
            out[i] = o[:k]
        return out
    from scipy.spatial import cKDTree
    tree = cKDTree(bins)
    _, cand = tree.query(queries, k=min(k + extra, bins.shape[0]))
    cand = np.asarray(cand, np.int64)
    sims = dot3(queries[:, None, :], bins[cand])
    # vectorised lexicographic (sim desc, id asc) via stable double argsort
    o1 = np.argsort(cand, axis=1, kind="stable")
    cand1 = np.take_along_axis(cand, o1, 1)
    sims1 = np.take_along_axis(sims, o1, 1)
    o2 = np.argsort(-sims1, axis=1, kind="stable")
    out = np.take_along_axis(cand1, o2, 1)[:, :k]
    zero = np.all(queries == 0.0, axis=1)
    if np.any(zero):   # all B dots tie at 0: the rule picks the lowest ids (shortlist cannot see that)
        out[zero] = np.arange(k)[None, :]
    return out


def bin_knn_table(bins, k=K_CAND, brute=False):
    """DECLARED: kNN graph of the atlas, row b = K nearest bins to bin b (includes b)."""
    return knn_shortlist(bins, bins, k, brute=brute)


def nearest_bin(d, bins, brute=False):
    """DECLARED: a(n) = argmax_b dot(d_n, bin_b), ties -> lowest id."""
    return knn_shortlist(d, bins, 1, brute=brute)[:, 0]


# ================================================================ row 4: KappaFromResultant
def kappa_from_resultant_batch(R_bar, eps_r=EPS_R, d=3.0, r0=KAPPA_R0, tau=KAPPA_TAU):
    """kappa.py:130-169."""
    R = np.clip(np.asarray(R_bar, np.float64), 0.0, 1.0 - eps_r)
    R2 = R * R
    k_low = (R * (d - R2)) / (1.0 - R2 + eps_r)
    k_high = -np.log(np.maximum(1.0 - R2, eps_r))
    s = sigmoid((R - r0) / max(tau, 1e-6))
    return (1.0 - s) * k_low + s * k_high


# ================================================================ row 5: BinSoftAssign
def _softmax_rows(logits):
    m = logits.max(axis=1, keepdims=True)
    e = np.exp(logits - m)
    return e / e.sum(axis=1, keepdims=True)


def bin_soft_assign_dense(point_dirs, bin_dirs, tau):
    """archive/legacy_operators/binning.py:56-76 + cert :118-125 (dense N x B)."""
    sims = point_dirs @ bin_dirs.T
    r = _softmax_rows(sims / tau)
    n = point_dirs.shape[0]
    ent = -np.sum(r * np.log(r + EPS_MASS), axis=1)
    avg_entropy = ent.sum() / (n + EPS_MASS)
    return dict(responsibilities=r, avg_entropy=avg_entropy, max_resp=r.max(),
                ess_total=math.exp(avg_entropy), support_frac=r.max())


def bin_soft_assign_scale(point_dirs, bin_dirs, knn, tau, nearest=None):
    """Scale mode (DECLARED truncation of binning.py:68-69): softmax restricted to the K
    candidates knn[a(n)], a(n) = nearest bin.  Returns (N,K) ids and responsibilities."""
    if nearest is None:
        nearest = nearest_bin(point_dirs, bin_dirs)
    ids = knn[nearest]
    sims = dot3(point_dirs[:, None, :], bin_dirs[ids])
    r = _softmax_rows(sims / tau)
    n = point_dirs.shape[0]
    ent = -np.sum(r * np.log(r + EPS_MASS), axis=1)
    avg_entropy = ent.sum() / (n + EPS_MASS)
    return dict(indices=ids, nearest=nearest, responsibilities=r, avg_entropy=avg_entropy,
                max_resp=r.max(), ess_total=math.exp(avg_entropy), support_frac=r.max())


# ================================================================ row 6: ScanBinMomentMatch (+kappa)
def _bin_raw_sums_dense(points, weights, r, origin):
    w_r = weights[:, None] * r                                   # binning.py:159-160
    d = point_directions(points, origin)                         # :162-164
    N = w_r.sum(axis=0)                                          # :166
    s_dir = w_r.T @ d                                            # :167
    S = np.einsum("nb,ni,nj->bij", w_r, d, d)                    # :168
    sum_p = w_r.T @ points                                       # :169
    sum_ppT = np.einsum("nb,ni,nj->bij", w_r, points, points)    # :171-172
    return N, s_dir, S, sum_p, sum_ppT


def _bin_raw_sums_sparse(points, weights, ids, r, origin, n_bins):
    d = point_directions(points, origin)
    m = (weights[:, None] * r).reshape(-1)
    b = ids.reshape(-1)
    pn = np.repeat(np.arange(points.shape[0]), ids.shape[1])
    N = np.zeros(n_bins)
    np.add.at(N, b, m)
    s_dir = np.zeros((n_bins, 3))
    np.add.at(s_dir, b, m[:, None] * d[pn])
    S = np.zeros((n_bins, 3, 3))
    np.add.at(S, b, m[:, None, None] * d[pn][:, :, None] * d[pn][:, None, :])
    sum_p = np.zeros((n_bins, 3))
    np.add.at(sum_p, b, m[:, None] * points[pn])
    sum_ppT = np.zeros((n_bins, 3, 3))
    np.add.at(sum_ppT, b, m[:, None, None] * points[pn][:, :, None] * points[pn][:, None, :])
    return N, s_dir, S, sum_p, sum_ppT


def finalize_scan_bins(N, s_dir, S, sum_p, sum_ppT, sum_cov=None):
    """binning.py:175-209: InvMass, centroid, PSD(scatter), kappa and cert scalars."""
    inv_N, eps_ratio = inv_mass(N, EPS_MASS)
    p_bar = sum_p * inv_N[:, None]
    scatter = sum_ppT * inv_N[:, None, None] - p_bar[:, :, None] * p_bar[:, None, :]
    if sum_cov is not None:
        scatter = scatter + sum_cov * inv_N[:, None, None]
    Sigma_p, delta = psd_project_batch(scatter, EPS_PSD)
    Rbar = np.sqrt(dot3(s_dir, s_dir)) * inv_N
    kappa = kappa_from_resultant_batch(Rbar)
    total = N.sum()
    return dict(N=N, s_dir=s_dir, S_dir_scatter=S, p_bar=p_bar, Sigma_p=Sigma_p, kappa_scan=kappa,
                ess=total ** 2 / ((N ** 2).sum() + EPS_MASS),
                support_frac=float(np.mean(N / (N + EPS_MASS))),
                psd_projection_delta=float(delta.sum()), mass_epsilon_ratio=float(eps_ratio.max()),
                sum_p=sum_p, sum_ppT=sum_ppT)


def scan_bin_moment_match_dense(points, weights, r, origin):
    """binning.py:139-209 with point_covariances = 0 (pipeline.py:586-587), lambda = 1."""
    return finalize_scan_bins(*_bin_raw_sums_dense(points, weights, r, origin))


def scan_bin_moment_match_scale(points, weights, ids, r, origin, n_bins):
    return finalize_scan_bins(*_bin_raw_sums_sparse(points, weights, ids, r, origin, n_bins))


# ================================================================ map bin stats (archive/bin_atlas.py)
@dataclass
class MapBinStats:
    S_dir: np.ndarray
    S_dir_scatter: np.ndarray
    N_dir: np.ndarray
    N_pos: np.ndarray
    sum_p: np.ndarray
    sum_ppT: np.ndarray

    @classmethod
    def empty(cls, B):
        """create_empty_map_stats, bin_atlas.py:117-134."""
        return cls(np.zeros((B, 3)), np.zeros((B, 3, 3)), np.zeros(B), np.zeros(B), np.zeros((B, 3)),
                   np.zeros((B, 3, 3)))

    def copy(self):
        return MapBinStats(*(x.copy() for x in (self.S_dir, self.S_dir_scatter, self.N_dir,
                                                 self.N_pos, self.sum_p, self.sum_ppT)))


def map_derived_stats(m: MapBinStats):
    """_compute_map_derived_stats_core, bin_atlas.py:166-200 -> (mu_dir, kappa, centroid, Sigma_c)."""
    nrm = np.sqrt(dot3(m.S_dir, m.S_dir))
    # _safe_normalize_jax(v, eps) = v / (||v|| + eps) (FS/common/primitives.py)
    mu_dir = m.S_dir / (nrm + EPS_MASS)[:, None]
    inv_Nd, _ = inv_mass(m.N_dir)
    kappa = kappa_from_resultant_batch(nrm * inv_Nd)
    inv_Np, _ = inv_mass(m.N_pos)
    centroid = m.sum_p * inv_Np[:, None]
    raw = m.sum_ppT * inv_Np[:, None, None] - centroid[:, :, None] * centroid[:, None, :]
    Sigma_c, _ = psd_project_batch(raw, EPS_PSD)
    return mu_dir, kappa, centroid, Sigma_c


def pose_cov_inflation_pushforward(m: MapBinStats, scan: dict, pose6, Sigma_pose6, gamma=FORGETTING_FACTOR):
    """Row 11 PoseCovInflationPushforward -- source deleted upstream; DECLARED restatement.

    Forgetting (bin_atlas.py:232-257) then additive update (bin_atlas.py:137-163) with the scan
    bin statistics pushed to world at z_t = (t, R), t_z := 0 (CHANGELOG.md:575-578):
      S_dir += R s_dir ; S_dir_scatter += R S R^T ; N_dir += N ; N_pos += N
      sum_p += N (R p_bar + t)
      sum_ppT += N [ R (Sigma_p + p_bar p_bar^T) R^T + J Sigma_pose J^T ]
                 + N (R p_bar t^T + t p_bar^T R^T + t t^T),    J = [I, -R [p_bar]x]
    """
    t = np.array([pose6[0], pose6[1], 0.0])
    R = se3.so3_exp(pose6[3:6])
    N = scan["N"]
    pb = scan["p_bar"]
    Rp = pb @ R.T                                   # (B,3) R p_bar
    RS = np.einsum("ij,bjk,lk->bil", R, scan["S_dir_scatter"], R)
    second = scan["Sigma_p"] + pb[:, :, None] * pb[:, None, :]
    R2 = np.einsum("ij,bjk,lk->bil", R, second, R)
    Stt, Str, Srr = Sigma_pose6[:3, :3], Sigma_pose6[:3, 3:], Sigma_pose6[3:, 3:]
    # J = [I, A] with A = -R [p]x  ->  J S J^T = Stt + A Srt + Str A^T + A Srr A^T
    K = np.zeros((pb.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -pb[:, 2], pb[:, 1]
    K[:, 1, 0], K[:, 1, 2] = pb[:, 2], -pb[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -pb[:, 1], pb[:, 0]
    A = -np.einsum("ij,bjk->bik", R, K)
    JSJ = (Stt[None] + np.einsum("bij,jk->bik", A, Str.T) + np.einsum("ij,bkj->bik", Str, A)
           + np.einsum("bij,jk,blk->bil", A, Srr, A))
    q = Rp + t[None, :]
    out = MapBinStats(
        S_dir=gamma * m.S_dir + scan["s_dir"] @ R.T,
        S_dir_scatter=gamma * m.S_dir_scatter + RS,
        N_dir=gamma * m.N_dir + N,
        N_pos=gamma * m.N_pos + N,
        sum_p=gamma * m.sum_p + N[:, None] * q,
        sum_ppT=gamma * m.sum_ppT + N[:, None, None] * (R2 + JSJ + q[:, :, None] * q[:, None, :]
                                                        - Rp[:, :, None] * Rp[:, None, :]),
    )
    return out


# ================================================================ row 7: MatrixFisherRotation
def matrix_fisher_rotation(R_pred, scan_s_dir, scan_S, scan_N, map_S_dir, map_S, map_N, eps=EPS_MASS):
    """_matrix_fisher_core matrix_fisher_evidence.py:155-256 + wrapper :310-394."""
    w_b = np.sqrt(scan_N * map_N + eps)
    sn = np.sqrt(dot3(scan_s_dir, scan_s_dir))
    mn = np.sqrt(dot3(map_S_dir, map_S_dir))
    u_scan = scan_s_dir / (sn + eps)[:, None]
    u_map = map_S_dir / (mn + eps)[:, None]
    conf = (sn * (1.0 / (scan_N + eps))) * (mn * (1.0 / (map_N + eps)))
    w_final = w_b * conf
    H = np.einsum("b,bi,bj->ij", w_final, u_map, u_scan)
    U, s, Vt = np.linalg.svd(H)
    det_sign = np.linalg.det(U @ Vt)
    U = U.copy()
    U[:, 2] = U[:, 2] * np.sign(det_sign)
    R_mf = U @ Vt
    V = Vt.T
    L_raw = V @ np.diag([s[1] + s[2], s[0] + s[2], s[0] + s[1]]) @ V.T
    N_eff = w_final.sum()
    delta_rot = se3.so3_log(np.asarray(R_pred).T @ R_mf)
    L_rot, cert = psd_project(L_raw, EPS_PSD)
    h_rot = L_rot @ delta_rot
    return dict(R_mf=R_mf, L_rot=L_rot, h_rot=h_rot, delta_rot=delta_rot, svd_s=s, H=H, N_eff=N_eff,
                scan_scatter_total=scan_S.sum(0), map_scatter_total=map_S.sum(0),
                psd_projection_delta=cert[0], mass_epsilon_ratio=eps / (N_eff + eps),
                nll=0.5 * float(delta_rot @ L_rot @ delta_rot),
                nll_per_ess=0.5 * float(delta_rot @ L_rot @ delta_rot) / (N_eff + eps))  # cert :355-375


# ================================================================ row 8: PlanarTranslationEvidence
def planar_translation(t_pred, R_hat, scan_p_bar, scan_Sigma_p, scan_N, map_centroid, map_Sigma_c,
                       map_N_pos, map_S_scatter, map_N_dir, eps_mass=EPS_MASS):
    """matrix_fisher_evidence.py:413-499 (core) + :502-671 (wrapper)."""
    T_map = map_S_scatter.sum(0) / (map_N_dir.sum() + eps_mass)
    ev = np.sort(np.linalg.eigvalsh(T_map))[::-1]
    lam1 = max(ev[0], eps_mass)
    lam3 = max(ev[2], 0.0)
    z_scale = lam3 / lam1
    eps = eps_mass
    t_b = map_centroid - scan_p_bar @ R_hat.T
    Sig = map_Sigma_c + np.einsum("ij,bjk,lk->bil", R_hat, scan_Sigma_p, R_hat)
    w_b = np.sqrt(scan_N * map_N_pos + eps)
    Sinv = np.linalg.inv(Sig + eps * np.eye(3)[None]) * w_b[:, None, None]
    L_full = Sinv.sum(0)
    h_full = np.einsum("bij,bj->bi", Sinv, t_b).sum(0)
    t_wls = np.linalg.solve(L_full + eps * np.eye(3), h_full)
    mask = np.array([1.0, 1.0, z_scale])
    L_raw = L_full * mask[:, None] * mask[None, :]
    N_eff = w_b.sum()
    delta = t_wls - np.asarray(t_pred)
    L_trans, cert = psd_project(L_raw, EPS_PSD)
    h_trans = L_trans @ delta
    return dict(t_wls=t_wls, L_trans=L_trans, h_trans=h_trans, delta_trans=delta, z_scale=z_scale,
                L_full=L_full, h_full=h_full, N_eff=N_eff, psd_projection_delta=cert[0],
                mass_epsilon_ratio=eps / (N_eff + eps),
                nll=0.5 * float(delta @ L_trans @ delta),
                nll_per_ess=0.5 * float(delta @ L_trans @ delta) / (N_eff + eps))  # cert :630-653


def combined_lidar_evidence_22d(mf, pt):
    """build_combined_lidar_evidence_22d, matrix_fisher_evidence.py:729-756."""
    L = np.zeros((22, 22))
    h = np.zeros(22)
    L[0:3, 0:3] = pt["L_trans"]
    h[0:3] = pt["h_trans"]
    L[3:6, 3:6] = mf["L_rot"]
    h[3:6] = mf["h_rot"]
    return L, h


# ================================================================ belief helpers (FS/common/belief.py)
@dataclass
class Belief:
    X_anchor: np.ndarray
    stamp_sec: float
    z_lin: np.ndarray
    L: np.ndarray
    h: np.ndarray

    def copy(self):
        return Belief(self.X_anchor.copy(), self.stamp_sec, self.z_lin.copy(), self.L.copy(), self.h.copy())

    def mean_increment(self, eps_lift=EPS_LIFT):
        """belief.py:373-387."""
        return spd_solve_lifted(self.L, self.h, eps_lift)[0]

    def mean_world_pose(self, eps_lift=EPS_LIFT):
        """belief.py:410-434: X_anchor o Exp(delta_pose)."""
        dz = self.mean_increment(eps_lift)
        return se3.se3_compose(self.X_anchor, se3.se3_exp(dz[0:6]))

    @classmethod
    def identity_prior(cls, stamp_sec=0.0, prior_precision=1e-6):
        """create_identity_prior, belief.py:320-358."""
        return cls(np.zeros(6), stamp_sec, np.zeros(22), prior_precision * np.eye(22), np.zeros(22))


# ================================================================ step 2: PredictDiffusion
def predict_diffusion(b: Belief, Q, dt_sec, lambda_ou=OU_LAMBDA):
    """_predict_diffusion_core predict.py:43-103 + wrapper cert :153-172."""
    mean_prev, _ = spd_solve_lifted(b.L, b.h, EPS_LIFT)
    cov_prev, lift_prev = spd_inverse_lifted(b.L, EPS_LIFT)
    ef = math.exp(-2.0 * lambda_ou * dt_sec)
    dc = (1.0 - ef) / (2.0 * lambda_ou + F64_EPS)
    cov_raw = ef * cov_prev + dc * np.asarray(Q)
    cov_psd, c1 = psd_project(cov_raw, EPS_PSD)
    L_pred, lift_inv = spd_inverse_lifted(cov_psd, EPS_LIFT)
    L_psd, c2 = psd_project(L_pred, EPS_PSD)
    h = L_psd @ mean_prev
    out = Belief(b.X_anchor.copy(), b.stamp_sec + dt_sec, b.z_lin.copy(), L_psd, h)
    infl = dict(lift_strength=lift_prev + lift_inv, psd_projection_delta=c1[0] + c2[0], dt_scale=dt_sec)
    return out, infl


# ================================================================ step 9/10/11 helpers
def excitation_scales(L_ev, L_prior, eps=1e-12):
    """excitation.py:15-30."""
    e_dt, e_ex = L_ev[15, 15], np.trace(L_ev[16:22, 16:22])
    p_dt, p_ex = L_prior[15, 15], np.trace(L_prior[16:22, 16:22])
    return e_dt / (e_dt + p_dt + eps), e_ex / (e_ex + p_ex + eps)


def apply_excitation_scaling(L, h, s_dt, s_ex):
    """excitation.py:33-64."""
    L = L.copy()
    h = h.copy()
    a_dt, a_ex = 1.0 - s_dt, 1.0 - s_ex
    L[15, :] *= a_dt
    L[:, 15] *= a_dt
    h[15] *= a_dt
    L[16:22, :] *= a_ex
    L[:, 16:22] *= a_ex
    h[16:22] *= a_ex
    return L, h


def info_fusion_additive(b: Belief, L_ev, h_ev, alpha):
    """fusion.py:150-230."""
    L_post, cert = psd_project(b.L + alpha * L_ev, EPS_PSD)
    out = Belief(b.X_anchor.copy(), b.stamp_sec, b.z_lin.copy(), L_post, b.h + alpha * h_ev)
    return out, dict(psd_projection_delta=cert[0], trust_alpha=alpha)


def bch3(xi1, xi2):
    """_bch3_correction, recompose.py:50-91."""
    v1, w1, v2, w2 = xi1[:3], xi1[3:6], xi2[:3], xi2[3:6]
    return 0.5 * np.concatenate([np.cross(w1, v2) + np.cross(v1, w2), np.cross(w1, w2)])


def frobenius_recompose(b: Belief, total_trigger, c_frob=C_FROB):
    """pose_update_frobenius_recompose, recompose.py:94-205."""
    dz = b.mean_increment()
    dpose = dz[0:6]
    s = total_trigger / (total_trigger + c_frob)
    corr = bch3(b.z_lin[0:6], dpose)
    dpc = dpose + s * corr
    X_new = se3.se3_compose(b.X_anchor, se3.se3_exp(dpc))
    shift = np.zeros(22)
    shift[0:6] = dpc
    out = Belief(X_new, b.stamp_sec, b.z_lin - shift, b.L.copy(), b.h - b.L @ shift)
    return out, dict(frobenius_strength=s, delta_pose=dpc)


def anchor_drift_update(b: Belief):
    """anchor_drift.py:93-191."""
    dz = b.mean_increment()
    dpose = dz[0:6]
    dm, dr = float(np.linalg.norm(dpose[0:3])), float(np.linalg.norm(dpose[3:6]))
    rho = min(max(max(dm / ANCHOR_M0, dr / ANCHOR_R0), 0.0), 1.0)
    X_new = se3.se3_compose(b.X_anchor, se3.se3_exp(rho * dpose))
    z_new = (1.0 - rho) * dz
    out = Belief(X_new, b.stamp_sec, z_new, b.L.copy(), b.L @ z_new)
    return out, dict(anchor_drift_rho=rho)


# ================================================================ row 13: IW process noise
PROCESS_BLOCK_MASKS = np.zeros((7, 6, 6))
for _i, _d in enumerate(PROCESS_BLOCK_DIMS):
    PROCESS_BLOCK_MASKS[_i, :_d, :_d] = 1.0


def process_noise_iw_suffstats(L_pred, h_pred, L_post, h_post):
    """inverse_wishart_jax.py:71-123."""
    mu_pred, _ = spd_solve_lifted(L_pred, h_pred, EPS_LIFT)
    mu_post, _ = spd_solve_lifted(L_post, h_post, EPS_LIFT)
    Sig, _ = spd_inverse_lifted(L_post, EPS_LIFT)
    r = mu_post - mu_pred
    r_pad = np.zeros((7, 6))
    Sb = np.zeros((7, 6, 6))
    for i, (s0, d) in enumerate(zip(PROCESS_BLOCK_STARTS, PROCESS_BLOCK_DIMS)):
        r_pad[i, :d] = r[s0:s0 + d]
        Sb[i, :d, :d] = Sig[s0:s0 + d, s0:s0 + d]
    dPsi = (r_pad[:, :, None] * r_pad[:, None, :] + Sb) * PROCESS_BLOCK_MASKS
    return dPsi, np.ones(7)


def datasheet_process_noise_state():
    """create_datasheet_process_noise_state, structures/inverse_wishart_jax.py:42-80."""
    p = np.array(PROCESS_BLOCK_DIMS, np.float64)
    nu = p + 1.0 + IW_NU_WEAK_ADD
    sig = [1e-4, 8.7e-7, 9.5e-5, 1e-8, 1e-6, 1e-6, 1e-8]  # constants.py:225-237
    Psi = np.zeros((7, 6, 6))
    for i, d in enumerate(PROCESS_BLOCK_DIMS):
        Psi[i, :d, :d] = np.eye(d) * sig[i] * IW_NU_WEAK_ADD
    return nu, Psi


def process_noise_Q(nu, Psi):
    """process_noise_state_to_Q_jax, inverse_wishart_jax.py:35-68."""
    dims = np.array(PROCESS_BLOCK_DIMS, np.float64)
    denom = softplus(50.0 * (nu - dims - 1.0)) / 50.0 + 1e-12
    Qb = Psi / denom[:, None, None] * PROCESS_BLOCK_MASKS
    Q = np.zeros((22, 22))
    for i, s0 in enumerate(PROCESS_BLOCK_STARTS):
        e = min(s0 + 6, 22)
        Q[s0:e, s0:e] = Qb[i, :e - s0, :e - s0]
    return psd_project(Q, EPS_PSD)[0]


def process_noise_iw_apply(nu, Psi, dPsi, dnu, nu_max=1000.0):
    """process_noise_iw_apply_suffstats_jax, inverse_wishart_jax.py:126-185."""
    rho = np.array(IW_RHO)
    raw = (rho[:, None, None] * Psi + dPsi) * PROCESS_BLOCK_MASKS
    Psi_new = np.zeros_like(raw)
    dsum = 0.0
    for i in range(7):
        Psi_new[i], c = psd_project(raw[i], EPS_PSD)
        dsum += c[0]
    nu_raw = rho * nu + dnu
    nu_min = np.array(PROCESS_BLOCK_DIMS, np.float64) + 1.0 + IW_NU_WEAK_ADD
    nu_floor = nu_min + softplus(nu_raw - nu_min)
    nu_new = nu_max - softplus(nu_max - nu_floor)
    return nu_new, Psi_new, np.array([dsum, np.abs(nu_new - nu_raw).sum()])


# ================================================================ row 13: IW measurement noise
MEAS_RHO = (0.995, 0.995, 0.99)            # gyro, accel, lidar: constants.py:279-281
MEAS_SIGMA = (8.7e-7, 9.5e-5, 0.01)        # constants.py:190,201,210


def datasheet_measurement_noise_state():
    """create_datasheet_measurement_noise_state, structures/measurement_noise_iw_jax.py:37-68:
    nu = p + 1 + 0.5, Psi = Sigma_prior * 0.5 per block [gyro, accel, lidar]."""
    nu = np.full(3, 3.0 + 1.0 + IW_NU_WEAK_ADD)
    Psi = np.stack([np.eye(3) * s * IW_NU_WEAK_ADD for s in MEAS_SIGMA])
    return nu, Psi


def _weighted_outer_psd(w, r):
    """sum_m w_norm[m] r_m r_m^T symmetrised and PSD-projected (measurement_noise_iw_jax.py:150-157)."""
    w_norm = w / (w.sum() + EPS_MASS)
    rrT = np.einsum("m,mi,mj->ij", w_norm, r, r)
    return psd_project(0.5 * (rrT + rrT.T), EPS_PSD)[0]


def imu_meas_iw_suffstats(imu_stamps, imu_gyro, imu_accel, w_int, gyro_bias, accel_bias, rotvec0, gravity_W):
    """Gyro + accel measurement-noise IW statistics of one scan: the pipeline's dt_imu, valid mask
    and omega_avg (FS/backend/pipeline.py:522-566, summed at :1024-1025) around
    imu_gyro_meas_iw_suffstats_from_avg_rate_jax (measurement_noise_iw_jax.py:130-167) and
    imu_accel_meas_iw_suffstats_from_gravity_dir_jax (:170-218).  Returns dPsi (3,3,3), dnu (3,)."""
    stamps = np.asarray(imu_stamps, np.float64).reshape(-1)
    valid = stamps > 0.0
    n_valid = int(valid.sum())
    dt_imu = float((stamps[valid].max() - stamps[valid].min()) / max(n_valid - 1, 1)) if n_valid >= 2 else 0.0
    dt_imu = max(dt_imu, 1e-12)
    w = np.asarray(w_int, np.float64) * valid.astype(np.float64)
    g_db = np.asarray(imu_gyro, np.float64) - np.asarray(gyro_bias)[None, :]
    omega_avg = np.einsum("m,mi->i", w / (w.sum() + EPS_MASS), g_db)
    if not np.all(np.isfinite(omega_avg)):
        raise ValueError(f"omega_avg contains non-finite values: {omega_avg}")
    dPsi = np.zeros((3, 3, 3))
    dPsi[0] = _weighted_outer_psd(w, g_db - omega_avg[None, :]) * dt_imu
    f_pred = -(se3.so3_exp(np.asarray(rotvec0, np.float64)).T @ np.asarray(gravity_W, np.float64))
    r_a = (np.asarray(imu_accel, np.float64) - np.asarray(accel_bias)[None, :]) - f_pred[None, :]
    dPsi[1] = _weighted_outer_psd(w, r_a) * dt_imu
    return dPsi, np.array([1.0, 1.0, 0.0])


def measurement_noise_iw_apply(nu, Psi, dPsi, dnu, nu_max=1000.0):
    """measurement_noise_apply_suffstats_jax, measurement_noise_iw_jax.py:59-100."""
    rho = np.array(MEAS_RHO)
    raw = rho[:, None, None] * Psi + dPsi
    raw = 0.5 * (raw + np.swapaxes(raw, -1, -2))
    Psi_new = np.zeros_like(raw)
    dsum = 0.0
    for i in range(3):
        Psi_new[i], c = psd_project(raw[i], EPS_PSD)
        dsum += c[0]
    nu_raw = rho * nu + dnu
    nu_min = 3.0 + 1.0 + IW_NU_WEAK_ADD
    nu_floor = nu_min + softplus(nu_raw - nu_min)
    nu_new = nu_max - softplus(nu_max - nu_floor)
    return nu_new, Psi_new, np.array([dsum, np.abs(nu_new - nu_raw).sum()])


# ================================================================ row 14: hypothesis combine
def hypothesis_barycenter(L_stack, h_stack, z_stack, weights):
    """_hypothesis_barycenter_core, hypothesis.py:51-117."""
    w = np.maximum(np.asarray(weights, np.float64), HYP_WEIGHT_FLOOR)
    wn = w / w.sum()
    L_raw = np.einsum("k,kij->ij", wn, L_stack)
    h = np.einsum("k,ki->i", wn, h_stack)
    z = np.einsum("k,ki->i", wn, z_stack)
    L, cert = psd_project(L_raw, EPS_PSD)
    mus = np.stack([spd_solve_lifted(L_stack[k], h_stack[k], EPS_LIFT)[0] for k in range(len(wn))])
    mom = np.einsum("k,ki->i", wn, mus)
    spread = float(np.sum(wn * np.sum((mus - mom[None]) ** 2, axis=1)))
    return dict(L=L, h=h, z_lin=z, weights=wn, psd_projection_delta=cert[0], spread=spread,
                L_raw=L_raw)
