"""Seeded synthetic LiDAR+IMU scans (SURVEY.md section 8(d) "Synthetic inputs").

VLP-16-like scanner: 16 rings at -15..+15 deg (2 deg steps), N/16 azimuths per ring swept over
0.1 s, azimuth-major firing order.  Ranges are ray-cast against a box room (walls x=+-10 m,
y=+-6 m, floor z=0, ceiling z=3 m) from a sensor 0.5 m above the base origin, with 1 cm range
noise.  The body moves with a constant twist (v=(1,0,0) m/s, w=(0,0,0.3) rad/s) so deskew has
work to do; points are expressed in the base frame at their own capture time.  Weights follow
the reference parse law (FS/backend/backend_node.py:448-459).  IMU at 200 Hz, padded to 512.
Odometry (the node's odom_pose / odom_cov_se3 / odom_twist / odom_twist_cov, backend_node.py:
1453-1535): the true base pose at the scan stamp t_scan plus N(0, (1 cm, 0.2 deg)) noise, and the
true body twist plus N(0, (2 cm/s, 0.5 deg/s)) noise, with matching diagonal covariances.
"""

from __future__ import annotations

import math

import numpy as np

LIDAR_ORIGIN = np.array([0.0, 0.0, 0.5])
V_BODY = np.array([1.0, 0.0, 0.0])
W_BODY = np.array([0.0, 0.0, 0.3])
SCAN_PERIOD = 0.1
IMU_RATE = 200.0
IMU_LEN = 512
T0 = 100.0


def _rot_z(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def body_pose(t):
    """World pose of the base at time t (planar constant twist from the origin at T0)."""
    dt = t - T0
    yaw = W_BODY[2] * dt
    w = W_BODY[2]
    # integrate v_body rotated by yaw(t): x = sin(w dt)/w, y = (1-cos(w dt))/w
    x = V_BODY[0] * math.sin(yaw) / w
    y = V_BODY[0] * (1.0 - math.cos(yaw)) / w
    return np.array([x, y, 0.0]), _rot_z(yaw)


def _raycast(origin, dirs):
    """Distance along unit dirs (M,3) from world origin to the first room plane."""
    big = np.full(dirs.shape[0], np.inf)
    for axis, lo, hi in ((0, -10.0, 10.0), (1, -6.0, 6.0), (2, 0.0, 3.0)):
        dcomp = dirs[:, axis]
        with np.errstate(divide="ignore", invalid="ignore"):
            t_hi = (hi - origin[axis]) / dcomp
            t_lo = (lo - origin[axis]) / dcomp
        t = np.where(dcomp > 0, t_hi, np.where(dcomp < 0, t_lo, np.inf))
        big = np.minimum(big, t)
    return big


def make_scan(n_points: int, scan_index: int = 0, seed: int = 0, noise: float = 0.01):
    """One scan of n_points (multiple of 16).  Returns dict with f32 xyz in a 16-byte
    PointCloud2-like record (x, y, z, intensity) plus f64 timestamps/weights and the IMU window."""
    rng = np.random.default_rng(seed + 7919 * scan_index)
    n_az = n_points // 16
    assert n_az * 16 == n_points, "n_points must be a multiple of 16"
    t_start = T0 + SCAN_PERIOD * scan_index
    elev = np.deg2rad(np.arange(-15.0, 16.0, 2.0))                # 16 rings
    az_frac = np.arange(n_az) / n_az
    az = 2.0 * math.pi * az_frac
    A, E = np.meshgrid(az, elev, indexing="ij")                     # azimuth-major order
    t = t_start + np.repeat(az_frac * SCAN_PERIOD, 16)
    d_sensor = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], -1).reshape(-1, 3)
    pts_base = np.empty((n_points, 3))
    ranges = np.empty(n_points)
    # ray-cast per azimuth column (pose changes over the sweep)
    for j in range(n_az):
        sl = slice(16 * j, 16 * j + 16)
        p_w, R_w = body_pose(t[16 * j])
        o_w = p_w + R_w @ LIDAR_ORIGIN
        dw = d_sensor[sl] @ R_w.T
        r = _raycast(o_w, dw) + noise * rng.standard_normal(16)
        ranges[sl] = r
        pts_base[sl] = LIDAR_ORIGIN[None, :] + d_sensor[sl] * r[:, None]
    sig = lambda x: 1.0 / (1.0 + np.exp(-x))  # noqa: E731
    w = sig((ranges - 0.5) / 0.25) * sig((50.0 - ranges) / 0.25) * (1.0 - 1e-12) + 1e-12
    rec = np.zeros((n_points, 4), np.float32)
    rec[:, :3] = pts_base.astype(np.float32)
    rec[:, 3] = 1.0
    # IMU window covering (t_start - 0.2, t_start + 0.35], padded with zeros to 512
    m = int(0.55 * IMU_RATE)
    imu_t = np.zeros(IMU_LEN)
    imu_t[:m] = t_start - 0.2 + np.arange(1, m + 1) / IMU_RATE
    gyro = np.zeros((IMU_LEN, 3))
    accel = np.zeros((IMU_LEN, 3))
    gyro[:m] = W_BODY[None, :] + 1e-3 * rng.standard_normal((m, 3))
    a_body = np.cross(W_BODY, V_BODY) + np.array([0.0, 0.0, 9.81])
    accel[:m] = a_body[None, :] + 1e-2 * rng.standard_normal((m, 3))
    # odometry at the scan stamp (drawn after the LiDAR and IMU noise, so those inputs are unchanged)
    t_scan = t_start + SCAN_PERIOD
    p_w, _ = body_pose(t_scan)
    sd_pose = np.array([0.01, 0.01, 0.01, np.deg2rad(0.2), np.deg2rad(0.2), np.deg2rad(0.2)])
    odom_pose = np.concatenate([p_w, [0.0, 0.0, W_BODY[2] * (t_scan - T0)]]) + sd_pose * rng.standard_normal(6)
    sd_twist = np.array([0.02, 0.02, 0.02, np.deg2rad(0.5), np.deg2rad(0.5), np.deg2rad(0.5)])
    odom_twist = np.concatenate([V_BODY, W_BODY]) + sd_twist * rng.standard_normal(6)
    return dict(xyz_record=rec, points=rec[:, :3].astype(np.float64), timestamps=t, weights=w,
                imu_stamps=imu_t, imu_gyro=gyro, imu_accel=accel, scan_start_time=t_start,
                scan_end_time=t_start + SCAN_PERIOD, dt_sec=SCAN_PERIOD,
                t_last_scan=t_start - SCAN_PERIOD, t_scan=t_scan,
                odom_pose=odom_pose, odom_cov_se3=np.diag(sd_pose ** 2), odom_twist=odom_twist,
                odom_twist_cov=np.diag(sd_twist ** 2))


ODOM_KEYS = ("odom_pose", "odom_cov_se3", "odom_twist", "odom_twist_cov")


def odom_kwargs(sc):
    """The scan's odometry as HypothesisContext.scan keyword arguments."""
    return {k: sc[k] for k in ODOM_KEYS if k in sc}


def scan_kwargs(sc):
    """Every host-side input of HypothesisContext.scan held by a scan dict (IMU window, times,
    scan-to-scan window, odometry)."""
    kw = {k: sc[k] for k in ("imu_stamps", "imu_gyro", "imu_accel", "scan_start_time", "scan_end_time", "dt_sec")}
    for k in ("t_last_scan", "t_scan"):
        if k in sc:
            kw[k] = sc[k]
    kw.update(odom_kwargs(sc))
    return kw
