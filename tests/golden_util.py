"""Loading the committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)."""

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ORIGIN = np.array([0.0, 0.0, 0.5])


def load(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def scan_dict(g, s):
    """Scan s of a scan_* fixture as the oracle pipeline's input dict."""
    rec = g["in_xyz_record"][s]
    return dict(xyz_record=rec, points=rec[:, :3].astype(np.float64), timestamps=g["in_timestamps"][s],
                weights=g["in_weights"][s], imu_stamps=g["in_imu_stamps"][s], imu_gyro=g["in_imu_gyro"][s],
                imu_accel=g["in_imu_accel"][s], scan_start_time=float(g["in_scan_start_time"][s]),
                scan_end_time=float(g["in_scan_end_time"][s]), dt_sec=float(g["in_dt_sec"][s]),
                t_last_scan=float(g["in_t_last_scan"][s]), t_scan=float(g["in_t_scan"][s]),
                **{k: g[f"in_{k}"][s] for k in ("odom_pose", "odom_cov_se3", "odom_twist", "odom_twist_cov")
                   if f"in_{k}" in g})
