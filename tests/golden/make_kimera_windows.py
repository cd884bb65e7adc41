#!/usr/bin/env python3
"""Real-sensor IMU / odometry scan windows from the reference's raw sensor dump (data only).

Source: /root/reference/docs/raw_sensor_dump/ (the first 300 IMU messages of the Kimera
10_14_acl_jackal-005 bag with the IMU extrinsic applied -- base frame, rad/s and m/s^2 -- and
the first 300 /odom messages; README.md there).  This container has the reference; the GPU box does
not, so the windows are committed as tests/golden/kimera_imu_odom_windows.npz.

For 11 scan stamps t_scan = t0 + 0.25 + 0.1 k the fixture holds the node's per-scan inputs
(FS/backend/backend_node.py:1927-1952 IMU slice padded to 512 slots, :1453-1535 odometry relative to
the first odom pose, pose as [t, rotvec]):
  imu window  (t_scan - 0.25, t_scan + 0.05], zero-padded to 512 (stamps 0 = padding)
  odometry    the sample nearest t_scan; the dump holds no covariances, so they are DECLARED:
              pose diag(1e-3 m^2 x3, 1e-4 rad^2 x3), twist diag(0.1^2 x3, 0.01^2 x3)
              (GC_ODOM_TWIST_VEL_SIGMA / GC_ODOM_TWIST_WZ_SIGMA, constants.py:324-328)
Stamps are shifted by -t0 + 100 s (the IMU window math uses differences; the shift keeps them > 0).

Usage: python tests/golden/make_kimera_windows.py
"""

import csv
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT]
from oracle import se3  # noqa: E402

DUMP = "/root/reference/docs/raw_sensor_dump"
M = 512
T_SHIFT = 100.0


def read(name):
    with open(os.path.join(DUMP, name)) as f:
        r = csv.reader(f)
        next(r)
        return np.array([[float(x) for x in row] for row in r])


def quat_to_rotvec(qx, qy, qz, qw):
    q = np.array([qx, qy, qz, qw]) / np.linalg.norm([qx, qy, qz, qw])
    x, y, z, w = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    return se3.so3_log(R)


def main():
    imu = read("imu_extrinsic_applied_first_300.csv")
    odom = read("odom_raw_first_300.csv")
    t0 = imu[0, 0]
    imu_t = imu[:, 0] - t0 + T_SHIFT
    od_t = odom[:, 0] - t0 + T_SHIFT
    od_pose = np.stack([np.concatenate([r[1:4], quat_to_rotvec(*r[4:8])]) for r in odom])
    first_inv = se3.se3_inverse(od_pose[0])
    od_rel = np.stack([se3.se3_compose(first_inv, p) for p in od_pose])
    od_twist = odom[:, 8:14]
    out = {k: [] for k in ("imu_stamps", "imu_gyro", "imu_accel", "t_scan", "t_last_scan", "odom_pose",
                           "odom_twist")}
    for k in range(11):
        ts = T_SHIFT + 0.25 + 0.1 * k
        sel = (imu_t > ts - 0.25) & (imu_t <= ts + 0.05)
        n = int(sel.sum())
        st, gy, ac = np.zeros(M), np.zeros((M, 3)), np.zeros((M, 3))
        st[:n], gy[:n], ac[:n] = imu_t[sel], imu[sel, 1:4], imu[sel, 4:7]
        j = int(np.argmin(np.abs(od_t - ts)))
        out["imu_stamps"].append(st)
        out["imu_gyro"].append(gy)
        out["imu_accel"].append(ac)
        out["t_scan"].append(ts)
        out["t_last_scan"].append(ts - 0.1)
        out["odom_pose"].append(od_rel[j])
        out["odom_twist"].append(od_twist[j])
    res = {k: np.stack([np.asarray(x, np.float64) for x in v]) for k, v in out.items()}
    res["odom_cov_se3"] = np.diag([1e-3] * 3 + [1e-4] * 3)
    res["odom_twist_cov"] = np.diag([0.1 ** 2] * 3 + [0.01 ** 2] * 3)
    path = os.path.join(HERE, "kimera_imu_odom_windows.npz")
    np.savez_compressed(path, **res)
    print(f"{path}: {os.path.getsize(path) / 1024:.0f} KiB, samples per window",
          [(s > 0).sum() for s in res["imu_stamps"]])


if __name__ == "__main__":
    main()
