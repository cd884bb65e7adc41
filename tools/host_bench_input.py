"""Inputs of tools/host_bench.cpp: the belief after three dense scans (golden fixture), the
datasheet Q and one synthetic IMU window, as raw f64."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd"), os.path.join(ROOT, "tests")]
from golden_util import load
from gcslam import synthetic
from oracle import ops
g = load("scan_dense_b48")
sc = synthetic.make_scan(16, 3)
Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
buf = np.concatenate([g["out_L"][2].ravel(), g["out_h"][2], Q.ravel(), sc["imu_stamps"], sc["imu_gyro"].ravel(),
                      sc["imu_accel"].ravel(), [sc["scan_start_time"], sc["scan_end_time"], sc["t_last_scan"],
                                                sc["t_scan"]], np.zeros(12)])
buf.astype(np.float64).tofile(os.path.join(ROOT, "tools", "host_bench_in.bin"))
