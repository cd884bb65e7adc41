#!/usr/bin/env python3
"""Host-side (Python) profile of the live primitive path: the drop-in
process_scan_single_hypothesis(..., primitive_map=) at the reference sizes (the bench's live_path
setup), under cProfile over N calls after a warm-up; prints the functions by total and cumulative
time, so the Python share of a call (tensor conversion, result allocation, ctypes marshalling) can
be told from the C-ABI calls.

  python tools/live_prof.py [calls=20]
"""

import cProfile
import os
import pstats
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch
    from gcslam import synthetic, primitive_map as gpm
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, datasheet_process_noise_state,
                                 process_noise_state_to_Q, process_scan_single_hypothesis)
    N = 8192
    cfg = PipelineConfig(K_HYP=1, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense",
                         lidar_origin_base=tuple(synthetic.LIDAR_ORIGIN), max_raw_points=N, device=0)
    ctx = cfg.make_context()
    am = gpm.create_empty_atlas_map(m_tile=cfg.primitive_map_max_size, max_tiles=512, device=0)
    Q = process_noise_state_to_Q(datasheet_process_noise_state())
    warm = 10
    scans = [synthetic.make_scan(N, k) for k in range(warm + calls)]
    state = dict(belief=BeliefGaussianInfo.create_identity_prior(), seq=0)

    def one(sc):
        r = process_scan_single_hypothesis(
            belief_prev=state["belief"], raw_points=sc["points"], raw_timestamps=sc["timestamps"],
            raw_weights=sc["weights"], raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8),
            imu_stamps=sc["imu_stamps"], imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
            odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"], scan_end_time=sc["scan_end_time"],
            dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"], t_scan=sc["t_scan"], Q=Q, config=cfg,
            odom_twist=sc["odom_twist"], odom_twist_cov=sc["odom_twist_cov"], camera_batch=None,
            scan_seq=state["seq"], primitive_map=am, map_bins=ctx)
        state["belief"] = r.belief_updated
        state["seq"] += 1

    for k in range(warm):
        one(scans[k])
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    prof.enable()
    for k in range(calls):
        one(scans[warm + k])
    torch.cuda.synchronize()
    prof.disable()
    st = pstats.Stats(prof)
    print(f"live path, {calls} calls (per-call times: divide by {calls})")
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
