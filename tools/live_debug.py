"""Diagnostics of one live-path scan: GPU drop-in vs oracle (surfel batch, per-tile counts)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd")]
import numpy as np
from gcslam import synthetic, primitive_map as gpm
from gcslam.pipeline import BeliefGaussianInfo, PipelineConfig, process_scan_single_hypothesis
from oracle import ops, pipeline as opipe, primitive_map as opm

N, m = 8192, 4096
cfg = PipelineConfig(K_HYP=1, N_POINTS_CAP=N, B_BINS=48, lidar_origin_base=(0, 0, 0.5), max_raw_points=N,
                     primitive_map_max_size=m, R_ACTIVE_TILES_Z=1, R_STENCIL_TILES_Z=1, N_ACTIVE_TILES=21,
                     N_STENCIL_TILES=21)
ctx = cfg.make_context()
am = gpm.create_empty_atlas_map(m_tile=m, max_tiles=64)
ocfg = opipe.PrimitivePathConfig(n_points_cap=N, lidar_origin=(0, 0, 0.5), m_tile=m, r_active_z=1, r_stencil_z=1)
Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
sc = synthetic.make_scan(N, 70)
res = process_scan_single_hypothesis(BeliefGaussianInfo.create_identity_prior(), sc["points"], sc["timestamps"],
                                     sc["weights"], None, None, sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"],
                                     sc["odom_pose"], sc["odom_cov_se3"], sc["scan_start_time"], sc["scan_end_time"],
                                     sc["dt_sec"], sc["t_last_scan"], sc["t_scan"], Q, cfg, sc["odom_twist"],
                                     sc["odom_twist_cov"], None, 0, primitive_map=am, map_bins=ctx)
tiles = {}
ref = opipe.process_scan_primitive_path(ops.Belief.identity_prior(), sc, Q, ocfg, tiles, 0, 0)
gb = res.measurement_batch
ob = ref["surfels"]
for f in ("weights", "thetas", "Lambdas", "etas"):
    g = getattr(gb, f).cpu().numpy()
    o = ob[f]
    print(f, "max abs diff", np.abs(g - o).max(), "max", np.abs(o).max())
print("valid eq", np.array_equal(gb.valid_mask.cpu().numpy().astype(bool), ob["valid_mask"]))
print("z_t diff", np.abs(res.z_t - ref["z_t"]).max())
print("gpu", {k: getattr(res.map_update_cert, k) for k in ("insert_count_total", "fused_count", "evicted_count", "merged_count", "insert_mass_total", "evicted_mass_total")})
print("ref", ref["map_update"])
w = ob["weights"][ob["valid_mask"]]
print("surfel weights: min", w.min(), "median", np.median(w), "n", w.size, "a", 1.0 / w.size, "a*w<1e-4:", int(np.sum(w / w.size < 1e-4)))
for tid in ref["active_tile_ids"]:
    g = am.read_tile(int(tid))
    o = tiles[int(tid)]
    if int(g["valid_mask"].sum()) != int(o["valid_mask"].sum()) or not np.array_equal(g["valid_mask"], o["valid_mask"]):
        gw, ow = g["weights"], o["weights"]
        d = np.where(g["valid_mask"] != o["valid_mask"])[0]
        print("tile", tid, "valid gpu", int(g["valid_mask"].sum()), "ref", int(o["valid_mask"].sum()), "diff slots", d[:10],
              "w gpu", gw[d[:5]], "w ref", ow[d[:5]], "ids", g["primitive_ids"][d[:5]], o["primitive_ids"][d[:5]])
