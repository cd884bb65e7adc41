"""ctypes binding of libgcslam_hip.so (include/gcslam_hip.h).

The library is loaded from this package directory.  There is no CPU fallback: a missing or
unloadable library raises at import time of the operators (docs/GC_SLAM.md:130 forbids
"GPU if available else CPU"; so does the north star).
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

LIB_NAME = "libgcslam_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

ABI_VERSION = 4  # include/gcslam_hip.h GCS_ABI_VERSION
D_Z = 22
CERT_LEN = 64
PAYLOAD_LEN = 840
SCAN_FIELDS = 26
MAP_FIELDS = 26
DERIVED_FIELDS = 16
MODE_DENSE, MODE_SCALE = 0, 1

c_double_p = C.POINTER(C.c_double)
c_int32_p = C.POINTER(C.c_int32)
c_int64_p = C.POINTER(C.c_int64)


class GcsConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_bins", C.c_int32), ("n_points_cap", C.c_int32),
                ("max_raw_points", C.c_int32), ("mode", C.c_int32), ("k_cand", C.c_int32),
                ("tau", C.c_double), ("lidar_origin", C.c_double * 3), ("deskew_rotation_only", C.c_int32),
                ("forgetting_factor", C.c_double), ("gravity_W", C.c_double * 3),
                ("use_imu_odom", C.c_int32), ("imu_gravity_scale", C.c_double), ("planar_z_ref", C.c_double),
                ("planar_z_sigma", C.c_double), ("planar_vz_sigma", C.c_double), ("alpha_min", C.c_double),
                ("alpha_max", C.c_double), ("c0_cond", C.c_double)]


class GcsScanInputs(C.Structure):
    # host arrays as plain addresses (arr.ctypes.data): a typed-pointer conversion costs ~2 us each
    _fields_ = [("xyz_dev", C.c_void_p), ("point_step", C.c_int32), ("timestamps_dev", C.c_void_p),
                ("weights_dev", C.c_void_p), ("n_points", C.c_int32), ("imu_stamps", C.c_void_p),
                ("imu_gyro", C.c_void_p), ("imu_accel", C.c_void_p), ("imu_len", C.c_int32),
                ("scan_start_time", C.c_double), ("scan_end_time", C.c_double), ("dt_sec", C.c_double),
                ("Q", C.c_void_p), ("L_ext", C.c_void_p), ("h_ext", C.c_void_p),
                ("t_last_scan", C.c_double), ("t_scan", C.c_double), ("xyz_format", C.c_int32),
                ("odom_pose", C.c_void_p), ("odom_cov_se3", C.c_void_p), ("odom_twist", C.c_void_p),
                ("odom_twist_cov", C.c_void_p), ("Sigma_g", C.c_void_p), ("Sigma_a", C.c_void_p)]


class GcsPointCloud2Layout(C.Structure):
    _fields_ = [("n_points", C.c_int32), ("point_step", C.c_int32), ("off_x", C.c_int32), ("off_y", C.c_int32),
                ("off_z", C.c_int32), ("off_ring", C.c_int32), ("ring_datatype", C.c_int32), ("off_t", C.c_int32),
                ("t_datatype", C.c_int32), ("header_stamp_sec", C.c_double), ("R_base_lidar", C.c_double * 9),
                ("t_base_lidar", C.c_double * 3)]


class GcsBelief(C.Structure):
    _fields_ = [("X_anchor", C.c_double * 6), ("stamp_sec", C.c_double), ("z_lin", C.c_double * D_Z),
                ("L", C.c_double * (D_Z * D_Z)), ("h", C.c_double * D_Z)]


class GcsScanOutputs(C.Structure):
    _fields_ = [("belief", GcsBelief), ("iw_process_dPsi", C.c_double * 252), ("iw_process_dnu", C.c_double * 7),
                ("z_t", C.c_double * 6), ("L_evidence", C.c_double * (D_Z * D_Z)), ("h_evidence", C.c_double * D_Z),
                ("R_mf", C.c_double * 9), ("t_wls", C.c_double * 3), ("cert", C.c_double * CERT_LEN),
                ("stage_ms", C.c_double * 8), ("iw_meas_dPsi", C.c_double * 27), ("iw_meas_dnu", C.c_double * 3),
                ("L_imu_odom", C.c_double * (D_Z * D_Z)), ("h_imu_odom", C.c_double * D_Z),
                ("imu_odom_certs", C.c_double * 77)]


class GcsScanBeginOutputs(C.Structure):
    _fields_ = [("z_lin_pose", C.c_double * 6), ("pose_pred", C.c_double * 6), ("n_points", C.c_int32),
                ("n_selected", C.c_int32), ("points_dev", C.c_void_p), ("timestamps_dev", C.c_void_p),
                ("weights_dev", C.c_void_p), ("deskew_ess", C.c_double), ("deskew_support", C.c_double),
                ("cert", C.c_double * CERT_LEN)]


class GcsLidarEvidence(C.Structure):
    _fields_ = [("L_lidar", C.c_void_p), ("h_lidar", C.c_void_p), ("trigger_sum", C.c_double),
                ("ess_sum", C.c_double), ("n_certs", C.c_int32), ("nll_sum", C.c_double)]


class GcsImuOdomInputs(C.Structure):
    _fields_ = [("m", C.c_int32), ("stamps", C.c_void_p), ("gyro", C.c_void_p), ("accel", C.c_void_p),
                ("w_int", C.c_void_p), ("t_last_scan", C.c_double), ("t_scan", C.c_double), ("dt_sec", C.c_double),
                ("pose0", C.c_void_p), ("pose_pred", C.c_void_p), ("mu_prev", C.c_void_p), ("mu_inc", C.c_void_p),
                ("gravity_W", C.c_void_p), ("Sigma_g", C.c_void_p), ("Sigma_a", C.c_void_p),
                ("odom_pose", C.c_void_p), ("odom_cov_se3", C.c_void_p), ("odom_twist", C.c_void_p),
                ("odom_twist_cov", C.c_void_p), ("planar_z_ref", C.c_double), ("planar_z_sigma", C.c_double),
                ("planar_vz_sigma", C.c_double)]


IMU_ODOM_CERT_LEN = 15
RCCL_ID_BYTES = 128
DEBUG_SCAN_SPIN_LIMIT, DEBUG_INJECT_SCAN_FAIL = 1, 2
DEBUG_SORTED_BUCKETS, DEBUG_BUCKET_CAPACITY = 3, 4
DEBUG_LAUNCH_GATE = 5
DEBUG_POINT_KERNEL = 6
DEBUG_DEVICE_PREINT = 7
DEBUG_PT_CLEAR = 8
DEBUG_MIRROR_TORN = 9
DEBUG_SENDBUF = 10
DEBUG_DEVICE_IMU_ODOM = 11
DEBUG_COMBINE_DELAY = 12
MAP_OWN, MAP_LEAD, MAP_FOLLOW, MAP_REC_LEN = 0, 1, 2, 48


# (name, restype, argtypes) for every symbol declared in include/gcslam_hip.h
class GcsSurfelConfig(C.Structure):
    _fields_ = [("n_surfel", C.c_int32), ("n_feat", C.c_int32), ("voxel_size_m", C.c_double),
                ("num_cells_1", C.c_int32), ("num_cells_2", C.c_int32), ("num_cells_z", C.c_int32),
                ("max_occupants", C.c_int32), ("min_points_per_voxel", C.c_int32),
                ("sensor_noise_var_per_axis", C.c_double), ("wishart_nu", C.c_double),
                ("wishart_psi_scale", C.c_double), ("kappa_main_scale", C.c_double), ("kappa_min", C.c_double),
                ("kappa_max", C.c_double), ("eig_min", C.c_double), ("eps_lift", C.c_double),
                ("max_points", C.c_int32), ("device", C.c_int32)]


class GcsSurfelOutputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("positions", "covariances", "normals", "kappas", "weights", "timestamps",
                                          "Lambdas", "thetas", "etas", "colors", "valid_mask", "source_indices",
                                          "cell_ids", "bucket", "count", "sources")] + \
               [("center", C.c_double * 3), ("n_valid", C.c_int32), ("cert", C.c_double * 2)]


GCS_ASSOC_CERT_LEN = 21
ASSOC_CERT_FIELDS = ("marginal_defect_a", "marginal_defect_b", "transport_mass_total", "sum_a", "sum_b", "sum_m",
                     "sum_novel", "p95_a", "p95_b", "nonzero_a", "nonzero_b", "b_recency_p95", "ess_total",
                     "mass_epsilon_ratio", "total_cost", "support_frac", "exact", "map_valid",
                     "cand_tiles_mean", "cand_prims_mean", "cand_prims_p95")


class GcsAssocConfig(C.Structure):
    _fields_ = [("k_assoc", C.c_int32), ("k_sinkhorn", C.c_int32), ("beta", C.c_double), ("epsilon", C.c_double),
                ("tau_a", C.c_double), ("tau_b", C.c_double), ("cost_subtract_row_min", C.c_int32),
                ("cost_scale_by_median", C.c_int32), ("a_policy", C.c_int32), ("b_policy", C.c_int32),
                ("eps_mass", C.c_double), ("eps_lift", C.c_double), ("eps_mass_dir", C.c_double), ("h_tile", C.c_double),
                ("r_stencil_tiles_xy", C.c_int32), ("r_stencil_tiles_z", C.c_int32), ("scan_seq", C.c_int64),
                ("recency_decay_lambda", C.c_double)]


class GcsAssocMeas(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("Lambdas", "thetas", "etas", "weights", "valid_mask")] + \
               [("n_total", C.c_int32), ("n_lobes", C.c_int32), ("n_valid", C.c_int32)]


class GcsAssocView(C.Structure):
    _fields_ = [("tile_ids", C.c_void_p), ("n_tiles", C.c_int32), ("m_tile_view", C.c_int32)] + \
               [(n, C.c_void_p) for n in ("positions", "directions", "kappas", "valid_mask",
                                          "last_supported_scan_seq", "candidate_tile_ids", "candidate_slots")]


# primitive map (gcs_pmap_*): field codes, view outputs and proposal / contribution rows
PM_FIELDS = ("Lambdas", "thetas", "etas", "weights", "timestamps", "created_timestamps", "colors", "cam_mass",
             "lidar_mass", "rgb_cam_accum", "rgb_cam_denom", "rgb", "last_supported_scan_seq", "last_update_scan_seq",
             "primitive_ids", "valid_mask")


class GcsPmapView(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("positions", "covariances", "directions", "kappas", "weights",
                                          "primitive_ids", "valid_mask", "last_supported_scan_seq", "etas", "colors",
                                          "candidate_slots", "candidate_tile_ids")]


class GcsPmapRows(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("Lambdas", "thetas", "etas", "weights", "responsibilities", "valid",
                                          "colors", "sources", "tile_pos", "slots")] + [("n", C.c_int32)]


class GcsPmapUpdateConfig(C.Structure):
    _fields_ = [("k_insert_tile", C.c_int32), ("block_size", C.c_int32), ("k_merge_pairs", C.c_int32),
                ("merge_max_tile_size", C.c_int32), ("h_tile", C.c_double), ("recency_decay_lambda", C.c_double),
                ("cull_threshold", C.c_double), ("forgetting_factor", C.c_double), ("merge_threshold", C.c_double),
                ("eps_lift", C.c_double), ("eps_mass", C.c_double), ("eps_psd", C.c_double)]


class GcsPmapUpdateInputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("Lambdas", "thetas", "etas", "weights", "valid", "colors", "sources")] + \
               [("n_total", C.c_int32), ("n_lobes", C.c_int32)] + \
               [(n, C.c_void_p) for n in ("responsibilities", "candidate_tile_ids", "candidate_slots", "row_masses")] + \
               [("k_assoc", C.c_int32)]


class GcsPmapUpdateStats(C.Structure):
    _fields_ = [("fused_count", C.c_int32), ("insert_count_total", C.c_int32), ("evicted_count", C.c_int32),
                ("merged_count", C.c_int32), ("fused_mass_total", C.c_double), ("insert_mass_total", C.c_double),
                ("insert_mass_p95", C.c_double), ("evicted_mass_total", C.c_double)]


class GcsVpeOutputs(C.Structure):
    _fields_ = [("L_pose", C.c_double * (D_Z * D_Z)), ("h_pose", C.c_double * D_Z), ("L_trans", C.c_double * 9),
                ("h_trans", C.c_double * 3), ("L_rot", C.c_double * 9), ("h_rot", C.c_double * 3),
                ("total_weighted_cost", C.c_double), ("mean_transported_mass", C.c_double), ("ess_total", C.c_double),
                ("support_frac", C.c_double), ("n_associations", C.c_int32), ("exact", C.c_int32)]


class GcsAssocOutputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("responsibilities", "candidate_pool_indices", "candidate_tile_ids",
                                          "candidate_slots", "row_masses", "cost_matrix")] + \
               [("cert", C.c_double * GCS_ASSOC_CERT_LEN), ("exact", C.c_int32), ("n_map_valid", C.c_int32)]


LIVE_MAX_TILES = 64


class GcsLiveArgs(C.Structure):
    _fields_ = [("surfels", C.c_void_p), ("assoc", C.c_void_p), ("map", C.c_void_p),
                ("n_tiles", C.c_int32), ("tile_ids", C.c_void_p), ("tile_slots", C.c_void_p), ("n_free", C.c_int32),
                ("free_slots", C.c_void_p), ("slot_written", C.c_void_p), ("next_global_id", C.c_int64),
                ("h_tile", C.c_double), ("r_active_xy", C.c_int32), ("r_active_z", C.c_int32),
                ("r_stencil_xy", C.c_int32), ("r_stencil_z", C.c_int32), ("n_active_expected", C.c_int32),
                ("n_stencil_expected", C.c_int32), ("scan_seq", C.c_int64), ("recency_lambda", C.c_double),
                ("recency_min_scale", C.c_double), ("m_tile_view", C.c_int32), ("eps_lift", C.c_double),
                ("eps_mass", C.c_double), ("assoc_cfg", C.c_void_p), ("update_cfg", C.c_void_p),
                ("timestamp", C.c_double), ("points_dev", C.c_void_p), ("timestamps_dev", C.c_void_p),
                ("weights_dev", C.c_void_p), ("n_points", C.c_int32), ("surfel_out", C.c_void_p),
                ("lidar_sources_dev", C.c_void_p), ("meas", GcsAssocMeas), ("batch_colors", C.c_void_p),
                ("batch_sources", C.c_void_p), ("view", C.c_void_p), ("view_tile_ids_dev", C.c_void_p),
                ("assoc_out", C.c_void_p), ("vpe_out", C.c_void_p), ("zero_dev", C.c_void_p),
                ("zero_bytes", C.c_int64)]


class GcsLiveOutputs(C.Structure):
    _fields_ = [("n_active", C.c_int32), ("n_stencil", C.c_int32), ("active_ids", C.c_int64 * LIVE_MAX_TILES),
                ("stencil_ids", C.c_int64 * LIVE_MAX_TILES), ("active_slots", C.c_int32 * LIVE_MAX_TILES),
                ("n_present_active", C.c_int32), ("n_created", C.c_int32),
                ("created_ids", C.c_int64 * LIVE_MAX_TILES), ("created_slots", C.c_int32 * LIVE_MAX_TILES),
                ("recency_stats", C.c_double * 3), ("trigger_sum", C.c_double), ("ess_sum", C.c_double),
                ("phase_us", C.c_double * 12),
                ("update", GcsPmapUpdateStats), ("counts", C.c_int32 * LIVE_MAX_TILES), ("next_global_id", C.c_int64)]


_SIGS = [
    ("gcs_version", C.c_char_p, []),
    ("gcs_abi_version", C.c_int, []),
    ("gcs_config_defaults", C.c_int, [C.POINTER(GcsConfig)]),
    ("gcs_ctx_create", C.c_int, [C.POINTER(GcsConfig), C.POINTER(C.c_void_p)]),
    ("gcs_ctx_destroy", C.c_int, [C.c_void_p]),
    ("gcs_last_error", C.c_char_p, [C.c_void_p]),
    ("gcs_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gcs_ctx_synchronize", C.c_int, [C.c_void_p]),
    ("gcs_ctx_enable_timing", C.c_int, [C.c_void_p, C.c_int32]),
    ("gcs_ctx_set_debug", C.c_int, [C.c_void_p, C.c_int32, C.c_int64]),
    ("gcs_ctx_mirror_stats", C.c_int, [C.c_void_p, c_int64_p]),
    ("gcs_debug_state_checksums", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    ("gcs_ctx_set_map_mode", C.c_int, [C.c_void_p, C.c_int32]),
    ("gcs_ctx_map_record", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gcs_map_follow", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("gcs_ctx_stage_times", C.c_int, [C.c_void_p, c_double_p, c_int64_p, C.c_int32]),
    ("gcs_ctx_host_split", C.c_int, [C.c_void_p, c_double_p, c_int64_p, C.c_int32]),
    ("gcs_ctx_worker_tid", C.c_int64, [C.c_void_p]),
    ("gcs_ctx_host_split_history", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32)]),
    ("gcs_ctx_set_atlas", C.c_int, [C.c_void_p, c_double_p]),
    ("gcs_ctx_get_atlas", C.c_int, [C.c_void_p, c_double_p, c_int32_p]),
    ("gcs_ctx_set_belief", C.c_int, [C.c_void_p, C.POINTER(GcsBelief)]),
    ("gcs_ctx_get_belief", C.c_int, [C.c_void_p, C.POINTER(GcsBelief)]),
    ("gcs_ctx_set_map", C.c_int, [C.c_void_p, c_double_p]),
    ("gcs_ctx_get_map", C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    ("gcs_ctx_get_scan_stats", C.c_int, [C.c_void_p, c_double_p]),
    ("gcs_ctx_get_bin_order", C.c_int, [C.c_void_p, c_int32_p]),
    ("gcs_ctx_device_arrays", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_void_p)]),
    ("gcs_ctx_set_iw_state", C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    ("gcs_ctx_get_iw_state", C.c_int, [C.c_void_p, c_double_p, c_double_p, c_double_p]),
    ("gcs_ctx_set_meas_iw_state", C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    ("gcs_ctx_get_meas_iw_state", C.c_int, [C.c_void_p, c_double_p, c_double_p, c_double_p]),
    ("gcs_scan", C.c_int, [C.c_void_p, C.POINTER(GcsScanInputs), C.POINTER(GcsScanOutputs)]),
    ("gcs_scan_begin", C.c_int, [C.c_void_p, C.POINTER(GcsScanInputs), C.POINTER(GcsScanBeginOutputs)]),
    ("gcs_scan_finish", C.c_int, [C.c_void_p, C.POINTER(GcsLidarEvidence), C.POINTER(GcsScanOutputs)]),
    ("gcs_parse_pointcloud2", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(GcsPointCloud2Layout), C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p]),
    ("gcs_point_stage", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_double,
                                  C.c_double, c_double_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, c_double_p]),
    ("gcs_bin_soft_assign", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("gcs_scan_bin_moment_match", C.c_int, [C.c_void_p, c_double_p]),
    ("gcs_matrix_fisher_rotation", C.c_int, [C.c_void_p, c_double_p]),
    ("gcs_planar_translation", C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    ("gcs_pushforward", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_double]),
    ("gcs_psd_project", C.c_int, [C.c_int32, c_double_p, C.c_double, c_double_p, c_double_p]),
    ("gcs_spd_solve_lifted", C.c_int, [C.c_int32, c_double_p, c_double_p, C.c_double, c_double_p]),
    ("gcs_spd_inverse_lifted", C.c_int, [C.c_int32, c_double_p, C.c_double, c_double_p]),
    ("gcs_svd3", C.c_int, [c_double_p, c_double_p, c_double_p, c_double_p]),
    ("gcs_psd_project3", C.c_int, [c_double_p, c_double_p, c_double_p]),
    ("gcs_debug_tile_order", C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    ("gcs_debug_preintegrate", C.c_int, [C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                         C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_int32, C.c_void_p]),
    ("gcs_mf_rotation", C.c_int, [c_double_p, c_double_p]),
    ("gcs_predict_diffusion", C.c_int, [C.POINTER(GcsBelief), c_double_p, C.c_double, C.POINTER(GcsBelief),
                                        c_double_p]),
    ("gcs_info_fusion_additive", C.c_int, [C.POINTER(GcsBelief), c_double_p, c_double_p, C.c_double,
                                           C.POINTER(GcsBelief), c_double_p]),
    ("gcs_preintegrate_imu", C.c_int, [C.c_int32, c_double_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                       c_double_p, c_double_p, c_double_p, c_double_p, c_double_p]),
    ("gcs_belief_world_pose", C.c_int, [C.POINTER(GcsBelief), c_double_p]),
    ("gcs_imu_odom_evidence", C.c_int, [C.POINTER(GcsImuOdomInputs), c_double_p, c_double_p, c_double_p]),
    ("gcs_imu_odom_evidence_device", C.c_int, [C.c_void_p, C.POINTER(GcsImuOdomInputs), c_double_p, c_double_p,
                                               c_double_p]),
    ("gcs_imu_meas_iw_suffstats", C.c_int, [C.c_int32] + [c_double_p] * 10),
    ("gcs_meas_iw_apply", C.c_int, [c_double_p] * 7),
    ("gcs_fibonacci_atlas", C.c_int, [C.c_int32, c_double_p]),
    ("gcs_knn_table", C.c_int, [C.c_int32, c_double_p, C.c_int32, c_int32_p]),
    ("gcs_nearest_bins", C.c_int, [C.c_int32, c_double_p, C.c_int32, c_double_p, c_int32_p]),
    ("gcs_hypothesis_payload", C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_void_p]),
    ("gcs_hypothesis_combine", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    ("gcs_hypothesis_barycenter", C.c_int, [C.c_int32] + [c_double_p] * 8),
    ("gcs_payload_pack", C.c_int, [C.POINTER(GcsBelief), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                   C.c_double, C.c_void_p]),
    ("gcs_payload_apply", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_double] + [C.c_void_p] * 4 +
     [C.POINTER(GcsBelief)] + [C.c_void_p] * 6),
    ("gcs_rccl_get_unique_id", C.c_int, [C.c_void_p]),
    ("gcs_rccl_comm_init", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("gcs_rccl_comm_destroy", C.c_int, [C.c_void_p]),
    ("gcs_datasheet_noise_states", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("gcs_rccl_comm_count", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("gcs_rccl_broadcast", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]),
    ("gcs_combine_allreduce", C.c_int, [C.c_void_p, C.c_void_p, C.c_double, C.c_double, C.c_int32, C.c_void_p,
                                        C.c_void_p]),
    ("gcs_scan_combine", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(GcsScanOutputs), C.c_void_p, C.c_double,
                                   C.c_double, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("gcs_process_iw_apply", C.c_int, [c_double_p] * 7),
    ("gcs_process_noise_Q", C.c_int, [c_double_p] * 3),
    ("gcs_meas_iw_mode", C.c_int, [c_double_p, c_double_p, C.c_int32, c_double_p]),
    ("gcs_ctx_describe", C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    ("gcs_surfel_config_defaults", C.c_int, [C.POINTER(GcsSurfelConfig)]),
    ("gcs_surfel_ctx_create", C.c_int, [C.POINTER(GcsSurfelConfig), C.POINTER(C.c_void_p)]),
    ("gcs_surfel_ctx_destroy", C.c_int, [C.c_void_p]),
    ("gcs_surfel_last_error", C.c_char_p, [C.c_void_p]),
    ("gcs_surfel_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gcs_extract_lidar_surfels", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                            C.POINTER(GcsSurfelOutputs)]),
    ("gcs_assoc_config_defaults", C.c_int, [C.POINTER(GcsAssocConfig)]),
    ("gcs_debug_short_log_exp", C.c_int, [c_double_p, C.c_int32, C.c_double, c_double_p, c_double_p, c_double_p]),
    ("gcs_debug_tab_log_exp", C.c_int, [c_double_p, C.c_int32, c_double_p, c_double_p]),
    ("gcs_assoc_ctx_create", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("gcs_assoc_ctx_destroy", C.c_int, [C.c_void_p]),
    ("gcs_assoc_last_error", C.c_char_p, [C.c_void_p]),
    ("gcs_assoc_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gcs_associate_primitives_ot", C.c_int, [C.c_void_p, C.POINTER(GcsAssocConfig), C.POINTER(GcsAssocMeas),
                                              C.POINTER(GcsAssocView), C.POINTER(GcsAssocOutputs)]),
    ("gcs_visual_pose_evidence", C.c_int, [C.c_void_p, C.POINTER(GcsAssocMeas), C.POINTER(GcsAssocView), C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int32, c_double_p, C.c_double, C.c_double,
                                           C.POINTER(GcsVpeOutputs)]),
    ("gcs_pmap_create", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("gcs_pmap_destroy", C.c_int, [C.c_void_p]),
    ("gcs_pmap_last_error", C.c_char_p, [C.c_void_p]),
    ("gcs_pmap_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gcs_pmap_clear_tile", C.c_int, [C.c_void_p, C.c_int32]),
    ("gcs_pmap_read", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    ("gcs_pmap_write", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    ("gcs_pmap_copy_tiles", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]),
    ("gcs_pmap_extract_view", C.c_int, [C.c_void_p, c_int32_p, c_int64_p, C.c_int32, C.c_int32, C.c_double,
                                        C.c_double, C.POINTER(GcsPmapView)]),
    ("gcs_pmap_insert_masked", C.c_int, [C.c_void_p, c_int32_p, C.c_int32, C.c_int32, C.POINTER(GcsPmapRows),
                                         C.c_double, C.c_int64, C.c_double, C.c_int64, C.c_void_p, c_int32_p,
                                         c_int32_p]),
    ("gcs_pmap_fuse", C.c_int, [C.c_void_p, c_int32_p, C.c_int32, C.POINTER(GcsPmapRows), C.c_double, C.c_int64,
                                C.c_double, c_int32_p]),
    ("gcs_pmap_cull", C.c_int, [C.c_void_p, c_int32_p, C.c_int32, C.c_double, c_int32_p, c_double_p, c_double_p,
                                c_int32_p]),
    ("gcs_pmap_forget", C.c_int, [C.c_void_p, c_int32_p, C.c_int32, C.c_double]),
    ("gcs_pmap_recency_inflate", C.c_int, [C.c_void_p, c_int32_p, C.c_int32, C.c_int64, C.c_double, C.c_double,
                                           c_double_p]),
    ("gcs_pmap_merge_reduce", C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_int32, C.c_double, C.c_double,
                                        c_int32_p, c_int32_p, c_int32_p]),
    ("gcs_pmap_map_update", C.c_int, [C.c_void_p, c_int32_p, c_int64_p, C.c_int32, c_double_p, C.c_double, C.c_int64,
                                      c_int64_p, C.POINTER(GcsPmapUpdateConfig), C.POINTER(GcsPmapUpdateInputs),
                                      C.POINTER(GcsPmapUpdateStats), c_int32_p]),
    ("gcs_live_scan", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(GcsScanBeginOutputs), C.POINTER(GcsLiveArgs),
                                C.POINTER(GcsLiveOutputs), C.POINTER(GcsScanOutputs)]),
    ("gcs_live_collect", C.c_int, [C.c_void_p, C.POINTER(GcsLiveOutputs)]),
    ("gcs_ma_hex_stencil", C.c_int, [c_double_p, C.c_double, C.c_int32, C.c_int32, c_int64_p, C.c_int32]),
]

SYMBOLS = [s[0] for s in _SIGS]

_lib = None


_AB_OPTIONAL = ("gcs_ctx_host_split", "gcs_ctx_worker_tid", "gcs_imu_odom_evidence_device",
                "gcs_ctx_host_split_history")  # (round 6 entries)


def load():
    """Load the HIP library (raises RuntimeError if it was not built: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # GCSLAM_LIB: an instrumented build of the same library (tools/phase_prof.py), never a fallback
    path = os.environ.get("GCSLAM_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with __graft_entry__.build() "
                           "(make -C gc-slam_amd); there is no CPU fallback")
    # One HIP runtime per process: torch wheels ship their own libamdhip64 (SONAME libamdhip64.so.7,
    # found through their RPATH as "libamdhip64.so").  Loaded after this library, torch would map a
    # second runtime next to /opt/rocm's and fail to initialise ("No HIP GPUs are available");
    # loaded first, this library's libamdhip64.so.7 dependency resolves to torch's copy, and the
    # streams and device pointers torch hands over belong to the same runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    # the structs above mirror include/gcslam_hip.h of this ABI: a library of another ABI would read
    # or write past them (ABI 3: gcs_assoc_outputs.cert grew to GCS_ASSOC_CERT_LEN 21; ABI 4: the one-call
    # live path's structs)
    lib.gcs_abi_version.restype = C.c_int
    abi = lib.gcs_abi_version()
    if abi != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI {abi}, this binding is ABI {ABI_VERSION}; rebuild the library "
                           "(make -C gc-slam_amd)")
    for name, res, args in _SIGS:
        # test-only and diagnostic entries may be absent from an older build loaded through GCSLAM_LIB
        # for a same-box A/B; every other entry point is required
        if (name.startswith("gcs_debug_") or name in _AB_OPTIONAL) and path != LIB_PATH and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(c_double_p)


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(c_int32_p)


def check(rc: int, ctx=None, what: str = "gcs call"):
    """Map gcs_status to the reference's exception types (fail fast, pipeline.py:546-548)."""
    if rc == 0:
        return
    # (ctx None: a failed gcs_ctx_create's message, kept per thread by the library)
    msg = load().gcs_last_error(ctx).decode(errors="replace")
    if rc in (-1, -3):
        raise ValueError(f"{what} failed ({rc}): {msg}")
    raise RuntimeError(f"{what} failed ({rc}): {msg}")


_BELIEF_FIELDS = (("X_anchor", 6), ("z_lin", D_Z), ("L", D_Z * D_Z), ("h", D_Z))


def belief_to_struct(X_anchor, stamp, z_lin, L, h) -> GcsBelief:
    b = GcsBelief()
    base = C.addressof(b)
    for (name, n), v in zip(_BELIEF_FIELDS, (X_anchor, z_lin, L, h)):
        a = np.ascontiguousarray(v, np.float64).reshape(-1)
        if a.shape[0] != n:
            raise ValueError(f"belief {name}: {a.shape[0]} values, expected {n}")
        C.memmove(base + getattr(GcsBelief, name).offset, a.ctypes.data, 8 * n)
    b.stamp_sec = float(stamp)
    return b


def struct_to_arrays(b: GcsBelief):
    """Copy a belief struct out as numpy arrays (buffer views, no per-element Python floats)."""
    view = np.ctypeslib.as_array
    return (view(b.X_anchor).copy(), float(b.stamp_sec), view(b.z_lin).copy(),
            view(b.L).reshape(D_Z, D_Z).copy(), view(b.h).copy())
