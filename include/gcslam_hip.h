/*
 * gcslam_hip.h -- C-ABI of the MI355X (gfx950) GC-SLAM bin-path per-scan backend.
 *
 * Plain pointers and sizes only.  "dev" pointers are HIP device pointers (HBM), "host"
 * pointers are ordinary host memory.  Every call returns 0 on success or a negative
 * gcs_status; gcs_last_error(ctx) holds the message.  A context owns one hypothesis on one
 * GPU (device buffers, HIP stream, belief, map-bin statistics); calls on one context must be
 * serialised by the caller, distinct contexts are independent (no global mutable state).
 *
 * Reference interfaces replaced (paths relative to the reference repo,
 * FS = fl_ws/src/fl_slam_poc/fl_slam_poc):
 *   gcs_scan                    FS/backend/pipeline.py:316-1591 process_scan_single_hypothesis
 *                               (14-step bin path, README.md:105-122)
 *   gcs_parse_pointcloud2       FS/backend/backend_node.py:377-468 parse_pointcloud2_vlp16 (+ :1677-1680)
 *   gcs_point_stage             FS/backend/operators/point_budget.py:117-221 point_budget_resample
 *                               + FS/backend/operators/deskew_constant_twist.py:72-117 (fused)
 *   gcs_bin_soft_assign         archive/legacy_operators/binning.py:79-131 bin_soft_assign
 *   gcs_scan_bin_moment_match   archive/legacy_operators/binning.py:212-324 (+ kappa.py:130-169)
 *   gcs_matrix_fisher_rotation  archive/legacy_operators/matrix_fisher_evidence.py:264-394
 *   gcs_planar_translation      archive/legacy_operators/matrix_fisher_evidence.py:502-671
 *   gcs_pushforward             PoseCovInflationPushforward (source deleted; CHANGELOG.md:1246)
 *                               + archive/bin_atlas.py:137-257 update/forgetting/derived stats
 *   gcs_psd_project             FS/common/primitives.py:80-123 domain_projection_psd_core
 *   gcs_info_fusion_additive    FS/backend/operators/fusion.py:150-230
 *   gcs_predict_diffusion       FS/backend/operators/predict.py:106-214
 *   gcs_preintegrate_imu        FS/backend/operators/imu_preintegration.py:47-147
 *   gcs_hypothesis_payload /    FS/backend/backend_node.py:1999-2119 (IW accumulation) and
 *   gcs_hypothesis_combine      FS/backend/operators/hypothesis.py:51-117 (barycenter)
 *   gcs_fibonacci_atlas         archive/bin_atlas.py:40-61
 *   gcs_associate_primitives_ot FS/backend/operators/primitive_association.py:239-553
 *                               associate_primitives_ot (+ tiling.py:148-186, measurement_batch.py:389-411)
 *   gcs_visual_pose_evidence    FS/backend/operators/visual_pose_evidence.py:260-412 visual_pose_evidence
 *   gcs_pmap_*                  FS/backend/structures/primitive_map.py:98-2031 (AtlasMap tiles in HBM;
 *                               extract_atlas_map_view, insert_masked, fuse, cull, forget,
 *                               recency_inflate, merge_reduce)
 *   gcs_extract_lidar_surfels   FS/backend/operators/lidar_surfel_extraction.py:339-431
 *                               extract_lidar_surfels (+ FS/common/ma_hex_web.py:243-303
 *                               bin_points_3d, FS/backend/structures/measurement_batch.py:272-381)
 */
#ifndef GCSLAM_HIP_H
#define GCSLAM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 4: the one-call live path (gcs_live_scan / gcs_live_collect, gcs_live_args / gcs_live_outputs) and
 * gcs_ma_hex_stencil.
 * 3: GCS_ASSOC_CERT_LEN 18 -> 21 (gcs_assoc_outputs grew), the scan mirror's sequence / checksum
 * (gcs_ctx_mirror_stats) and the state checksums (gcs_debug_state_checksums) */
#define GCS_ABI_VERSION 4
#define GCS_D_Z 22
#define GCS_SCAN_FIELDS 26   /* ScanBinStats, field-major: N, s_dir[3], S_dir_scatter[9], p_bar[3], Sigma_p[9], kappa */
#define GCS_MAP_FIELDS 26    /* MapBinStats: S_dir[3], S_dir_scatter[9], N_dir, N_pos, sum_p[3], sum_ppT[9] */
#define GCS_DERIVED_FIELDS 16 /* mu_dir[3], kappa, centroid[3], Sigma_c[9] */
#define GCS_PAYLOAD_LEN 840  /* hypothesis all-reduce payload (f64) */

typedef enum {
  GCS_OK = 0,
  GCS_ERR_ARG = -1,      /* maps to ValueError */
  GCS_ERR_HIP = -2,      /* maps to RuntimeError */
  GCS_ERR_NONFINITE = -3,/* maps to ValueError (reference fail-fast, pipeline.py:546-548) */
  GCS_ERR_STATE = -4
} gcs_status;

typedef enum { GCS_MODE_DENSE = 0, GCS_MODE_SCALE = 1 } gcs_mode;

typedef struct gcs_ctx gcs_ctx;

typedef struct {
  int32_t device;              /* HIP device ordinal */
  int32_t n_bins;              /* B */
  int32_t n_points_cap;        /* N_POINTS_CAP (constants.py:64; raised for C2/C3) */
  int32_t max_raw_points;      /* capacity of the raw input */
  int32_t mode;                /* gcs_mode */
  int32_t k_cand;              /* K candidates per point in scale mode (16) */
  double tau;                  /* soft-assign temperature (declared) */
  double lidar_origin[3];      /* LiDAR origin in base (pipeline.py:589-593) */
  int32_t deskew_rotation_only;/* pipeline.py:482-483 */
  double forgetting_factor;    /* PipelineConfig.forgetting_factor (0.99) */
  double gravity_W[3];         /* constants.py:80 */
  /* step 9 IMU / odometry evidence family (pipeline.py:595-776) and fusion scale (fusion.py:46-142);
   * PipelineConfig fields (pipeline.py:96-223).  Fill with gcs_config_defaults() first. */
  int32_t use_imu_odom;        /* 1: the reference's branch (default); 0: LiDAR-only ablation */
  double imu_gravity_scale;    /* PipelineConfig.imu_gravity_scale (1.0) */
  double planar_z_ref, planar_z_sigma, planar_vz_sigma;  /* constants.py:294-310 (0, 0.1, 0.01) */
  double alpha_min, alpha_max; /* constants.py:89-90 (1, 1) */
  double c0_cond;              /* constants.py:92 (1e6) */
} gcs_config;

typedef struct {
  /* LiDAR scan resident on the device (PointCloud2-like: float x,y,z at offsets 0,4,8) */
  const void* xyz_dev;
  int32_t point_step;
  const double* timestamps_dev;
  const double* weights_dev;
  int32_t n_points;
  /* IMU window (host, padded to imu_len with zero stamps) */
  const double* imu_stamps;    /* [imu_len] */
  const double* imu_gyro;      /* [imu_len*3] */
  const double* imu_accel;     /* [imu_len*3] */
  int32_t imu_len;
  double scan_start_time, scan_end_time, dt_sec;
  const double* Q;             /* [22*22] host; NULL = context's IW-derived Q */
  const double* L_ext;         /* optional external evidence [22*22] (IMU/odom family), may be NULL */
  const double* h_ext;         /* [22] */
  /* scan-to-scan IMU window of the measurement-noise IW statistics (pipeline.py:331-332,448-453) */
  double t_last_scan, t_scan;
  /* 0: float32 x,y,z at bytes 0,4,8 of each point_step record; 1: float64 x,y,z (gcs_parse_pointcloud2) */
  int32_t xyz_format;
  /* odometry (host; NULL = the node's "no odometry yet" inputs: identity pose, 1e12 I covariances,
   * backend_node.py:939-940,2047-2051).  Pose [t, rotvec] relative to the first odometry pose,
   * covariances row-major 6x6 in ROS [x,y,z,roll,pitch,yaw] order, twist [vx,vy,vz,wx,wy,wz] body. */
  const double* odom_pose;     /* [6] */
  const double* odom_cov_se3;  /* [36] */
  const double* odom_twist;    /* [6] */
  const double* odom_twist_cov;/* [36] */
  /* IMU noise proxies (3x3); NULL = IW mode of the context's measurement-noise state
   * (backend_node.py:2020-2023, measurement_noise_iw_jax.py:38-56) */
  const double* Sigma_g;
  const double* Sigma_a;
} gcs_scan_inputs;

/* Layout of a PointCloud2 message (sensor_msgs/PointField offsets and datatype codes) for
 * gcs_parse_pointcloud2; the VLP-16 layout has FLOAT32 x, y, z and a ring field. */
typedef struct {
  int32_t n_points;             /* width * height */
  int32_t point_step;
  int32_t off_x, off_y, off_z;  /* FLOAT32 */
  int32_t off_ring, ring_datatype;
  int32_t off_t, t_datatype;    /* per-point "t" (else "time") field; off_t < 0: none (header stamp) */
  double header_stamp_sec;
  double R_base_lidar[9];       /* row-major; points are returned in the base frame */
  double t_base_lidar[3];
} gcs_pointcloud2_layout;

typedef struct {
  double X_anchor[6];
  double stamp_sec;
  double z_lin[GCS_D_Z];
  double L[GCS_D_Z * GCS_D_Z];
  double h[GCS_D_Z];
} gcs_belief;

/* Certificate / diagnostic scalars of one scan (indices documented in DESIGN.md). */
#define GCS_CERT_LEN 64
typedef struct {
  gcs_belief belief;                 /* belief after AnchorDriftUpdate */
  double iw_process_dPsi[7 * 36];
  double iw_process_dnu[7];
  double z_t[6];                     /* post-recompose world pose used by the map update */
  double L_evidence[GCS_D_Z * GCS_D_Z];
  double h_evidence[GCS_D_Z];
  double R_mf[9];
  double t_wls[3];
  double cert[GCS_CERT_LEN];
  double stage_ms[8];                /* host-measured stage times */
  double iw_meas_dPsi[3 * 9];        /* measurement-noise IW statistics [gyro, accel, lidar] 3x3 blocks */
  double iw_meas_dnu[3];
  double L_imu_odom[GCS_D_Z * GCS_D_Z]; /* summed IMU/odometry evidence (pipeline.py:745-750), untempered */
  double h_imu_odom[GCS_D_Z];
  /* the eleven IMU/odometry certificates in all_certs order [odom, imu, imu_dep, gyro, preint, planar,
   * vz, odom_vel, odom_wz, kinematic, odom_dep], 7 fields each: [ess_total, support_frac, nll_per_ess,
   * lift_strength, psd_projection_delta, mass_epsilon_ratio, trust_alpha] */
  double imu_odom_certs[11 * 7];
} gcs_scan_outputs;

/* Inputs of the IMU/odometry evidence branch on its own (gcs_imu_odom_evidence): every quantity
 * the reference's _compute_imu_odom_branch reads (pipeline.py:595-776). */
typedef struct {
  int32_t m;                               /* IMU window length (>= 2) */
  const double *stamps, *gyro, *accel;     /* [m], [m*3], [m*3]; stamps <= 0 are padding */
  const double* w_int;                     /* scan-to-scan window weights [m] */
  double t_last_scan, t_scan, dt_sec;
  const double* pose0;                     /* belief_prev.mean_world_pose [6] */
  const double* pose_pred;                 /* belief_pred.mean_world_pose [6] */
  const double* mu_prev;                   /* belief_prev.mean_increment [22] */
  const double* mu_inc;                    /* belief_pred.mean_increment [22] */
  const double* gravity_W;                 /* [3], gravity scale applied */
  const double *Sigma_g, *Sigma_a;         /* [9] each */
  const double *odom_pose, *odom_cov_se3, *odom_twist, *odom_twist_cov;
  double planar_z_ref, planar_z_sigma, planar_vz_sigma;
} gcs_imu_odom_inputs;

/* ---------------------------------------------------------------- context */
const char* gcs_version(void);
int gcs_abi_version(void);
/* the reference's PipelineConfig / constants.py defaults (dense mode, B=48, cap 8192, K=16) */
int gcs_config_defaults(gcs_config* cfg);
int gcs_ctx_create(const gcs_config* cfg, gcs_ctx** out);
int gcs_ctx_destroy(gcs_ctx* ctx);
/* ctx NULL: the message of this thread's last failed gcs_ctx_create (e.g. an atlas the tiled bin
 * kernel cannot hold) */
const char* gcs_last_error(const gcs_ctx* ctx);
int gcs_ctx_set_stream(gcs_ctx* ctx, void* hip_stream);
int gcs_ctx_synchronize(gcs_ctx* ctx);
/* device stage timing: hipEvents stamped by the stages' own kernel dispatches on the context
 * stream.  stage_mask bit s enables stage s (0 = off): [0 point kernel (+ its fold when not
 * deferred), 1 sort+bucket, 2 bin moment-match kernel (+ fused Matrix-Fisher in scale mode),
 * 3 MF (dense / per-op), 4 planar, 5 pushforward, 6 budget kernel (row 1 mass sums),
 * 7 the bin kernel's partial-row fold (+ R_mf)].  Stages 6 + 0 + 2 + 7 are the
 * BinSoftAssign + ScanBinMomentMatch chain (bench.py roofline_chain).  Each timed stage costs a
 * few us of queue time. */
#define GCS_N_STAGES 8
int gcs_ctx_enable_timing(gcs_ctx* ctx, int32_t stage_mask);
/* Debug knobs (tests): GCS_DEBUG_SCAN_SPIN_LIMIT bounds k_scan's decoupled look-back spin (default
 * 1 << 22; when it runs out the scan returns GCS_ERR_HIP), GCS_DEBUG_INJECT_SCAN_FAIL != 0 makes
 * one look-back tile take that failure path on every scan. */
#define GCS_DEBUG_SCAN_SPIN_LIMIT 1
#define GCS_DEBUG_INJECT_SCAN_FAIL 2
/* GCS_DEBUG_SORTED_BUCKETS != 0: gcs_scan buckets points by the sorted path (k_scan, k_place,
 * k_bucket_rank) instead of the direct buckets; GCS_DEBUG_BUCKET_CAPACITY (4..32, multiple of 4)
 * lowers the direct buckets' row capacity so a test can force the overflow redo (cert[57] = 1). */
#define GCS_DEBUG_SORTED_BUCKETS 3
#define GCS_DEBUG_BUCKET_CAPACITY 4
/* GCS_DEBUG_LAUNCH_GATE: 1 (off by default; GCSLAM_GATE=1) gcs_scan queues its device front before the host prologue and a
 * one-wave gate kernel ahead of k_points waits on the device for the deskew twist; 0 (default) launches
 * the point stage after the prologue;
 * -1 (fault test) never opens the gate, so the gate kernel runs into its timeout and the scan returns
 * GCS_ERR_HIP. */
#define GCS_DEBUG_LAUNCH_GATE 5
/* GCS_DEBUG_POINT_KERNEL != 0: scale-mode scans run the round-3 point kernel (one wave per SIMD)
 * instead of k_points_lean (same arithmetic, bitwise the same outputs; A/B and its parity test). */
#define GCS_DEBUG_POINT_KERNEL 6
/* GCS_DEBUG_DEVICE_PREINT != 0 (or GCSLAM_DEVICE_PREINT=1): gcs_scan / gcs_scan_begin compute the
 * IMU window weights and the preintegration (deskew twist) on the device (k_preint) instead of the
 * host prologue; ignored with the launch gate.  A/B knob and its parity test. */
#define GCS_DEBUG_DEVICE_PREINT 7
/* GCS_DEBUG_PT_CLEAR (default 1; GCSLAM_PT_CLEAR=0 turns it off): gcs_scan's k_pt zeroes the next
 * scan's bucket counts and active-flag buffer, so that scan's k_budget only sums the weights; 0 keeps
 * the clears in k_budget (A/B knob and its bitwise test). */
#define GCS_DEBUG_PT_CLEAR 8
/* GCS_DEBUG_MIRROR_TORN (microseconds, 0 = off): the PT fold stores the scan mirror's sequence word
 * and checksum first and its data that long after, so the host meets a mirror whose data words have
 * not arrived; gcs_scan must re-read until the checksum matches (gcs_ctx_mirror_stats counts it) and
 * return the same results.  Test knob of the mirror guard. */
#define GCS_DEBUG_MIRROR_TORN 9
/* GCS_DEBUG_SENDBUF: where gcs_combine_allreduce's ncclAllReduce reads its send buffer.  -1 (default):
 * device memory when the communicator spans more than one rank (the packed payload is copied from the
 * pinned host buffer by the copy engine on the combine stream, so RCCL's ring kernels never read host
 * memory across PCIe inside the collective), the pinned host buffer itself at world size 1; 0: always
 * the host buffer; 1: always device memory (the world-1 test of the world > 1 path). */
#define GCS_DEBUG_SENDBUF 10
/* GCS_DEBUG_DEVICE_IMU_ODOM != 0 (or GCSLAM_DEVICE_IMU_ODOM=1): the step-9 IMU / odometry branch of gcs_scan /
 * gcs_scan_begin runs on the device (gcs_imu_odom_evidence_device's kernel) beside the bin path's kernels,
 * instead of the host C++ branch (the default). */
#define GCS_DEBUG_DEVICE_IMU_ODOM 11
/* GCS_DEBUG_COMBINE_DELAY (microseconds, 0 = off, at most 1,000,000): gcs_combine_allreduce queues a
 * kernel that waits this long on the combine stream ahead of ncclAllReduce -- the world-1 form of a
 * straggling peer rank.  A delay past the host poll's 20 ms sends the wait to its stream-synchronize
 * path (gcs_ctx_mirror_stats' payload syncs count it); the combined state must not change.  Test knob. */
#define GCS_DEBUG_COMBINE_DELAY 12
int gcs_ctx_set_debug(gcs_ctx* ctx, int32_t key, int64_t value);
/* The scan mirror (the PT fold's copy of the scan's scalars and device error words to pinned host
 * memory, with the scan's sequence number and a checksum; the host accepts it only when both match):
 * out[0] mirrors accepted, out[1] of them after at least one re-read (a data word arrived after the
 * sequence word), out[2] accepted only after the 20 ms poll gave up and the stream synchronized;
 * out[3..5] the same for the hypothesis all-reduce's stamped sum (gcs_combine_allreduce with a
 * communicator): all-reduces run, re-read, via stream sync. */
int gcs_ctx_mirror_stats(gcs_ctx* ctx, int64_t* out /*6*/);
/* Determinism diagnostics (tools/determinism_check.py, tests): 64-bit FNV-1a checksums of the
 * context's device state after its streams drain: [0] ScanBinStats, [1] MapBinStats, [2] derived map
 * stats, [3] touched bytes, [4] both active-flag buffers, [5] the bin kernel's partial rows, [6] the
 * device scalar block, [7] the host mirror's scalar block (device order; byte images). */
int gcs_debug_state_checksums(gcs_ctx* ctx, uint64_t* out /*8*/);
int gcs_ctx_stage_times(gcs_ctx* ctx, double* ms_sum /*GCS_N_STAGES*/, int64_t* counts /*GCS_N_STAGES*/,
                        int32_t reset);
/* The host split of every gcs_scan since the last reset, summed (ms): [0..7] the scan's stage_ms
 * (gcs_scan_outputs: pre-device, device submit + wait, tail, whole scan, budget launch + predict,
 * device launch calls, tail numerics, pushforward launch calls), [8] gcs_scan_combine's combine, [9]
 * gcs_scan_combine's whole call; *n the scans counted (n_combine[0]: the combines).  Accumulated in the
 * library on every scan, so a caller's timed region decomposes exactly, with no per-scan reads. */
int gcs_ctx_host_split(gcs_ctx* ctx, double* ms_sum /*10*/, int64_t* n /*2*/, int32_t reset);
/* The same split per scan, for its distribution (p50 / p90 / max, slow scans): the latest
 * min(n_max, scans since the reset, 4096) scans, oldest first, 6 floats each -- [pre-device, device
 * submit + wait, tail, whole gcs_scan, combine, whole gcs_scan_combine call] in ms (the last two 0 for
 * a scan not run by gcs_scan_combine); *n_out the scans written. */
int gcs_ctx_host_split_history(gcs_ctx* ctx, float* out /*n_max*6*/, int32_t n_max, int32_t* n_out);
/* The OS thread id of the context's launch worker (0 before its first job): a caller that pins its
 * own thread can keep the worker off that core (bench.py). */
int64_t gcs_ctx_worker_tid(gcs_ctx* ctx);
int gcs_ctx_set_atlas(gcs_ctx* ctx, const double* dirs_host /*B*3*/);
int gcs_ctx_get_atlas(gcs_ctx* ctx, double* dirs_host /*B*3*/, int32_t* knn_host /*B*K*/);
int gcs_ctx_set_belief(gcs_ctx* ctx, const gcs_belief* b);
int gcs_ctx_get_belief(gcs_ctx* ctx, gcs_belief* b);
int gcs_ctx_set_map(gcs_ctx* ctx, const double* map_host /*26*B field-major*/);
int gcs_ctx_get_map(gcs_ctx* ctx, double* map_host /*26*B*/, double* derived_host /*16*B*/);
int gcs_ctx_get_scan_stats(gcs_ctx* ctx, double* scan_host /*26*B*/);
/* device pointers of the resident per-bin arrays (field-major, length-B rows) in DEVICE bin
 * order; set/get_map and get_scan_stats convert to reference (atlas) order.  scan_dev is
 * read-only for the caller: in scale mode the rows of bin tiles empty in consecutive scans are
 * left in place rather than rewritten. */
int gcs_ctx_device_arrays(gcs_ctx* ctx, double** scan_dev, double** map_dev, double** derived_dev);
/* order[device bin] = reference bin id (scale mode: Hilbert patches of the sphere; dense: identity) */
int gcs_ctx_get_bin_order(gcs_ctx* ctx, int32_t* order /*B*/);
int gcs_ctx_set_iw_state(gcs_ctx* ctx, const double* nu7, const double* Psi7x36);
int gcs_ctx_get_iw_state(gcs_ctx* ctx, double* nu7, double* Psi7x36, double* Q22x22);
/* measurement-noise IW state [gyro, accel, lidar] (structures/measurement_noise_iw_jax.py:29-68);
 * cert2 = [psd_delta, nu_delta] of the last apply in gcs_hypothesis_combine (may be NULL) */
int gcs_ctx_set_meas_iw_state(gcs_ctx* ctx, const double* nu3, const double* Psi3x9);
int gcs_ctx_get_meas_iw_state(gcs_ctx* ctx, double* nu3, double* Psi3x9, double* cert2);

/* ---------------------------------------------------------------- the per-scan pipeline */
int gcs_scan(gcs_ctx* ctx, const gcs_scan_inputs* in, gcs_scan_outputs* out);

/* ---------------------------------------------------------------- live primitive path
 * The same scan split around the live path's LiDAR evidence (FS/backend/pipeline.py:778-1011), which
 * the caller builds with the primitive-path entry points between the two calls:
 *   gcs_scan_begin: budget (device), PredictDiffusion, IMU window + preintegration, deskew (device:
 *     deskewed points / weights / budget timestamps into context-owned device arrays), the
 *     measurement-noise IW statistics and the IMU/odometry branch with its z_lin_pose (:751-755);
 *   the caller: extract_lidar_surfels on those arrays, recency inflation + map view at pose_pred,
 *     associate_primitives_ot, visual_pose_evidence at z_lin_pose -> L_lidar, h_lidar (:778-1011);
 *   gcs_scan_finish: evidence sum + power tempering with the LiDAR certificates' terms, excitation
 *     scaling, FusionScaleFromCertificates, InfoFusionAdditive, recompose, process IW statistics,
 *     AnchorDriftUpdate (:1038-1230, 1494-1502); no bin-map pushforward: the caller runs step 12b
 *     (the primitive map update) at out->z_t (:1232-1492).
 * Any context mode works (its bin atlas is not used). */
typedef struct {
  double z_lin_pose[6];          /* [t, rotvec] read by visual_pose_evidence (pipeline.py:755, :318-322) */
  double pose_pred[6];           /* belief_pred.mean_world_pose: the map branch's stencil centre (:801-802) */
  int32_t n_points;              /* rows of the arrays below (N_POINTS_CAP: selected rows + zero padding) */
  int32_t n_selected;
  /* in: caller-owned device buffers of N_POINTS_CAP rows, or NULL for the context's own (valid until
   * its next scan); out: the buffers written */
  double* points_dev;            /* [n_points*3] deskewed points */
  double* timestamps_dev;        /* [n_points] budget timestamps */
  double* weights_dev;           /* [n_points] deskewed weights */
  double deskew_ess;             /* the deskew certificate: ess_total (IMU preintegration ESS), */
  double deskew_support;         /* support_frac (retained weight fraction) */
  double cert[GCS_CERT_LEN];     /* the scan's certificate slots filled so far */
} gcs_scan_begin_outputs;

typedef struct {
  const double* L_lidar;         /* [22*22] visual_pose_evidence L_pose (build_visual_pose_evidence_22d) */
  const double* h_lidar;         /* [22] */
  double trigger_sum;            /* sum of total_trigger_magnitude over the map-branch certs (surfel,
                                    recency inflation, association) and the visual cert (pipeline.py:1211) */
  double ess_sum;                /* sum of support.ess_total over the LiDAR certs after deskew (surfel,
                                    association, visual; aggregate_certificates, pipeline.py:1049-1056) */
  int32_t n_certs;               /* their count */
  double nll_sum;                /* sum of mismatch.nll_per_ess over the same certs */
} gcs_lidar_evidence;

int gcs_scan_begin(gcs_ctx* ctx, const gcs_scan_inputs* in, gcs_scan_begin_outputs* out);
int gcs_scan_finish(gcs_ctx* ctx, const gcs_lidar_evidence* ev, gcs_scan_outputs* out);

/* ---------------------------------------------------------------- per-operator device entry points */
/* parse_pointcloud2_vlp16 (FS/backend/backend_node.py:377-468) + the no-TF base transform
 * (:1677-1680) on the device, over the raw message bytes: points_dev [n*3] f64 base frame (feed
 * gcs_scan with xyz_format = 1, point_step = 24), t_dev (s; ns converted when any value exceeds
 * 1e6), w_dev (range-sigmoid weights), ring_dev (u8, may be NULL).  Async on the context stream. */
int gcs_parse_pointcloud2(gcs_ctx* ctx, const void* data_dev, const gcs_pointcloud2_layout* layout,
                          double* points_dev, double* t_dev, double* w_dev, uint8_t* ring_dev);
/* PointBudgetResample + DeskewConstantTwist + directions + BinSoftAssign normalisers, fused.
 * Outputs (device, length n_points_cap; NULL to skip): deskewed points [cap*3], deskewed
 * weights, budget weights, nearest bin (scale mode).  cert_host receives scalars
 * [mass_in, mass_sel, mass_scale, sum_w_budget, sum_wn2, sum_w_deskew, sum_entropy, max_resp]. */
int gcs_point_stage(gcs_ctx* ctx, const void* xyz_dev, int32_t point_step, const double* t_dev, const double* w_dev,
                    int32_t n_points, double t0, double t1, const double* xi_body6,
                    double* p0_dev, double* w_out_dev, double* w_budget_dev, int32_t* nearest_dev, double* cert_host);
/* BinSoftAssign materialised for parity (scale: [cap*K] ids + responsibilities; dense: [cap*B]).
 * Requires a preceding gcs_point_stage on the same context. */
int gcs_bin_soft_assign(gcs_ctx* ctx, int32_t* ids_dev, double* resp_dev);
/* ScanBinMomentMatch (+Kappa) over the last point stage; writes the context's ScanBinStats
 * (gcs_ctx_device_arrays) and cert_host = [sum N, sum N^2, sum N/(N+eps), psd_delta, max eps ratio]. */
int gcs_scan_bin_moment_match(gcs_ctx* ctx, double* cert_host);
/* MatrixFisherRotation + PlanarTranslation over the context's scan and map stats.
 * mf_host  = [H(9), N_eff, map_scatter_total(9), map_N_dir_total, scan_N_total, R_mf(9), s(3), V(9)]
 * pt_host  = [L_full(9), h_full(3), N_eff] */
int gcs_matrix_fisher_rotation(gcs_ctx* ctx, double* mf_host);
int gcs_planar_translation(gcs_ctx* ctx, const double* R_hat9, double* pt_host);
/* PoseCovInflationPushforward of the context's scan stats into its map at pose z_t. */
int gcs_pushforward(gcs_ctx* ctx, const double* z_t6, const double* Sigma_pose36, double gamma);

/* ---------------------------------------------------------------- host-side numerics (no GPU) */
/* matrix orders n <= 24 (the 22-D state and its blocks); larger n returns GCS_ERR_ARG */
int gcs_psd_project(int32_t n, const double* M, double eps_psd, double* M_psd, double* cert6);
int gcs_spd_solve_lifted(int32_t n, const double* L, const double* b, double eps_lift, double* x);
int gcs_spd_inverse_lifted(int32_t n, const double* L, double eps_lift, double* Linv);
int gcs_svd3(const double* H, double* U, double* s, double* V);
/* The kernels' 3x3 DomainProjectionPSD (primitives.py:80-123; gcs_math.h psd_project3: exact-zero
 * and Cholesky fast paths, clamped-eigenpair deflation, Jacobi fallback), host build of the same
 * code; delta = ||M_psd - M_sym||_F. */
int gcs_psd_project3(const double* M /*3x3*/, double* M_psd /*3x3*/, double* delta);
/* Test entry: the bin kernel's tile dispatch order for per-tile active flags and staged-record counts
 * (n tiles; xcd != 0: grouped per XCD, n % 8 == 0), computed on `device` into order[n]. */
int gcs_debug_tile_order(int32_t device, const uint8_t* active, const uint32_t* work, int32_t n, int32_t xcd,
                         int32_t* order);
/* Test entry: k_preint on `device` over one IMU window (m samples; stamps[m], gyro/accel[m*3]):
 * smooth_window_weights(stamps, t0, t1, sigma) then preintegrate_imu_relative_pose_jax
 * (imu_preintegration.py:20-147) and the deskew twist se3_log(delta_pose) (pipeline.py:466-483;
 * rotation_only zeroes its translation).  out[16] = xi[6], ess, delta_pose[6], delta_v[3]. */
int gcs_debug_preintegrate(int32_t device, int32_t m, const double* stamps, const double* gyro, const double* accel,
                           double t0, double t1, double sigma, const double* rotvec /*3*/, const double* gyro_bias /*3*/,
                           const double* accel_bias /*3*/, const double* gravity /*3*/, int32_t rotation_only,
                           double* out /*16*/);
/* det-fixed Matrix-Fisher rotation R = U diag(1,1,det(UV^T)) V^T of H (matrix_fisher_evidence.py:215-222):
 * the same routine the device fold runs (polar Newton, SVD for reflections / rank deficiency) */
int gcs_mf_rotation(const double* H /*3x3*/, double* R /*3x3*/);
int gcs_predict_diffusion(const gcs_belief* prev, const double* Q, double dt_sec, gcs_belief* pred, double* cert4);
int gcs_info_fusion_additive(const gcs_belief* pred, const double* L_ev, const double* h_ev, double alpha,
                             gcs_belief* post, double* psd_delta);
int gcs_preintegrate_imu(int32_t m, const double* stamps, const double* gyro, const double* accel, const double* weights,
                         const double* rotvec_start, const double* gyro_bias, const double* accel_bias,
                         const double* gravity_W, double* delta_pose6, double* ess);
int gcs_belief_world_pose(const gcs_belief* b, double* pose6); /* belief.py:410-434 */
/* gyro + accel measurement-noise IW statistics of one IMU window (pipeline.py:522-566;
 * measurement_noise_iw_jax.py:130-218); w_int = scan-to-scan window weights, stamps <= 0 are padding */
/* _compute_imu_odom_branch (pipeline.py:595-776): L [22*22], h [22] (dependence scales applied);
 * cert = [trigger sum of the eleven certs, ess_imu_weighted, kappa, transport_sigma, imu scale,
 *         odom scale, mean reliability, odom nll, imu nll/ess, gyro nll, dt_int, dt_imu, omega_avg(3)] */
#define GCS_IMU_ODOM_CERT_LEN 15
int gcs_imu_odom_evidence(const gcs_imu_odom_inputs* in, double* L, double* h, double* cert);
/* The same branch on the device (gcs_imu_odom.hip k_imu_odom: one workgroup; window statistics, the
 * scan-to-scan preintegration and the IMU factor's medians and weighted sums in parallel, the eleven
 * factors' assembly -- the host branch's own code -- on lane 0) on ctx's stream for it, same outputs.
 * m <= 1024.  gcs_scan / gcs_scan_begin take it under GCS_DEBUG_DEVICE_IMU_ODOM / GCSLAM_DEVICE_IMU_ODOM=1. */
int gcs_imu_odom_evidence_device(gcs_ctx* ctx, const gcs_imu_odom_inputs* in, double* L, double* h, double* cert);
int gcs_imu_meas_iw_suffstats(int32_t m, const double* stamps, const double* gyro, const double* accel,
                              const double* w_int, const double* gyro_bias, const double* accel_bias,
                              const double* rotvec0, const double* gravity_W, double* dPsi3x9, double* dnu3);
/* measurement_noise_apply_suffstats_jax (measurement_noise_iw_jax.py:59-100) */
int gcs_meas_iw_apply(const double* nu3, const double* Psi3x9, const double* dPsi3x9, const double* dnu3,
                      double* nu_out, double* Psi_out, double* cert2);
int gcs_fibonacci_atlas(int32_t n_bins, double* dirs /*B*3*/);
int gcs_knn_table(int32_t n_bins, const double* dirs, int32_t k, int32_t* knn /*B*k*/);
int gcs_nearest_bins(int32_t n_bins, const double* dirs, int32_t n_query, const double* q /*n*3*/, int32_t* out);

/* ---------------------------------------------------------------- hypotheses (multi-GPU combine) */
/* Pack this hypothesis' contribution (weights pre-applied) for an RCCL sum all-reduce:
 * [w_iw dPsi 252 | w_iw dnu 7 | w_iw dPsi_meas 27 | w_iw dnu_meas 3 | w L 484 | w h 22 | w z 22 | w mu 22 | w |mu|^2 1] */
int gcs_hypothesis_payload(gcs_ctx* ctx, double w_iw, double w_bary, double* payload_host);
/* hypothesis_barycenter_projection (hypothesis.py:51-236) on host arrays, no context and no side
 * effects: weights floored at 0.0025 and renormalised, L = PSD(sum w L_k), h, z_lin = sum w (h, z).
 * cert6 = [psd_delta, floor_adjustment, ess = 1/sum w^2, support_frac, spread_proxy, cond] */
int gcs_hypothesis_barycenter(int32_t n_hyp, const double* L_stack /*n*484*/, const double* h_stack /*n*22*/,
                              const double* z_stack /*n*22*/, const double* weights /*n*/, double* L_out, double* h_out,
                              double* z_out, double* cert6);
/* process_noise_iw_apply_suffstats_jax (inverse_wishart_jax.py:126-185): state (nu7, Psi 7x36) <- apply
 * (dPsi, dnu); cert2 = [psd_delta, nu_delta].  process_noise_state_to_Q_jax (:35-68). */
int gcs_process_iw_apply(const double* nu7, const double* Psi7x36, const double* dPsi7x36, const double* dnu7,
                         double* nu_out, double* Psi_out, double* cert2);
int gcs_process_noise_Q(const double* nu7, const double* Psi7x36, double* Q22x22);
/* measurement_noise_mean_jax (IW mode, measurement_noise_iw_jax.py:38-56) of block idx (0 gyro, 1 accel, 2 lidar) */
int gcs_meas_iw_mode(const double* nu3, const double* Psi3x9, int32_t idx, double* Sigma3x3);
/* Runtime description of a context (RuntimeManifest, pipeline.py:1629-1793, for the bin path): JSON
 * with the library version, device, declared parameters (tau rule, K, cap, map mode, pushforward
 * form) and kernel set.  Writes at most len bytes (NUL-terminated); returns GCS_ERR_ARG if too short. */
int gcs_ctx_describe(gcs_ctx* ctx, char* buf, int32_t len);
/* Apply the summed payload: barycenter (PSD of L), process IW apply + Q rebuild and
 * measurement-noise IW apply (backend_node.py:2102-2119; both stored in ctx).
 * combined_out may be NULL; cert_out = [psd_delta, spread, iw_psd_delta, iw_nu_delta]. */
int gcs_hypothesis_combine(gcs_ctx* ctx, const double* payload_sum, int32_t scan_count, gcs_belief* combined_out,
                           double* cert_out);

/* The node's initial noise states (create_datasheet_process_noise_state,
 * structures/inverse_wishart_jax.py:42-80; create_datasheet_measurement_noise_state,
 * structures/measurement_noise_iw_jax.py:37-68): process nu[7], Psi[7*36]; measurement nu[3], Psi[3*9]. */
int gcs_datasheet_noise_states(double* nu7, double* Psi252, double* mnu3, double* mPsi27);

/* Context-free forms of the same payload (host numerics, no GPU): pack one hypothesis' contribution
 * (any stats pointer may be NULL = zeros) and apply a summed payload to explicit IW states. */
int gcs_payload_pack(const gcs_belief* b, const double* dPsi252, const double* dnu7, const double* meas_dPsi27,
                     const double* meas_dnu3, double w_iw, double w_bary, double* payload /*840*/);
int gcs_payload_apply(const double* payload_sum, int32_t scan_count, const double* X_anchor6, double stamp_sec,
                      const double* nu7, const double* Psi7x36, const double* meas_nu3, const double* meas_Psi3x9,
                      gcs_belief* combined_out /*may be NULL*/, double* nu_out, double* Psi_out, double* Q_out,
                      double* meas_nu_out, double* meas_Psi_out, double* cert4);

/* ---------------------------------------------------------------- RCCL (one rank per GPU) */
/* The per-scan hypothesis exchange (backend_node.py:1999-2119, hypothesis.py:92-115):
 * gcs_combine_allreduce packs this context's payload, sum-all-reduces it over the RCCL communicator
 * on the context stream (xGMI between MI355X GPUs), and applies the combine + IW updates, so every
 * rank holds bitwise-identical Q and IW states.  comm NULL = a single rank (no exchange).  The
 * communicator comes from gcs_rccl_comm_init with an id from gcs_rccl_get_unique_id on one rank,
 * broadcast by the launcher. */
#define GCS_RCCL_ID_BYTES 128
int gcs_rccl_get_unique_id(uint8_t* id /*GCS_RCCL_ID_BYTES*/);
int gcs_rccl_comm_init(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t* id, void** comm);
int gcs_rccl_comm_destroy(void* comm);
/* Ranks the communicator holds (ncclCommCount) and this rank's index in it (ncclCommUserRank):
 * bench.py reports them so a multi-GPU line shows RCCL saw every rank. */
int gcs_rccl_comm_count(void* comm, int32_t* count, int32_t* user_rank);
/* In-place ncclBroadcast of `bytes` bytes of device memory from rank `root` on `stream` (NULL: the
 * device's null stream), then a stream synchronize: the live primitive map's per-scan update record
 * (gcslam.distributed.MapRecordChannel, ~0.5 MB at the reference sizes) from the lead to the ranks
 * that replay it (backend_node.py:2079-2083). */
int gcs_rccl_broadcast(void* comm, void* buf, int64_t bytes, int32_t root, void* stream);
/* gcs_scan then gcs_combine_allreduce in one call (the node's per-scan step, backend_node.py:2036-2119,
 * without a caller round trip between them); combine_ms (may be NULL): the combine's host wall time. */
int gcs_scan_combine(gcs_ctx* ctx, const gcs_scan_inputs* in, gcs_scan_outputs* out, void* comm, double w_iw,
                     double w_bary, int32_t scan_count, gcs_belief* combined_out, double* cert /*4*/,
                     double* combine_ms);
int gcs_combine_allreduce(gcs_ctx* ctx, void* comm, double w_iw, double w_bary, int32_t scan_count,
                          gcs_belief* combined_out /*may be NULL*/, double* cert4 /*may be NULL*/);


/* ---------------------------------------------------------------- one map for all hypotheses */
/* The reference node keeps ONE map: every hypothesis of a scan reads self.primitive_map and only
 * hypothesis 0's update is stored (backend_node.py:2036-2083).  With one hypothesis per GPU each
 * context holds a copy of that map:
 *   GCS_MAP_OWN (default)  every context updates its own map from its own scan (per-hypothesis maps,
 *                          no map traffic; declared);
 *   GCS_MAP_LEAD           hypothesis 0: updates its map and keeps the scan's map-update record
 *                          [deskew twist 6 | z_t 6 | pose covariance 6x6] (GCS_MAP_REC_LEN f64);
 *   GCS_MAP_FOLLOW         hypotheses 1..: gcs_scan skips its own pushforward, and gcs_map_follow
 *                          replays the lead's update on the same raw scan (point + bin stage at the
 *                          lead's twist, pushforward at the lead's z_t and covariance), so the map
 *                          stays bitwise the lead's.  No map rows move between GPUs: the record rides
 *                          the per-scan payload all-reduce (GCS_PAYLOAD_LEN + GCS_MAP_REC_LEN f64,
 *                          the lead's record plus zeros) when every rank's context is LEAD or FOLLOW.
 * A follower's scan s reads the map after the lead's scan s - 1 (declared lag: the reference's
 * sequential loop lets hypothesis k > 0 read hypothesis 0's update of the same scan). */
#define GCS_MAP_OWN 0
#define GCS_MAP_LEAD 1
#define GCS_MAP_FOLLOW 2
#define GCS_MAP_REC_LEN 48
int gcs_ctx_set_map_mode(gcs_ctx* ctx, int32_t mode);
/* the last gcs_scan's map-update record (any mode) */
int gcs_ctx_map_record(gcs_ctx* ctx, double* rec /*GCS_MAP_REC_LEN*/);
/* replay the lead's update of this scan (in: the scan's gcs_scan inputs; only the point stream,
 * the scan window and n_points are read); rec NULL = the record the last gcs_combine_allreduce
 * carried from the lead (a single rank, comm NULL: its own record -- bench.py --map-mode follow times
 * a follower's scan on one GPU that way) */
int gcs_map_follow(gcs_ctx* ctx, const gcs_scan_inputs* in, const double* rec /*GCS_MAP_REC_LEN or NULL*/);

/* ---------------------------------------------------------------- primitive path: LiDAR surfels */
/* extract_lidar_surfels (lidar_surfel_extraction.py:339-431) on the GPU: sentinel mask and weighted
 * centre, MA-hex 3D hash-grid cell of every point (ma_hex_web.py:221-303), the first max_occupants
 * points of each cell in index order (stable radix sort by cell), one weighted plane fit per cell
 * (3x3 eigh, Wishart-regularised covariance, kappa; :84-163), the valid cells in cell-id order
 * into n_surfel slots (:297-321) and the LiDAR slice of the MeasurementBatch in information form
 * (measurement_batch.py:298-331).  A surfel context owns the workspace for up to max_points points
 * on one GPU; calls on one context must be serialised. */
typedef struct gcs_surfel_ctx gcs_surfel_ctx;

typedef struct {
  int32_t n_surfel;                   /* lidar_surfel_extraction.py:46 (GC_N_SURFEL = 1024) */
  int32_t n_feat;                     /* :47 (GC_N_FEAT = 512): the LiDAR slice starts there */
  double voxel_size_m;                /* :48 */
  int32_t num_cells_1, num_cells_2, num_cells_z, max_occupants;  /* :50-53 (32, 32, 8, 32) */
  int32_t min_points_per_voxel;       /* :54 */
  double sensor_noise_var_per_axis;   /* :55 */
  double wishart_nu, wishart_psi_scale;          /* :56-57 */
  double kappa_main_scale, kappa_min, kappa_max; /* :58-60 */
  double eig_min;                     /* :61 */
  double eps_lift;                    /* :62 (GC_EPS_LIFT) */
  int32_t max_points;                 /* capacity of the context (points per call) */
  int32_t device;
} gcs_surfel_config;

/* Outputs: device pointers, each may be NULL (not written).  Row counts: n_surfel unless noted.
 * Slots past n_valid hold the reference's padding (positions / normals / kappas / weights /
 * timestamps 0, covariances I; batch rows 0, cell_ids -1). */
typedef struct {
  double* positions;     /* n_surfel x 3   surfel centroids (lidar_surfel_extraction.py:307) */
  double* covariances;   /* n_surfel x 9   Wishart-regularised Sigma */
  double* normals;       /* n_surfel x 3 */
  double* kappas;        /* n_surfel */
  double* weights;       /* n_surfel       sum of member weights */
  double* timestamps;    /* n_surfel */
  double* Lambdas;       /* n_surfel x 9   MeasurementBatch LiDAR slice: inv(Sigma + eps_lift I) */
  double* thetas;        /* n_surfel x 3   Lambda mu */
  double* etas;          /* n_surfel x 3 lobes x 3: lobe 0 = kappa n, others 0 */
  double* colors;        /* n_surfel x 3   grey from normal z (measurement_batch.py:262-269) */
  uint8_t* valid_mask;   /* n_surfel */
  int32_t* source_indices; /* n_surfel */
  int32_t* cell_ids;     /* n_surfel       MA-hex cell of each slot (-1 past n_valid) */
  int32_t* bucket;       /* n_cells x max_occupants point indices (-1 padding) */
  int32_t* count;        /* n_cells        occupancy clipped to max_occupants */
  int32_t* sources;      /* n_surfel       MeasurementBatch sources of the LiDAR slice: 1 on valid rows (the
                            rows past n_valid are not written) */
  /* host results */
  double center[3];      /* the weighted centre the cells are hashed around (:264-267) */
  int32_t n_valid;       /* surfels in the LiDAR slice */
  double cert[2];        /* SupportCert: ess_total = n_valid, support_frac = n_valid / n_surfel */
} gcs_surfel_outputs;

int gcs_surfel_config_defaults(gcs_surfel_config* cfg);
int gcs_surfel_ctx_create(const gcs_surfel_config* cfg, gcs_surfel_ctx** out);
int gcs_surfel_ctx_destroy(gcs_surfel_ctx* ctx);
const char* gcs_surfel_last_error(const gcs_surfel_ctx* ctx);
/* stream: a hipStream_t (NULL = the context's own); work on it is ordered after the caller's */
int gcs_surfel_ctx_set_stream(gcs_surfel_ctx* ctx, void* stream);
/* points: n x 3 f64, timestamps / weights: n f64 (device); n <= max_points.  Synchronises. */
int gcs_extract_lidar_surfels(gcs_surfel_ctx* ctx, const double* points_dev, const double* timestamps_dev,
                              const double* weights_dev, int32_t n, gcs_surfel_outputs* out);

/* ---------------------------------------------------------------- primitive path: OT association */
/* associate_primitives_ot (primitive_association.py:239-553) on the GPU: per measurement the MA-hex
 * stencil pool (n_stencil x m_tile_view view entries) costed by ||x_i - x_j||^2 + beta H^2_vMF
 * (:152-197; 1e12 where the view entry is invalid or the stencil tile is not in the view), the
 * k_assoc cheapest by (cost, pool position) (lax.sort with num_keys=1 is stable on cost alone, :376),
 * the selected candidates' unmasked cost + recency (eps lambda dt) with the row minimum subtracted,
 * then k_sinkhorn fixed iterations of unbalanced Sinkhorn (:105-138) on one workgroup; the OTCert /
 * SupportCert / InfluenceCert scalars land in cert[] (GCS_ASSOC_CERT_* slots).  An association
 * context owns the workspace for up to max_meas rows, max_pool view entries and k_assoc <= max_k
 * (<= 32; max_meas <= 2048 / 1024 / 512 for max_k <= 8 / 16 / 32). */
/* slots CAND_*: the MapUpdateCert's candidate statistics (pipeline.py:879-905: distinct candidate tiles
 * and valid candidates per valid measurement, means over the valid rows and the counts' p95), computed
 * beside the Sinkhorn iterations */
#define GCS_ASSOC_CERT_LEN 21
enum {
  GCS_ASSOC_CERT_DEFECT_A = 0, GCS_ASSOC_CERT_DEFECT_B, GCS_ASSOC_CERT_MASS_TOTAL, GCS_ASSOC_CERT_SUM_A,
  GCS_ASSOC_CERT_SUM_B, GCS_ASSOC_CERT_SUM_M, GCS_ASSOC_CERT_SUM_NOVEL, GCS_ASSOC_CERT_P95_A, GCS_ASSOC_CERT_P95_B,
  GCS_ASSOC_CERT_NONZERO_A, GCS_ASSOC_CERT_NONZERO_B, GCS_ASSOC_CERT_B_RECENCY_P95, GCS_ASSOC_CERT_ESS,
  GCS_ASSOC_CERT_MASS_EPS_RATIO, GCS_ASSOC_CERT_TOTAL_COST, GCS_ASSOC_CERT_SUPPORT_FRAC, GCS_ASSOC_CERT_EXACT,
  GCS_ASSOC_CERT_MAP_VALID, GCS_ASSOC_CERT_CAND_TILES_MEAN, GCS_ASSOC_CERT_CAND_PRIMS_MEAN,
  GCS_ASSOC_CERT_CAND_PRIMS_P95
};
enum { GCS_ASSOC_A_UNIFORM = 0, GCS_ASSOC_A_WEIGHT = 1 };  /* MeasurementMassPolicy (:40-48) */
enum { GCS_ASSOC_B_UNIFORM = 0 };                          /* MapMassPolicy (:51-59): only UNIFORM runs */
typedef struct gcs_assoc_ctx gcs_assoc_ctx;

typedef struct {            /* AssociationConfig, primitive_association.py:206-236 */
  int32_t k_assoc, k_sinkhorn;                     /* GC_K_ASSOC = 8, GC_K_SINKHORN = 50 */
  double beta, epsilon, tau_a, tau_b;              /* 0.5, 0.1, 0.5, 0.5 */
  int32_t cost_subtract_row_min, cost_scale_by_median;  /* 1, 0 */
  int32_t a_policy, b_policy;                      /* GCS_ASSOC_A_*, GCS_ASSOC_B_* */
  double eps_mass;                                 /* AssociationConfig.eps_mass: marginals, b rows, ESS */
  double eps_lift, eps_mass_dir;                   /* operator arguments eps_lift / eps_mass: measurement
                                                      means and directions (:296-297) */
  double h_tile;                                   /* GC_H_TILE = 2.0 */
  int32_t r_stencil_tiles_xy, r_stencil_tiles_z;   /* 1, 0 */
  int64_t scan_seq;
  double recency_decay_lambda;                     /* 0.02 */
} gcs_assoc_config;

typedef struct {            /* MeasurementBatch (measurement_batch.py:68-135), device pointers */
  const double* Lambdas;    /* n_total x 9 */
  const double* thetas;     /* n_total x 3 */
  const double* etas;       /* n_total x n_lobes x 3 */
  const double* weights;    /* n_total */
  const uint8_t* valid_mask;/* n_total */
  int32_t n_total, n_lobes;
  int32_t n_valid;          /* n_camera_valid + n_lidar_valid (host count, :272) */
} gcs_assoc_meas;

typedef struct {            /* AtlasMapView (primitive_map.py:270-300), device pointers */
  const int64_t* tile_ids;  /* n_tiles, view order */
  int32_t n_tiles, m_tile_view;     /* view entries = n_tiles x m_tile_view */
  const double* positions;  /* entries x 3 */
  const double* directions; /* entries x 3 */
  const double* kappas;     /* entries */
  const uint8_t* valid_mask;/* entries */
  const int64_t* last_supported_scan_seq;  /* entries */
  const int64_t* candidate_tile_ids;       /* entries */
  const int32_t* candidate_slots;          /* entries */
} gcs_assoc_view;

typedef struct {            /* PrimitiveAssociationResult (:71-92): device pointers, n_total x k_assoc */
  double* responsibilities; /* required */
  int32_t* candidate_pool_indices;  /* may be NULL */
  int64_t* candidate_tile_ids;      /* may be NULL */
  int64_t* candidate_slots;         /* may be NULL */
  double* row_masses;       /* n_total, required */
  double* cost_matrix;      /* required */
  /* host results */
  double cert[GCS_ASSOC_CERT_LEN];
  int32_t exact;            /* 1: the empty case (no valid measurement or map entry, :272-287) */
  int32_t n_map_valid;
} gcs_assoc_outputs;

int gcs_assoc_config_defaults(gcs_assoc_config* cfg);
/* Host evaluation of the Sinkhorn's short log / exp / x^y (gcs_math.h log_short, exp_short,
 * pow_sinkhorn; the device runs the same code) for the accuracy test against numpy. */
int gcs_debug_short_log_exp(const double* x, int32_t n, double y, double* log_out, double* exp_out, double* pow_out);
/* Host evaluation of the table-driven log / exp of the Sinkhorn loop (gcs_math.h log_tab, exp_tab;
 * NaN outside their domains: positive normal x / |x| < 700), for the same accuracy test. */
int gcs_debug_tab_log_exp(const double* x, int32_t n, double* log_out, double* exp_out);
int gcs_assoc_ctx_create(int32_t max_meas, int32_t max_pool, int32_t max_k, int32_t device, gcs_assoc_ctx** out);
int gcs_assoc_ctx_destroy(gcs_assoc_ctx* ctx);
const char* gcs_assoc_last_error(const gcs_assoc_ctx* ctx);
/* stream: a hipStream_t (NULL = the context's own); work on it is ordered after the caller's */
int gcs_assoc_ctx_set_stream(gcs_assoc_ctx* ctx, void* stream);
/* Synchronises; unsupported policies return GCS_ERR_ARG with the reference's message. */
int gcs_associate_primitives_ot(gcs_assoc_ctx* ctx, const gcs_assoc_config* cfg, const gcs_assoc_meas* meas,
                                const gcs_assoc_view* view, gcs_assoc_outputs* out);

/* visual_pose_evidence (visual_pose_evidence.py:260-412): 22-D pose evidence from the association's
 * soft correspondences at z_lin_pose = [t, rotvec] -- WLS translation (L_t = sum_i (sum_k pi) Lambda_i,
 * h_t, cost; :104-148) and the vMF scatter rotation (S = sum pi sqrt(k_i k_m) mu_m mu_i^T, SVD,
 * det-fixed U V^T, so3_log of R_scatter R_pred^T, L_rot = diag(s + eps); :150-240) -- summed in a
 * fixed order over the first n_valid valid rows on the association context's stream; the 3x3 SVD
 * and so3_log on the host.  exact = 1: the empty case (L = eps I, h = 0; :293-318). */
typedef struct {
  double L_pose[GCS_D_Z * GCS_D_Z], h_pose[GCS_D_Z];
  double L_trans[9], h_trans[3], L_rot[9], h_rot[3];
  double total_weighted_cost, mean_transported_mass;
  double ess_total, support_frac;   /* SupportCert */
  int32_t n_associations, exact;
} gcs_vpe_outputs;
int gcs_visual_pose_evidence(gcs_assoc_ctx* ctx, const gcs_assoc_meas* meas, const gcs_assoc_view* view,
                             const double* responsibilities, const int32_t* candidate_pool_indices,
                             const double* row_masses, int32_t k_assoc, const double* z_lin_pose, double eps_lift,
                             double eps_mass, gcs_vpe_outputs* out);

/* ---------------------------------------------------------------- primitive path: the primitive map */
/* The AtlasMap's tile storage (FS/backend/structures/primitive_map.py:98-227) resident in HBM, and
 * its maintenance operators on the GPU:
 *   gcs_pmap_extract_view      extract_atlas_map_view (:356-450, top m_view slots by weight per tile,
 *                              _select_topk_slots_fixed :303-322; view core :474-498)
 *   gcs_pmap_insert_masked     primitive_map_insert_masked (:807-981; eviction targets by
 *                              _select_lowest_mass_slots_fixed :325-353), several tiles per call
 *   gcs_pmap_fuse              primitive_map_fuse (:992-1163), the pipeline's per-active-tile loop
 *                              (pipeline.py:1301-1327) in one call
 *   gcs_pmap_cull              primitive_map_cull (:1175-1304, weight threshold)
 *   gcs_pmap_forget            primitive_map_forget (:1314-1384)
 *   gcs_pmap_recency_inflate   primitive_map_recency_inflate (:1400-1484)
 *   gcs_pmap_merge_reduce      primitive_map_merge_reduce (:1501-2031) for tiles of <= max_merge slots
 * A map context holds max_tiles tiles of m_tile slots (tile storage index 0..max_tiles-1; the caller
 * maps MA-hex tile ids to storage indices, as the AtlasMap dict does).  Per field the storage is
 * [tile][slot][width] (the reference's array shapes).  Sorts are stable radix sorts on the
 * reference's single key (lax.sort with num_keys = 1; -0.0 == 0.0); scatter-adds accumulate in
 * input order; no floating-point atomics: bitwise reproducible.  Every call synchronises. */
typedef struct gcs_pmap gcs_pmap;
enum {  /* field codes for gcs_pmap_read / gcs_pmap_write: element type and width per slot */
  GCS_PM_LAMBDAS = 0,  /* f64 x 9 */
  GCS_PM_THETAS,       /* f64 x 3 */
  GCS_PM_ETAS,         /* f64 x n_lobes*3 */
  GCS_PM_WEIGHTS,      /* f64 */
  GCS_PM_TIMESTAMPS,   /* f64 */
  GCS_PM_CREATED,      /* f64 */
  GCS_PM_COLORS,       /* f64 x 3 */
  GCS_PM_CAM_MASS,     /* f64 */
  GCS_PM_LIDAR_MASS,   /* f64 */
  GCS_PM_RGB_ACCUM,    /* f64 x 3 */
  GCS_PM_RGB_DENOM,    /* f64 */
  GCS_PM_RGB,          /* f64 x 3 */
  GCS_PM_LAST_SUPPORTED, /* i64 */
  GCS_PM_LAST_UPDATE,  /* i64 */
  GCS_PM_IDS,          /* i64 */
  GCS_PM_VALID,        /* u8 */
  GCS_PM_NFIELDS
};

typedef struct {            /* AtlasMapView outputs (device pointers, n_tiles x m_view rows; any may be NULL) */
  double* positions;        /* x 3 */
  double* covariances;      /* x 9 */
  double* directions;       /* x 3 */
  double* kappas;
  double* weights;
  int64_t* primitive_ids;
  uint8_t* valid_mask;
  int64_t* last_supported_scan_seq;
  double* etas;             /* x n_lobes*3 */
  double* colors;           /* x 3 (the tile's rgb) */
  int32_t* candidate_slots;
  int64_t* candidate_tile_ids;
} gcs_pmap_view;

typedef struct {            /* one row per proposal / contribution (device pointers; optional ones may be NULL) */
  const double* Lambdas;    /* n x 9 (world frame) */
  const double* thetas;     /* n x 3 */
  const double* etas;       /* n x n_lobes*3 */
  const double* weights;    /* n */
  const double* responsibilities; /* n (fuse) */
  const uint8_t* valid;     /* n: fuse valid_mask / insert valid_new_mask */
  const double* colors;     /* n x 3, optional */
  const int32_t* sources;   /* n (0 camera, 1 LiDAR), optional */
  const int32_t* tile_pos;  /* fuse: n, index into the call's tile list (-1: no tile) */
  const int32_t* slots;     /* fuse: n, target slot */
  int32_t n;
} gcs_pmap_rows;

int gcs_pmap_create(int32_t m_tile, int32_t max_tiles, int32_t n_lobes, int32_t max_merge, int32_t device,
                    gcs_pmap** out);
int gcs_pmap_destroy(gcs_pmap* pm);
const char* gcs_pmap_last_error(const gcs_pmap* pm);
int gcs_pmap_set_stream(gcs_pmap* pm, void* stream);
/* create_empty_tile (:148-174) into storage index tile */
int gcs_pmap_clear_tile(gcs_pmap* pm, int32_t tile);
/* one field of one tile, host buffer of m_tile x width elements */
int gcs_pmap_read(gcs_pmap* pm, int32_t tile, int32_t field, void* host);
int gcs_pmap_write(gcs_pmap* pm, int32_t tile, int32_t field, const void* host);
/* Device-to-device copy of whole tiles (every field) from src storage slots to dst storage slots (maps of
 * the same m_tile, n_lobes and device; dst == src allowed): the working copy of a hypothesis that reads
 * the node's map but must not update it (backend_node.py:2062,2079-2083). */
int gcs_pmap_copy_tiles(gcs_pmap* dst, const int32_t* dst_tiles, const gcs_pmap* src, const int32_t* src_tiles,
                        int32_t n);
/* tiles: n host storage indices in view order (-1: a tile missing from the map, viewed as empty);
 * tile_ids: the n MA-hex ids written to candidate_tile_ids */
int gcs_pmap_extract_view(gcs_pmap* pm, const int32_t* tiles, const int64_t* tile_ids, int32_t n, int32_t m_view,
                          double eps_lift, double eps_mass, gcs_pmap_view* out);
/* primitive_map_insert_masked for n tiles, K proposals each (rows tile-major, rows.n = n K); ids from
 * next_global_id in tile order.  new_ids (device, n K, -1 where masked) may be NULL; n_inserted and
 * count (host, n each): proposals inserted and the tile's valid count afterwards. */
int gcs_pmap_insert_masked(gcs_pmap* pm, const int32_t* tiles, int32_t n, int32_t K, const gcs_pmap_rows* rows,
                           double timestamp, int64_t scan_seq, double recency_decay_lambda, int64_t next_global_id,
                           int64_t* new_ids, int32_t* n_inserted, int32_t* count);
/* primitive_map_fuse on each of the n tiles with the rows whose tile_pos names it (valid & tile
 * match, pipeline.py:1304-1305); every listed tile gets the call's timestamp at every row's slot and
 * its rgb rebuilt, as the reference's per-tile call does.  n_fused (host): unique row slots. */
int gcs_pmap_fuse(gcs_pmap* pm, const int32_t* tiles, int32_t n, const gcs_pmap_rows* rows, double timestamp,
                  int64_t scan_seq, double eps_mass, int32_t* n_fused);
/* per tile (host, n each): culled count, mass dropped, sum of all weights, valid count afterwards */
int gcs_pmap_cull(gcs_pmap* pm, const int32_t* tiles, int32_t n, double weight_threshold, int32_t* n_culled,
                  double* mass_dropped, double* weight_sum, int32_t* count);
int gcs_pmap_forget(gcs_pmap* pm, const int32_t* tiles, int32_t n, double forgetting_factor);
/* stats (host): [downscale total, cov inflation trace, valid count] over the n tiles */
int gcs_pmap_recency_inflate(gcs_pmap* pm, const int32_t* tiles, int32_t n, int64_t scan_seq,
                             double recency_decay_lambda, double min_scale, double* stats);
/* the whole tile's Bhattacharyya pairs (m_tile <= max_merge); pairs (host, 2 x max_pairs): the merged
 * (kept, removed) slots in selection order */
int gcs_pmap_merge_reduce(gcs_pmap* pm, int32_t tile, double merge_threshold, int32_t max_pairs, double eps_psd,
                          double eps_lift, int32_t* n_merged, int32_t* pairs, int32_t* count);

/* Step 12b of process_scan_single_hypothesis (pipeline.py:1232-1492): the map update at z_t from the
 * scan's MeasurementBatch and PrimitiveAssociationResult over the n active tiles (storage indices +
 * MA-hex ids, the association stencil's tiles): per association block (block_associations_for_fuse,
 * primitive_association.py:561-588) the world-frame rows fused into every active tile; the novelty
 * proposals (a - row mass)+ w of the measurements whose world mean falls in the tile, k_insert_tile
 * per tile by a stable rank, inserted masked (ids from *next_global_id, advanced); then cull, forget
 * and merge-reduce per tile (the merge only when m_tile <= merge_max_tile_size, else the reference's
 * budget cap).  counts (host, n): the tiles' valid counts afterwards. */
typedef struct {            /* PipelineConfig fields (pipeline.py:187-206) and operator epsilons */
  int32_t k_insert_tile;    /* GC_K_INSERT_TILE = 64 */
  int32_t block_size;       /* GC_ASSOC_BLOCK_SIZE = 256 */
  int32_t k_merge_pairs;    /* GC_K_MERGE_PAIRS_PER_TILE = 4 */
  int32_t merge_max_tile_size;  /* GC_PRIMITIVE_MERGE_MAX_TILE_SIZE = 2048 */
  double h_tile;            /* GC_H_TILE = 2.0 */
  double recency_decay_lambda;  /* 0.02 */
  double cull_threshold;    /* 1e-4 */
  double forgetting_factor; /* 0.995 */
  double merge_threshold;   /* 0.1 */
  double eps_lift, eps_mass, eps_psd;  /* 1e-9, 1e-12, 1e-12 */
} gcs_pmap_update_config;

typedef struct {            /* device pointers */
  const double* Lambdas;    /* MeasurementBatch: n_total x 9 (body frame) */
  const double* thetas;     /* n_total x 3 */
  const double* etas;       /* n_total x n_lobes x 3 */
  const double* weights;    /* n_total */
  const uint8_t* valid;     /* n_total */
  const double* colors;     /* n_total x 3, may be NULL */
  const int32_t* sources;   /* n_total, may be NULL (LiDAR) */
  int32_t n_total, n_lobes;
  const double* responsibilities;    /* PrimitiveAssociationResult: n_total x k_assoc */
  const int64_t* candidate_tile_ids; /* n_total x k_assoc */
  const int64_t* candidate_slots;    /* n_total x k_assoc */
  const double* row_masses;          /* n_total */
  int32_t k_assoc;
} gcs_pmap_update_inputs;

typedef struct {            /* MapUpdateCert counters (pipeline.py:1454-1487) */
  int32_t fused_count, insert_count_total, evicted_count, merged_count;
  double fused_mass_total, insert_mass_total, insert_mass_p95, evicted_mass_total;
} gcs_pmap_update_stats;

int gcs_pmap_map_update(gcs_pmap* pm, const int32_t* tiles, const int64_t* tile_ids, int32_t n, const double* z_t6,
                        double timestamp, int64_t scan_seq, int64_t* next_global_id,
                        const gcs_pmap_update_config* cfg, const gcs_pmap_update_inputs* in,
                        gcs_pmap_update_stats* stats, int32_t* counts);

/* ---------------------------------------------------------------- the live primitive path in one call */
/* process_scan_single_hypothesis's live primitive path (pipeline.py:316-1591: the map branch :778-926,
 * visual pose evidence :980-1010, step 12b :1232-1492) as one stream-ordered chain on the context's
 * stream:
 *   gcs_scan_begin -> the active and stencil MA-hex tiles around the predicted position
 *   (tiling.py:167-209) -> surfels of the deskewed points -> recency inflation of the active tiles the
 *   map holds -> the atlas view over the stencil (a tile the map lacks is viewed as empty) -> OT
 *   association -> visual pose evidence at z_lin_pose -> gcs_scan_finish (trigger / ESS sums of the
 *   surfel, recency, association and visual certificates, pipeline.py:1049-1056,1211) -> step 12b at
 *   z_t over the active tiles (new tiles take free storage slots in order, AtlasMap.index).
 * The same kernels on the same arguments as the per-operator entry points, bit for bit, with host
 * waits only where a host value feeds the next launch (begin, the surfel count, the pose evidence).
 * Step 12b is left queued: gcs_live_collect waits for it and returns its statistics; no other call
 * on the context or the map may come between the two.  Contexts: the surfel / association / map
 * contexts are switched to the gcs_ctx's stream.  Stencils of at most 64 tiles. */
#define GCS_LIVE_MAX_TILES 64
typedef struct {
  gcs_surfel_ctx* surfels;
  gcs_assoc_ctx* assoc;
  gcs_pmap* map;
  /* the AtlasMap's tile directory (primitive_map.py:182-227; AtlasMap.tiles / _free / _written) */
  int32_t n_tiles;
  const int64_t* tile_ids;       /* [n_tiles] MA-hex ids held */
  const int32_t* tile_slots;     /* [n_tiles] their storage indices */
  int32_t n_free;
  const int32_t* free_slots;     /* [n_free] free storage indices, in the order new tiles take them */
  const uint8_t* slot_written;   /* [max_tiles] 1: the slot may hold data (a new tile there is cleared) */
  int64_t next_global_id;
  /* tiling and operator parameters (PipelineConfig) */
  double h_tile;
  int32_t r_active_xy, r_active_z, r_stencil_xy, r_stencil_z;
  int32_t n_active_expected, n_stencil_expected;  /* N_ACTIVE_TILES / N_STENCIL_TILES (checked) */
  int64_t scan_seq;
  double recency_lambda, recency_min_scale;
  int32_t m_tile_view;
  double eps_lift, eps_mass;
  const gcs_assoc_config* assoc_cfg;          /* scan_seq / recency_decay_lambda as above */
  const gcs_pmap_update_config* update_cfg;
  double timestamp;                            /* scan_end_time: step 12b's timestamp */
  /* the scan's device buffers (caller-allocated; the surfels read points / timestamps / weights) */
  const double* points_dev;
  const double* timestamps_dev;
  const double* weights_dev;
  int32_t n_points;
  gcs_surfel_outputs* surfel_out;  /* device pointers: the batch's LiDAR slice + the extractor arrays */
  int32_t* lidar_sources_dev;      /* the batch's sources from the LiDAR slice start: 1 on valid rows */
  gcs_assoc_meas meas;             /* the whole MeasurementBatch; n_valid is set from the surfel count */
  const double* batch_colors;      /* n_total x 3 (step 12b) */
  const int32_t* batch_sources;    /* n_total (step 12b) */
  gcs_pmap_view* view;             /* n_stencil x m_tile_view rows */
  int64_t* view_tile_ids_dev;      /* n_stencil: AtlasMapView.tile_ids */
  gcs_assoc_outputs* assoc_out;
  gcs_vpe_outputs* vpe_out;
  void* zero_dev;                  /* zeroed on the stream before the surfels (the batch's arrays), may be NULL */
  int64_t zero_bytes;
} gcs_live_args;

typedef struct {
  int32_t n_active, n_stencil;
  int64_t active_ids[GCS_LIVE_MAX_TILES], stencil_ids[GCS_LIVE_MAX_TILES];
  int32_t active_slots[GCS_LIVE_MAX_TILES];        /* storage index of each active tile (step 12b) */
  int32_t n_present_active;                        /* active tiles the map held before the scan */
  int32_t n_created;                               /* new tiles, in creation order */
  int64_t created_ids[GCS_LIVE_MAX_TILES];
  int32_t created_slots[GCS_LIVE_MAX_TILES];
  double recency_stats[3];                         /* gcs_pmap_recency_inflate's stats */
  double trigger_sum, ess_sum;                     /* the gcs_lidar_evidence handed to the finish */
  double phase_us[12];  /* host clock since the call's entry: [0] begin returned, [1] surfels queued,
                           [3] recency / view / association / pose evidence queued, [4] the one wait for them
                           returned and their results collected, [5] finish returned, [6] step 12b queued;
                           [7] gcs_live_collect's wait (set by gcs_live_collect); [2], [8]-[11] unused (the
                           surfel count is read on the device) */
  /* after gcs_live_collect */
  gcs_pmap_update_stats update;
  int32_t counts[GCS_LIVE_MAX_TILES];              /* valid counts of the active tiles */
  int64_t next_global_id;
} gcs_live_outputs;

/* in: the scan (NULL: gcs_scan_begin already ran on ctx and begin holds its outputs).  begin, out:
 * as gcs_scan_begin / gcs_scan_finish. */
int gcs_live_scan(gcs_ctx* ctx, const gcs_scan_inputs* in, gcs_scan_begin_outputs* begin, const gcs_live_args* a,
                  gcs_live_outputs* lo, gcs_scan_outputs* out);
int gcs_live_collect(gcs_ctx* ctx, gcs_live_outputs* lo);
/* the MA-hex tile ids of tiling.py:167-209 (ma_hex_stencil_tile_ids) around center; returns the count
 * (or GCS_ERR_ARG when it exceeds cap) */
int gcs_ma_hex_stencil(const double* center3, double h_tile, int32_t radius_xy, int32_t radius_z, int64_t* out,
                       int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* GCSLAM_HIP_H */
