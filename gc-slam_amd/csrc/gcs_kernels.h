// Kernel argument blocks and launcher prototypes (internal; the public C-ABI is include/gcslam_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gcs_layout.h"

namespace gcs {

// k_scan draws its tile numbers from a self re-arming ticket (device word, zeroed at creation)

struct ParseArgs {
  const uint8_t* data;  // raw PointCloud2 bytes (device)
  int n, point_step;
  int off_x, off_y, off_z, off_ring, ring_datatype, off_t, t_datatype;
  double header_stamp;
  double R[9], tb[3];   // R_base_lidar, t_base_lidar
  double* points;       // n x 3 base frame
  double* t;
  double* w;
  uint8_t* ring;        // may be null
  uint32_t* ns_flag;
};

struct BudgetArgs {
  const double* w;
  int n_raw, stride;
  double* partials;
  double* scalars;
  uint32_t* zero32;  // scale-mode bucketing state cleared for this scan (may be null)
  int n_zero32;
  uint8_t* zero8;
  int n_zero8;
};

// Clears k_pt does for the next scan (gcs_scan only): its bucket counts (n32 words) and its
// active-flag buffer (n8 bytes)
struct PtClear {
  uint32_t* c32 = nullptr;
  long n32 = 0;
  uint8_t* c8 = nullptr;
  long n8 = 0;
};

// The PT fold's copy of the scan's results to the pinned host mirror (gcs_layout.h Mirror): the
// scalar block, the device error words (read, then zeroed for the next scan), the sequence number and
// the checksum.  torn != 0 (test knob): the sequence word and checksum are stored first and the data
// ~torn microseconds later, so the host meets a mirror whose words have not all arrived.
struct MirrorArgs {
  double* mirror = nullptr;  // device view of the host mirror (null: no copy)
  uint32_t* err = nullptr;   // 4 device error words
  uint64_t seq = 0;
  int torn = 0;
};

struct PointKernelArgs {
  // raw PointCloud2-like input (device)
  const uint8_t* xyz;  // float x,y,z at byte offsets 0,4,8 of each record (double when xyz_f64)
  int point_step;      // bytes per record
  int xyz_f64;
  const double* timestamps;
  const double* weights;
  int n_raw, n_sel, stride, cap;
  // deskew
  double t0, t1;
  double xi[6];
  double origin[3];
  double tau;
  // atlas
  const double* bin_dirs;  // B x 4 (x, y, z, pad)
  int n_bins;
  const int* knn;          // B x k
  int k;
  const int* pools;        // ncell x pool_width, nearest-first (angle from the cell centre), -1 padded
  const float* pool_bound; // per entry: upper bound of the dot with it and every later entry (-2 padded)
  const int* bin_ref;      // device id -> reference id (the nearest-bin tie rule: lower reference id)
  int pool_width, grid;
  // outputs
  PointRec* recs;
  uint32_t* keys;
  uint32_t* slots;
  uint32_t* counts;  // per-bin bucket sizes (cleared by k_budget)
  // direct buckets (scale mode, gcs_scan): members[b * capb + slot] = point index for slot < capb;
  // the first arrival of a bucket marks its K candidate bins and their tiles active (flags); a slot
  // >= capb sets *overflow (host-mapped) and the scan is redone with the sorted bucketing
  uint32_t* members;
  int capb;
  uint8_t* flags;
  int tile_shift;  // log2 of the bin kernel's tile (flags[n_bins + (bin >> tile_shift)] marks active tiles)
  uint32_t* overflow;
  const double* budget_partials;  // k_budget block partials (folded by every k_points block)
  int budget_blocks;
  // self-budget mode (gcs_scan / gcs_map_follow, scale mode; round 6): no k_budget -- each block writes
  // its points' raw mass sums (sum of every raw weight it covers, sum of the selected ones) to
  // mass_rows[block], the records carry w / Z without the budget's mass_scale (the bin kernel folds the
  // rows and applies it as it stages them), and the cert partial row holds raw sums
  // [sum w, sum w^2, sum w win, sum H, max r] that the bin kernel's block 0 scales.  Null: k_budget ran.
  double2* mass_rows;
  double* scalars;
  // optional debug/parity outputs (may be null)
  double* p0_out;
  double* w_out;
  double* w_budget_out;
  int* nearest_out;
  double* iz_out;  // 1 / Z per point (per-operator soft-assign materialisation; the record holds w / Z)
  double* t_out;   // budget-selected timestamps (deskew-only stage: n_bins == 0)
  // the deskew twist in device memory (gcs_scan's pre-launched front: written by k_gate, which the
  // stream runs right before this kernel); null: xi above
  const double* xi_dev;
};
constexpr uint64_t kGateTimeoutTicks = 20000000ull;  // 200 ms of the 100 MHz constant clock

struct BucketArgs {
  int n_bins, k;
  const uint32_t* counts;
  const uint32_t* keys;
  const uint32_t* slots;
  const int* knn;
  uint32_t* starts;
  uint32_t* scan_status;  // per 4096-bucket tile look-back word (re-armed by k_bins_scale)
  uint32_t* scan_ticket;
  uint32_t* slot_idx;     // bucket-ordered point indices, arrival order within a bucket
  uint32_t* perm;         // bucket-ordered point indices, point-index order within a bucket
  uint8_t* flags;         // active bins (cleared by k_budget)
  int tile_shift;         // log2 of the bin kernel's tile
  // error words in host-mapped memory, written only on the rare paths: [0] k_scan look-back spin
  // bound exhausted (the scan's bucket starts are invalid -> gcs_scan fails), [1] k_bucket_rank took
  // the in-order compaction path for a bucket above kRankMax members (correct, degenerate; reported)
  uint32_t* err;
  uint32_t spin_limit;    // look-back spin bound (gcs_ctx_set_debug; default 1 << 22)
  int inject_scan_fail;   // test hook: tile 1 behaves as if its look-back bound were exhausted
};

struct BinKernelArgs {
  const PointRec* recs;   // point order
  const uint32_t* perm;   // bucket order -> point index (scale mode, sorted bucketing)
  const uint32_t* members;  // direct buckets (k_points): bucket b's members at b * capb, arrival order
  int capb;
  const uint32_t* starts;
  const uint32_t* counts;
  const uint8_t* flags;
  uint8_t* tile_dirty;     // per tile: rows / partial row differ from the zero-bin values (persistent)
  const int* rknn_off;
  const int* rknn;
  const uint16_t* rknn_local;  // per reverse-kNN entry: index in its tile's source list
  const int* tile_src_off;     // per tile of bins_tile() bins: CSR into tile_src
  const int* tile_src;         // ascending unique source buckets of the tile
  const double* bin_dirs;
  const double* map;  // map sufficient stats (fused Matrix-Fisher term, scale mode)
  int n_bins, cap;
  int tile_bins;  // bins per k_bins_scale workgroup (bins_tile_for)
  double origin[3];
  double tau;
  double* scan;  // 26 x B field-major
  double* scalars;
  const double* pts_partials;  // if set: k_points' partial rows, folded by block 0
  int pts_blocks;
  // k_points' self-budget mass rows (PointKernelArgs.mass_rows; null: the records carry mass_scale):
  // every staging block folds them (fixed order) into mass_scale; block 0 publishes the budget scalars
  const double2* mass_rows;
  int mass_nrows;
  uint32_t* zero_after;  // bucketing scratch (mid-list length, look-back words) re-armed for the next scan
  int n_zero_after;
  // split finalize (sparse maps, 128-bin tiles; round 6): the gather kernel leaves each active bin's 19
  // raw sums here (field-major, 19 x B) and k_bins_finalize, one thread per bin at full occupancy, writes
  // ScanBinStats, the Matrix-Fisher terms and the active tiles' partial rows.  Null: fused phase D.
  double* raw;
  const int* tile_order;  // block -> tile (k_tile_order; null: identity)
  uint32_t* tile_work;    // per tile: records the tile staged (written for active tiles; may be null)
};

struct PushArgs {
  double R[9];
  double t[3];
  double Stt[9];  // translation block of the pose covariance
  double F[9];    // R S_rt   (rotation rows, translation columns)
  double G[9];    // R S_rr R^T
  double gamma;
};

// Launchers.  e0/e1 (may be null) are stamped with the first kernel's start and the last
// kernel's end through hipExtLaunchKernel, so stage timing adds no marker packets to the queue.
hipError_t launch_parse(const ParseArgs& a, hipStream_t s);
hipError_t launch_budget(const BudgetArgs& a, int nblk, hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// fold: run k_points' cert fold now (else k_bins_scale block 0 folds it, BinKernelArgs.pts_partials)
int points_blocks(long cap, bool scale);  // k_points grid (lanes per point in scale mode)
int points_max_blocks();
// IMU window weights + preintegration on the device (gcs_preint.hip; imu_preintegration.py:20-147)
struct PreintArgs {
  const double* imu;  // pinned host: stamps[m], gyro[m*3], accel[m*3]
  int m;              // samples kept (the trailing run of repeated stamps trimmed to its first)
  int n_tail;         // trimmed samples: zero steps carrying weight w(tail_stamp) each
  double tail_stamp;
  double t0, t1, sigma;  // smooth_window(t, t0, t1, sigma)
  double rotvec[3], gb[3], ab[3], g[3];
  int rotation_only;
  double* xi_dev;     // device: the deskew twist (PointKernelArgs.xi_dev)
  double* host_out;   // pinned host or null: xi[6], ess, delta_pose[6], delta_v[3]
};
hipError_t launch_preint(const PreintArgs& a, hipStream_t s);
// the IMU / odometry evidence family on the device (gcs_imu_odom.hip): one workgroup, windows of at most
// kImuOdomMaxM samples.  win (device): stamps[m], gyro[3m], accel[3m], w_int[m], then the small inputs at
// the ImuOdomSmall offsets; out (device): host::ImuOdomOut + [dt_int, dt_imu, omega_avg 3] (kIoOutWords
// words); host (pinned, mapped; may be null): out's words, the call's sequence number, a checksum
// ... and past those words, kImuOdomStatWords of the window statistics the assembly kernel reads
constexpr int kImuOdomMaxM = 1024;
constexpr int kImuOdomStatWords = 24;
enum ImuOdomSmall : int {
  kIoPose0 = 0, kIoPosePred = 6, kIoMuPrev = 12, kIoMuInc = 34, kIoGravity = 56, kIoSigmaG = 59, kIoSigmaA = 68,
  kIoOdomPose = 77, kIoOdomCov = 83, kIoOdomTwist = 119, kIoOdomTwistCov = 125, kIoSmallLen = 161
};
struct ImuOdomDevArgs {
  const double* win;
  int m;
  double t_last_scan, t_scan, dt_sec;
  double planar_z_ref, planar_z_sigma, planar_vz_sigma;
  double* out;
  double* host;
  uint64_t* dseq;  // device: the calls' sequence counter
};
hipError_t launch_imu_odom(const ImuOdomDevArgs& a, hipStream_t s);
hipError_t launch_gate(const uint64_t* gate, uint64_t seq, double* xi_out, uint32_t* err, hipStream_t s);
// the hypothesis all-reduce's stage-out (gcs_combine_allreduce): the device sum to a host buffer of n
// words + [n] sequence number (*dseq + 1, stored back to *dseq) + [n + 1] checksum (mirror_word_hash)
hipError_t launch_payload_out(const double* src, double* host, int n, uint64_t* dseq, hipStream_t s);
hipError_t launch_delay(int us, hipStream_t s);  // GCS_DEBUG_COMBINE_DELAY
// legacy: the round-3 k_points (scale mode) instead of k_points_lean; mir: the fold's host mirror
// (gcs_scan_begin: the scalars and error words without a D2H copy)
hipError_t launch_points(const PointKernelArgs& a, bool scale, double* partials, int nblk, bool fold, hipStream_t s,
                         hipEvent_t e0, hipEvent_t e1, bool legacy = false, const MirrorArgs& mir = MirrorArgs{});
int scan_tiles(int n_bins);
hipError_t launch_bucketing(const BucketArgs& b, int n, hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// Bins per k_bins_scale tile: 64 (four lanes per bin); GCSLAM_BIN_TILE=32 selects 32-bin tiles with
// eight lanes per bin (measured slower at C2, kept for A/B and parity-tested); 128 / 256 select wider
// tiles with two lanes / one lane per bin and phase D on every wave.
int bins_tile_for(long cap, int n_bins);
int bins_scale_blocks(int n_bins, int tile_bins);
int partial_stride(int nv);  // doubles per block-partial row
// doubles a partials buffer needs for nblocks rows of nv values (+ the two-level fold's rows)
size_t partials_need(long nblocks, int nv);
int bins_max_tile_sources(int tile_bins);  // capacity of its source list
int bins_max_tile_entries(int tile_bins);  // capacity of its reverse-kNN entry list
int bins_partial_nv();
int push_blocks(int n_bins);
// e0/e1 bracket k_bins_scale itself (the roofline kernel), f0/f1 its partial-row fold
hipError_t launch_bins_scale(const BinKernelArgs& a, double* partials, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                             hipEvent_t f0, hipEvent_t f1);
hipError_t launch_dense(const BinKernelArgs& a, double* bin_partials, double* partials, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1);
hipError_t launch_mf(const double* scan, const double* map, int B, double* partials, int nblk, double* scalars,
                     hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// mir.mirror (may be null): host mirror that receives the scalar block after the fold (MirrorArgs)
// act (scan-active bin flags, null = all) and touched (bin has map mass) let k_pt and
// k_pushforward skip bins that are zero in both the scan and the map
hipError_t launch_pt(const double* scan, const double* map, const double* derived, int B, double* partials, int nblk,
                     double* scalars, const MirrorArgs& mir, const uint8_t* act, const uint8_t* touched,
                     hipStream_t s, hipEvent_t e0, hipEvent_t e1, PtClear clr = PtClear{});
// the next scan's bin-tile dispatch order from this scan's active tiles and their staged records
hipError_t launch_tile_order(const uint8_t* active, const uint32_t* work, int n, int* order, hipStream_t s);
// xcd: the XCD-grouped order (k_tile_order_xcd, n % 8 == 0), else the class order alone
hipError_t launch_tile_order_variant(const uint8_t* active, const uint32_t* work, int n, int* order, bool xcd,
                                     hipStream_t s);
hipError_t launch_pushforward(const double* scan, double* map, double* derived, int B, const PushArgs& pa,
                              double* partials, double* scalars, const uint8_t* act, uint8_t* touched, hipStream_t s,
                              hipEvent_t e0, hipEvent_t e1);
// also rebuilds touched from the map
hipError_t launch_map_derive(const double* map, double* derived, int B, double* partials, double* scalars,
                             uint8_t* touched, hipStream_t s);

}  // namespace gcs
