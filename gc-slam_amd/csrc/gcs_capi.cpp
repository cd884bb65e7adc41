// C-ABI of libgcslam_hip.so (include/gcslam_hip.h): per-hypothesis context, the 14-step
// bin-path scan (FS/backend/pipeline.py:316-1591 calling convention), per-operator entry
// points for parity tests, host numerics and the hypothesis all-reduce payload.
#include "gcslam_hip.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <sys/syscall.h>
#include <unistd.h>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "gcs_atlas.h"
#include "gcs_host.h"
#include "gcs_imu_odom_core.h"
#include "gcs_kernels.h"
#include "gcs_layout.h"
#include "gcs_live.h"
#include "gcs_math.h"

using namespace gcs;
using host::Belief;
using host::DZ;

// device stages timed with hipEvents when timing is enabled
enum { ST_POINTS = 0, ST_SORT = 1, ST_BINS = 2, ST_MF = 3, ST_PT = 4, ST_PUSH = 5, ST_BUDGET = 6, ST_BINS_FOLD = 7,
       kStages = 8 };
static_assert(kStages == GCS_N_STAGES, "stage count of the C-ABI");

namespace {
using clk = std::chrono::steady_clock;
double ms_between(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}
}  // namespace

struct gcs_scan_state {
  Belief prev, pred;
  double mu_prev[DZ], mu_inc[DZ], pose0[6], pose_pred[6], xi[6];
  double sigma_warp = 0.0;
  host::PreintOut pre;
  bool use_io = false;
  double io_extra[5] = {0, 0, 0, 0, 0};
  double Tsum = 0.0;
  double cert[GCS_CERT_LEN] = {};
  double Lext[DZ * DZ] = {}, hext[DZ] = {};
  clk::time_point T0, Tp, T1, Ts, T2;
};

struct gcs_ctx {
  gcs_config cfg{};
  int B = 0, cap = 0, K = 0, G = 0, pool_width = 0, ncell = 0, max_raw = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  // atlas (device)
  double* d_bin_dirs = nullptr;
  int* d_knn = nullptr;
  int* d_rknn_off = nullptr;
  int* d_rknn = nullptr;
  int* d_pools = nullptr;
  float* d_pool_bound = nullptr;  // per pool entry: dot upper bound of it and every later entry
  std::vector<double> dirs_host;  // reference order
  std::vector<int> knn_host;      // reference rows and ids
  // device bin order (scale mode: Hilbert patches; dense: identity); order[dev] = reference id
  std::vector<int> order, inv;
  int* d_bin_ref = nullptr;  // device -> reference id (nearest / candidate ids reported in reference ids)
  int* d_tile_src_off = nullptr;
  int* d_tile_src = nullptr;
  uint16_t* d_rknn_local = nullptr;
  int max_tile_src = 0;
  int tile_bins = 64;  // bins per k_bins_scale tile (bins_tile_for)
  int tile_shift = 6;
  // per-point
  PointRec* d_recs = nullptr;
  double* d_iz = nullptr;  // 1 / Z per point, written by the per-operator point stage (gcs_bin_soft_assign)
  bool iz_valid = false;
  // live primitive path (gcs_scan_begin / gcs_scan_finish): deskewed points (cap x 3), weights and
  // budget timestamps on the device, the prologue's state carried to the tail
  double *d_live_p0 = nullptr, *d_live_w = nullptr, *d_live_t = nullptr;
  gcs_scan_state* scan_st = nullptr;
  gcs_scan_outputs* live_out = nullptr;
  bool live_pending = false;
  gcs_pmap* live_map = nullptr;  // gcs_live_scan: the map whose step 12b gcs_live_collect has to read
  // gcs_live_scan hands step 12b's launch calls (~20 kernels) to the worker thread and returns while it
  // makes them (GCSLAM_LIVE_ASYNC=0: inline); gcs_live_collect waits for the worker first
  bool live_async = true;
  bool begin_mirror = true;      // gcs_scan_begin reads the point fold's mirror (GCSLAM_BEGIN_MIRROR=0: copies)
  uint32_t *d_keys = nullptr, *d_slots = nullptr, *d_sorted = nullptr;
  int* d_nearest = nullptr;
  // per-bin bucketing
  // d_counts holds B counts, [B] = mid-list length, [B+1] pad, then one look-back word per
  // 4096-bucket tile: the whole range is cleared by k_budget every scan
  uint32_t *d_counts = nullptr, *d_starts = nullptr, *d_perm = nullptr;
  int n_counts_words = 0;
  uint32_t* d_tickets = nullptr;
  // active-bin flags, double-buffered by scan: the next scan's k_budget clears one buffer while the
  // previous scan's k_pushforward (on push_stream) still reads the other
  uint8_t* d_flags = nullptr;
  uint8_t* d_flags_buf[2] = {nullptr, nullptr};
  // zeroed for the next scan by gcs_scan's k_pt (PtClear): that scan's k_budget skips the clears
  bool counts_clean = false;
  bool flags_clean[2] = {false, false};
  bool pt_clear = true;  // GCSLAM_PT_CLEAR=0 / GCS_DEBUG_PT_CLEAR 0: k_budget clears as before (A/B)
  int budget_max = 128;  // k_budget's block cap (GCSLAM_BUDGET_BLOCKS, 1..1024)
  int flags_cur = 0;
  uint8_t* d_touched = nullptr;     // per bin: the map holds mass (k_map_derive / k_pushforward)
  uint8_t* d_tile_dirty = nullptr;  // k_bins_scale: tile output not the zero-bin values (persistent)
  // multi-round bin grids (C3): block -> tile order built after each pushforward (k_tile_order) from
  // the scan's active tiles and their staged records (d_tile_work); GCSLAM_TILE_ORDER=0: identity
  int* d_tile_order = nullptr;
  uint32_t* d_tile_work = nullptr;
  bool tile_order_on = false;
  // GCSLAM_TILE_ORDER_PUSH=1: k_tile_order deferred to the push stream behind the scan's
  // pushforward (or onto the main stream ahead of the next bin kernel when no pushforward went out on
  // its own stream).  Off: measured slower at C3 (0.2245 -> 0.2355 ms per step, profiles/r04/tod1/):
  // on the main stream behind the PT fold it fills the device while the host runs the tail, the
  // combine and the next prologue; behind the pushforward and its fold it ends after k_points and
  // the next bin kernel waits for it.
  bool tile_order_defer = false;
  bool tile_order_pending = false;
  double* d_bins_part = nullptr;    // k_bins_scale partial rows (persistent: clean tiles keep theirs)
  double* d_bins_raw = nullptr;     // split bin path: active bins' 19 raw sums (field-major; 128-bin tiles)
  double* d_scan = nullptr;
  double* d_map = nullptr;
  double* d_derived = nullptr;
  double* d_bin_partials = nullptr;
  // reductions
  double* d_partials = nullptr;
  size_t partials_len = 0;
  double* d_part_pts = nullptr;  // k_points block partials (folded later in the scale-mode scan)
  double* d_part_push = nullptr; // k_pushforward block partials (its fold runs on push_stream)
  uint32_t* d_parse_flag = nullptr;  // PointCloud2 parse: some per-point time > 1e6 (ns)
  // gcs_scan launches k_pushforward on its own stream, so it overlaps the next scan's point and
  // bucketing kernels; the main stream waits for ev_push before the next bin kernel (join)
  hipStream_t push_stream = nullptr;
  hipEvent_t ev_push = nullptr;
  // recorded on the main stream behind the scan's device stages; the pushforward's stream waits for
  // it (wait_mirror returns before the main stream is idle)
  hipEvent_t ev_stages = nullptr;
  bool stages_done = false;  // wait_mirror saw the scan's stages complete (no event wait for the push)
  bool push_pending = false;
  bool push_main = false;  // experiment knob (GCSLAM_PUSH_MAIN=1): k_pushforward on the main stream
  // Asynchronous pushforward launch (GCSLAM_PUSH_THREAD=0 turns it off): the launch calls of
  // k_pushforward and its fold (~10 us of host time per scan, on the scan's critical path) are made
  // by a per-context worker thread; every later use of the map, the flags or the push event first
  // waits for the worker (push_wait), so the device order is the synchronous one.
  bool push_async = true;
  std::thread push_thread;
  std::atomic<uint64_t> push_req{0}, push_done{0};
  std::atomic<bool> push_stop{false}, push_sleeping{false};
  std::mutex push_mu;
  std::condition_variable push_cv;
  struct PushJob {
    // 0: the scan's pushforward, 1: the next scan's k_budget (row 1 mass sums), 2: the scan's device
    // front (k_budget, the gated k_points, the push join, the bin kernel + fold, k_pt + fold, k_tile_order)
    int kind;
    const gcs_scan_inputs* in;
    uint64_t seq;
    double z_t[6], Sig6[36], gamma;
    hipStream_t s;
    double* partials;
    uint8_t* flags;
    BudgetArgs ba;
    int nblk;
    // 3: the live path's step 12b (gcs_live_scan): the new tiles' clears and the map update's launches
    gcs_pmap* pm;
    int32_t n12, ncl;
    int32_t tiles12[GCS_LIVE_MAX_TILES], clear12[GCS_LIVE_MAX_TILES];
    int64_t tids12[GCS_LIVE_MAX_TILES];
    double ts12;
    int64_t seq12, next12;
    gcs_pmap_update_config ucfg;
    gcs_pmap_update_inputs uin;
  };
  // a ring of two job slots: a submission waits only while both are taken, so the next scan's front
  // queues behind the last scan's pushforward launches instead of waiting for them
  PushJob push_jobs[2]{};
  int push_rc = 0;
  std::string push_err;
  // launch gate of the pre-launched point stage (gcs_scan): [0] sequence word, [1..6] the deskew twist;
  // coherent host memory polled by k_points (GCSLAM_GATE=0: the point stage is launched after the prologue)
  uint64_t* h_gate = nullptr;
  uint64_t* d_gate = nullptr;
  double* d_gate_xi = nullptr;  // device memory: k_gate's copy of the twist for k_points
  uint64_t gate_seq = 0, gate_next = 0;
  // Measured and left off by default (GCSLAM_GATE=1 or GCS_DEBUG_LAUNCH_GATE turns it on): the
  // worker is still making the last pushforward's launch calls when the front is queued, so k_points
  // is launched no earlier than from the main thread, and the gate kernel adds a dependency hop:
  // C2 113.5 vs 106.9 us per step, same box (profiles/r03/gate/)
  bool gate_on = false;
  bool gate_withhold = false;  // fault test (GCS_DEBUG_LAUNCH_GATE = -1): the gate is never opened
  // IMU weights + preintegration on the device (k_preint, GCSLAM_DEVICE_PREINT=1 or
  // GCS_DEBUG_DEVICE_PREINT; not with the launch gate): the prologue stages the IMU window in pinned
  // memory and queues k_preint, k_points reads its twist, the tail reads its record after the sync
  bool device_preint = false;
  // the IMU / odometry evidence family on the device (k_imu_odom, gcs_imu_odom.hip; GCSLAM_DEVICE_IMU_ODOM=1
  // or GCS_DEBUG_DEVICE_IMU_ODOM): launched on io_stream by scan_imu_odom, its stamped record read by
  // finish_imu_odom before the tail needs the evidence
  bool device_imu_odom = false;
  bool io_dev_pending = false;
  hipStream_t io_stream = nullptr;
  double* h_io_stage = nullptr;   // pinned: the window + small inputs (the H2D copy's source)
  double* d_io_win = nullptr;     // device: the same
  double* d_io_out = nullptr;     // device: the kernel's record (kIoOutWords)
  double* h_io_out = nullptr;     // pinned, coherent, mapped: the stamped copy (kIoOutWords + 2)
  double* dh_io_out = nullptr;
  uint64_t* d_io_seq = nullptr;
  uint64_t io_seq = 0;
  int64_t io_rereads = 0, io_syncs = 0;
  hipEvent_t ev_preint = nullptr;  // recorded after each k_preint: its window and record are not touched before it
  bool ev_preint_pending = false;
  bool preint_pending = false;       // the next point stage reads the device twist (d_gate_xi)
  bool preint_host_pending = false;  // st.xi / st.pre / cert[10] still to be read from h_preint_out
  double* h_preint_in = nullptr;     // pinned: the staged window (7 doubles per sample)
  int64_t preint_in_cap = 0;
  double* h_preint_out = nullptr;    // pinned: xi[6], ess, delta_pose[6], delta_v[3]
  int pts_blocks = 0;
  bool pts_fold_pending = false;
  double* d_scalars = nullptr;
  // the scan's host mirror (gcs_layout.h Mirror): pinned, coherent, mapped; written by the PT fold
  double* h_scalars = nullptr;
  double* d_scalars_mirror = nullptr;  // device view of h_scalars
  uint64_t mirror_seq = 0;             // sequence number of the last mirror-writing PT fold
  int64_t mirror_scans = 0, mirror_rereads = 0, mirror_syncs = 0;  // accepted / re-read / via stream sync
  int mirror_torn = 0;                 // test knob (GCS_DEBUG_MIRROR_TORN): data stores delayed, in us
  // device error words (BucketArgs.err, k_points' overflow, k_gate): [0] look-back bound exhausted,
  // [1] degenerate-bucket compaction taken, [2] a direct bucket overflowed, [3] launch gate timeout.
  // Device memory, carried to the host by the mirror (zeroed there) or by pull_err; h_err holds them
  // until the host check that reads a word clears it.
  uint32_t h_err[4] = {0u, 0u, 0u, 0u};
  uint32_t* d_err = nullptr;
  // direct buckets (gcs_scan, scale mode): k_points writes each bucket's members into a fixed row of
  // capb slots and marks the active bins itself; the bin kernel ranks them while staging, so the
  // sorted bucketing (k_scan, k_place, k_bucket_rank) is skipped.  A bucket past capb members sets
  // h_err[2]: that scan is redone with the sorted bucketing, and so are the context's later scans.
  uint32_t* d_members = nullptr;
  int capb = 32, capb_eff = 32;
  bool direct_buckets = true;   // GCSLAM_SORTED_BUCKETS=1 / GCS_DEBUG_SORTED_BUCKETS: always sorted
  bool sorted_sticky = false;   // a bucket overflowed: sorted bucketing from now on
  bool use_direct = false;      // the stages of the current gcs_scan call
  uint32_t spin_limit = 1u << 22;
  int inject_scan_fail = 0;
  // the round-3 point kernel instead of k_points_lean (GCSLAM_POINTS=legacy / GCS_DEBUG_POINT_KERNEL)
  bool legacy_points = [] {
    const char* e = getenv("GCSLAM_POINTS");
    return e && strcmp(e, "legacy") == 0;
  }();
  // hypothesis all-reduce payload (gcs_combine_allreduce): pinned host staging + device buffer
  double* h_payload = nullptr;   // pinned, coherent, mapped: the packed payload (dh_payload: device view)
  double* dh_payload = nullptr;
  double* d_payload = nullptr;   // device: RCCL's receive buffer
  double* d_payload_in = nullptr;  // device: the send buffer when the communicator spans > 1 rank
  int combine_delay_us = 0;      // GCS_DEBUG_COMBINE_DELAY: a straggling peer, simulated on the combine stream
  int sendbuf_mode = -1;         // GCS_DEBUG_SENDBUF: -1 by world size, 0 host, 1 device
  void* comm_seen = nullptr;     // the communicator whose rank count comm_world holds
  int comm_world = 1;
  double* h_psum = nullptr;      // pinned, coherent, mapped: the sum + sequence + checksum (k_payload_out)
  double* dh_psum = nullptr;
  hipStream_t comm_stream = nullptr;  // the all-reduce's own stream (never queued behind the scan's kernels)
  uint64_t pay_seq = 0;          // host copy of d_pay_seq (k_payload_out increments it once per call)
  uint64_t* d_pay_seq = nullptr;
  int64_t pay_rereads = 0, pay_syncs = 0;
  // host state
  Belief belief{};
  // the lifted Cholesky factor of belief.L and its inverse, left by the last scan's tail (the
  // recompose factors post.L, and the anchor drift keeps L): the next PredictDiffusion starts from
  // them instead of factoring and inverting the same matrix again.  Cleared by gcs_ctx_set_belief.
  // one map for all hypotheses (GCS_MAP_*): the last scan's map-update record and the lead's record
  // carried by the last gcs_combine_allreduce
  int map_mode = GCS_MAP_OWN;
  double map_rec[GCS_MAP_REC_LEN] = {};
  double lead_rec[GCS_MAP_REC_LEN] = {};
  bool have_lead_rec = false;
  bool prev_fac_valid = false;
  host::SpdFactor prev_fac;
  double prev_cov[DZ * DZ];
  double iw_nu[7], iw_Psi[7 * 36], Q[DZ * DZ];
  double last_dPsi[7 * 36], last_dnu[7];
  double meas_nu[3], meas_Psi[3 * 9], meas_cert[2] = {0.0, 0.0};  // measurement-noise IW state
  double last_meas_dPsi[3 * 9], last_meas_dnu[3];
  bool have_last = false;
  int last_n_sel = 0, last_stride = 1;
  int budget_blocks = 0;
  // gcs_ctx_host_split: every scan's stage_ms and combine, summed
  double host_sums[10] = {};
  int64_t host_n[2] = {0, 0};
  // the same split per scan since the last reset, the latest kHostHist scans: [pre-device, device
  // submit + wait, tail, whole scan, combine, whole gcs_scan_combine call] (ms; gcs_ctx_host_split_history)
  static constexpr int kHostHist = 4096;
  std::vector<float> host_hist = std::vector<float>((size_t)kHostHist * 6, 0.0f);
  std::atomic<int64_t> worker_tid{0};
  bool budget_pending = false;  // k_budget already queued for the coming point stage (gcs_scan)
  // self-budget scans (round 6; GCSLAM_SELF_BUDGET=0 for A/B): no k_budget -- k_points writes per-block
  // mass rows (d_mass_rows) and unscaled records, the bin kernel folds the rows and applies mass_scale
  // (PointKernelArgs.mass_rows).  budget_self: the pending point stage runs so; recs_deferred: the
  // records the next bin kernel stages carry no mass_scale yet.
  bool self_budget = [] {
    const char* e = getenv("GCSLAM_SELF_BUDGET");
    return !(e && atoi(e) == 0);
  }();
  bool budget_self = false, recs_deferred = false;
  double2* d_mass_rows = nullptr;
  std::vector<double> wimu, wint;  // IMU window weights: within-scan, scan-to-scan (scratch)
  host::ImuOdomOut io;             // step 9 IMU/odometry evidence of the current scan (scratch)
  double grav[3] = {0.0, 0.0, 0.0};  // gravity_W * imu_gravity_scale
  // device stage timing (hipEvents on the context stream; harvested lazily)
  uint32_t timing_mask = 0;
  // a ring of event pairs per stage: each stamped launch takes the next pair, and the pairs are read
  // back (harvest) only by gcs_ctx_stage_times or when a ring is full -- never on the scan's path
  static constexpr int kEvRing = 256;
  std::vector<hipEvent_t> ev[kStages];  // 2 * kEvRing events per stage once timing is enabled
  int ev_n[kStages] = {};               // pairs recorded since the last harvest
  double stage_ms_sum[kStages] = {};
  long stage_count[kStages] = {};
};

namespace {

// Without a context (the push worker's calls) the message goes to this thread's slot, so the
// worker reports the failing call's own error text rather than a later hipGetLastError().
thread_local std::string t_fail_msg;
// set on the push worker: its stage calls report into t_fail_msg (the main thread owns c->err), make
// their launches themselves and do not wait for their own job
thread_local bool t_on_worker = false;

int fail(gcs_ctx* c, int code, const std::string& m) {
  if (c && !t_on_worker) c->err = m;
  else t_fail_msg = m;
  return code;
}

// wait until the push worker has made the launch calls of the last submitted pushforward
int push_wait(gcs_ctx* c) {
  if (t_on_worker || !c->push_thread.joinable()) return GCS_OK;
  const uint64_t r = c->push_req.load(std::memory_order_acquire);
  while (c->push_done.load(std::memory_order_acquire) != r) __builtin_ia32_pause();
  if (c->push_rc) {
    const int rc = c->push_rc;
    c->push_rc = 0;
    return fail(c, rc, c->push_err);
  }
  return GCS_OK;
}

// a free job slot: waits while both are taken (the worker still launching two jobs)
gcs_ctx::PushJob& claim_job(gcs_ctx* c) {
  const uint64_t r = c->push_req.load(std::memory_order_relaxed);
  while (r - c->push_done.load(std::memory_order_acquire) >= 2) __builtin_ia32_pause();
  return c->push_jobs[r & 1];
}

// order the main stream after an in-flight scan pushforward (map, derived, touched, map totals)
// A pushforward whose event has already completed needs no stream wait: its writes are visible to
// every later dispatch, and the wait's barrier packet costs the main queue a few µs (C2 trace: the
// bin kernel started 6.5 µs after k_points ended behind an event that had fired 30 µs before).
// GCSLAM_JOIN_WAIT=always: the stream wait on every scan.
int join_push(gcs_ctx* c) {
  static const bool always = [] {
    const char* e = getenv("GCSLAM_JOIN_WAIT");
    return e && strcmp(e, "always") == 0;
  }();
  if (int rc = push_wait(c)) return rc;
  if (!c->push_pending) return GCS_OK;
  if (always || hipEventQuery(c->ev_push) != hipSuccess) (void)hipStreamWaitEvent(c->stream, c->ev_push, 0);
  c->push_pending = false;
  return GCS_OK;
}

#define HIPCHK(ctx, expr)                                                                         \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return fail((ctx), GCS_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

constexpr int kRedBlocks = 1024;
int red_blocks(long n) { return (int)std::max(1L, std::min((long)kRedBlocks, (n + 255) / 256)); }
// k_pt's grid: GCSLAM_PT_BLOCKS caps it (default kRedBlocks: four bins per thread at C3)
constexpr int kPtBlocksMax = 8192;
int pt_blocks(long n) {
  static const int cap = [] {
    const char* e = getenv("GCSLAM_PT_BLOCKS");
    return e ? std::max(1, std::min(kPtBlocksMax, atoi(e))) : kRedBlocks;
  }();
  return (int)std::max(1L, std::min((long)cap, (n + 255) / 256));
}

// read back a stage's recorded event pairs (oldest first; each waits for its end event)
void harvest_stage(gcs_ctx* c, int st) {
  for (int i = 0; i < c->ev_n[st]; ++i) {
    (void)hipEventSynchronize(c->ev[st][2 * i + 1]);
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, c->ev[st][2 * i], c->ev[st][2 * i + 1]) == hipSuccess) {
      c->stage_ms_sum[st] += ms;
      c->stage_count[st] += 1;
    }
  }
  c->ev_n[st] = 0;
}
void harvest(gcs_ctx* c) {
  for (int st = 0; st < kStages; ++st) harvest_stage(c, st);
}

// Stage events are stamped by the stage's own kernel dispatches (hipExtLaunchKernel), so timing
// adds no marker packets (a hipEventRecord marker costs ~10 us of queue time per record).
struct StageEv {
  hipEvent_t e0 = nullptr, e1 = nullptr;
};
StageEv stage_ev(gcs_ctx* c, int st) {
  StageEv e;
  if (((c->timing_mask >> st) & 1u) && !c->ev[st].empty()) {
    if (c->ev_n[st] == gcs_ctx::kEvRing) harvest_stage(c, st);  // a full ring (long timed runs)
    const int i = c->ev_n[st]++;
    e.e0 = c->ev[st][2 * i];
    e.e1 = c->ev[st][2 * i + 1];
  }
  return e;
}

void to_host_belief(const gcs_belief& in, Belief& b) {
  memcpy(b.X_anchor, in.X_anchor, sizeof(b.X_anchor));
  b.stamp = in.stamp_sec;
  memcpy(b.z_lin, in.z_lin, sizeof(b.z_lin));
  memcpy(b.L, in.L, sizeof(b.L));
  memcpy(b.h, in.h, sizeof(b.h));
}

void from_host_belief(const Belief& b, gcs_belief& out) {
  memcpy(out.X_anchor, b.X_anchor, sizeof(b.X_anchor));
  out.stamp_sec = b.stamp;
  memcpy(out.z_lin, b.z_lin, sizeof(b.z_lin));
  memcpy(out.L, b.L, sizeof(b.L));
  memcpy(out.h, b.h, sizeof(b.h));
}

template <class T>
int upload(gcs_ctx* c, T*& dst, const std::vector<T>& src) {
  if (dst) (void)hipFree(dst);
  dst = nullptr;
  HIPCHK(c, hipMalloc(&dst, std::max<size_t>(1, src.size()) * sizeof(T)));
  if (!src.empty()) HIPCHK(c, hipMemcpy(dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return GCS_OK;
}

// Reference-order field-major rows (F x B) <-> device bin order
void to_device_order(const gcs_ctx* c, int F, const double* ref, double* dev) {
  const size_t B = c->B;
  for (int f = 0; f < F; ++f)
    for (size_t i = 0; i < B; ++i) dev[f * B + i] = ref[f * B + c->order[i]];
}
void to_reference_order(const gcs_ctx* c, int F, const double* dev, double* ref) {
  const size_t B = c->B;
  for (int f = 0; f < F; ++f)
    for (size_t i = 0; i < B; ++i) ref[f * B + c->order[i]] = dev[f * B + i];
}

int upload_atlas(gcs_ctx* c) {
  const int B = c->B, K = c->K;
  const bool scale = c->cfg.mode == GCS_MODE_SCALE;
  // device order: Hilbert patches in scale mode (k_bins_scale tiles), identity in dense mode
  if (scale) {
    atlas::hilbert_order(c->dirs_host.data(), B, c->order);
  } else {
    c->order.resize(B);
    for (int b = 0; b < B; ++b) c->order[b] = b;
  }
  c->inv.assign(B, 0);
  for (int i = 0; i < B; ++i) c->inv[c->order[i]] = i;
  std::vector<double> d4((size_t)B * 4, 0.0);
  for (int i = 0; i < B; ++i)
    for (int k = 0; k < 3; ++k) d4[(size_t)i * 4 + k] = c->dirs_host[(size_t)c->order[i] * 3 + k];
  HIPCHK(c, hipMemcpy(c->d_bin_dirs, d4.data(), d4.size() * sizeof(double), hipMemcpyHostToDevice));
  if (int rc = upload(c, c->d_bin_ref, c->order)) return rc;
  if (scale) {
    // candidate rule on reference ids (ties -> lower reference id), then renamed to device ids
    c->knn_host.assign((size_t)B * K, 0);
    atlas::knn(c->dirs_host.data(), B, K, c->knn_host.data());
    std::vector<int> knn_dev((size_t)B * K);
    for (int i = 0; i < B; ++i)
      for (int k = 0; k < K; ++k) knn_dev[(size_t)i * K + k] = c->inv[c->knn_host[(size_t)c->order[i] * K + k]];
    std::vector<int> off, idx, pools;
    atlas::reverse(knn_dev.data(), B, K, off, idx);
    std::vector<int> src_off, src;
    std::vector<uint16_t> local;
    c->max_tile_src = atlas::tile_sources(off, idx, B, c->tile_bins, src_off, src, local);
    if (c->max_tile_src > bins_max_tile_sources(c->tile_bins))
      return fail(c, GCS_ERR_ARG, "bin atlas too irregular for the tiled bin kernel (tile source list too long)");
    for (int b0 = 0; b0 < B; b0 += c->tile_bins)
      if (off[std::min(B, b0 + c->tile_bins)] - off[b0] > bins_max_tile_entries(c->tile_bins))
        return fail(c, GCS_ERR_ARG, "bin atlas too irregular for the tiled bin kernel (tile reverse-kNN list too long)");
    c->G = atlas::grid_for_bins(B);
    c->ncell = 6 * c->G * c->G;
    // pools keep ascending reference ids (exact nearest-bin tie rule) and hold device ids
    std::vector<float> pbound;  // nearest-first pools with early-exit bounds (k_points' nearest-bin search)
    atlas::cell_pools(c->dirs_host.data(), B, c->G, pools, c->pool_width, &pbound);
    if (int rc = upload(c, c->d_pool_bound, pbound)) return rc;
    for (int& id : pools)
      if (id >= 0) id = c->inv[id];
    if (int rc = upload(c, c->d_pools, pools)) return rc;
    HIPCHK(c, hipMemcpy(c->d_knn, knn_dev.data(), knn_dev.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_rknn_off, off.data(), off.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_rknn, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice));
    if (int rc = upload(c, c->d_tile_src_off, src_off)) return rc;
    if (int rc = upload(c, c->d_tile_src, src)) return rc;
    if (int rc = upload(c, c->d_rknn_local, local)) return rc;
  }
  HIPCHK(c, hipStreamSynchronize(nullptr));  // pageable copies may return before their DMA lands
  return GCS_OK;
}

int submit_budget(gcs_ctx* c, const BudgetArgs& ba, int nblk, hipStream_t s);

// ---------------------------------------------------------------- device stages
// fold_later: leave k_points' cert fold to block 0 of the next k_bins_scale (scale-mode scan)
// Row 1's mass sums (k_budget) need only the weights: gcs_scan queues them before its host
// prologue so they run while the host predicts and preintegrates.  Timed (stage ST_BUDGET), the launch
// is made here with the kernel's own start / end events; otherwise by the worker thread.
// self: a self-budget scan (gcs_ctx::self_budget): only the per-scan clears are launched, when the last
// scan's k_pt did not do them (k_budget with no weights to sum); usually nothing is.
int stage_budget(gcs_ctx* c, const double* w, int n_raw, bool toggle = true, bool self = false) {
  if (n_raw < 0 || n_raw > c->max_raw) return fail(c, GCS_ERR_ARG, "n_points exceeds max_raw_points");
  int stride = std::max(1, (int)((n_raw + (long)c->cap - 1) / c->cap));  // ceil(N/cap), point_budget.py:160
  int n_sel = (n_raw + stride - 1) / stride;
  c->last_n_sel = n_sel;
  c->last_stride = stride;
  hipStream_t s = c->stream;
  if (c->d_flags_buf[0] && toggle) {  // this scan's flag buffer (the other may still be read by k_pushforward)
    c->flags_cur ^= 1;
    c->d_flags = c->d_flags_buf[c->flags_cur];
  }
  BudgetArgs ba{};
  ba.w = w;
  ba.n_raw = n_raw;
  ba.stride = stride;
  ba.partials = c->d_partials;
  ba.scalars = c->d_scalars;
  ba.zero32 = c->d_counts;  // counts only: the bucketing scratch after them is re-armed by k_bins_scale
  ba.n_zero32 = c->d_counts ? c->B : 0;
  ba.zero8 = c->d_flags;
  ba.n_zero8 = c->d_flags ? c->B + bins_scale_blocks(c->B, c->tile_bins) : 0;
  if (c->counts_clean) ba.n_zero32 = 0;  // the last scan's k_pt zeroed them
  c->counts_clean = false;
  if (c->d_flags_buf[0]) {
    if (c->flags_clean[c->flags_cur]) ba.n_zero8 = 0;
    c->flags_clean[c->flags_cur] = false;
  }
  // k_budget's grid: at most budget_max blocks (every k_points block folds all of its partial rows,
  // and on a busy GPU -- the previous scan's pushforward -- each block waits for a CU slot)
  c->budget_blocks = std::min(red_blocks(std::max(n_raw, 1)), c->budget_max);
  c->budget_pending = true;
  c->budget_self = self;
  if (self) {
    if (ba.n_zero32 == 0 && ba.n_zero8 == 0) return GCS_OK;  // nothing to clear: no launch
    ba.n_raw = 0;  // the clears only (its zero partial rows are read by nobody)
  }
  StageEv ev = stage_ev(c, ST_BUDGET);
  if (!ev.e0 && c->push_async && !t_on_worker) return submit_budget(c, ba, c->budget_blocks, s);
  if (int rc = push_wait(c)) return rc;  // the worker's queued launches precede this one on the stream
  HIPCHK(c, launch_budget(ba, c->budget_blocks, s, ev.e0, ev.e1));
  return GCS_OK;
}

// deskew_only: the live primitive path's point stage (gcs_scan_begin): budget gather + deskew into
// p0_out / w_out / t_out, no soft assign
int stage_points(gcs_ctx* c, const void* xyz, int point_step, const double* t, const double* w, int n_raw, double t0,
                 double t1, const double* xi, double* p0_out, double* w_out, double* wb_out, bool fold_later = false,
                 bool xyz_f64 = false, double* iz_out = nullptr, bool deskew_only = false, double* t_out = nullptr,
                 bool to_host = false) {
  if (n_raw < 0 || n_raw > c->max_raw) return fail(c, GCS_ERR_ARG, "n_points exceeds max_raw_points");
  if (point_step < (xyz_f64 ? 24 : 12)) return fail(c, GCS_ERR_ARG, "point_step too small for x, y, z");
  StageEv ev = stage_ev(c, ST_POINTS);
  // a self-budget scan: scale mode, the cert fold left to the bin kernel, no per-point outputs (they
  // carry the budget weights) -- gcs_scan, its pre-launched front and gcs_map_follow
  const bool self_ok = c->self_budget && c->cfg.mode == GCS_MODE_SCALE && !deskew_only && fold_later && !p0_out &&
                       !w_out && !wb_out && !iz_out && !t_out;
  if (!c->budget_pending)  // k_budget not queued earlier by gcs_scan
    if (int rc = stage_budget(c, w, n_raw, true, self_ok)) return rc;
  if (c->budget_self && !self_ok) return fail(c, GCS_ERR_STATE, "self-budget point stage with per-point outputs");
  if (int rc = push_wait(c)) return rc;  // k_budget's launch call (worker) precedes k_points on the stream
  c->budget_pending = false;
  const int n_sel = c->last_n_sel, stride = c->last_stride;
  hipStream_t s = c->stream;
  PointKernelArgs a{};
  a.xyz = (const uint8_t*)xyz;
  a.point_step = point_step;
  a.xyz_f64 = xyz_f64 ? 1 : 0;
  a.timestamps = t;
  a.weights = w;
  a.n_raw = n_raw;
  a.n_sel = n_sel;
  a.stride = stride;
  a.cap = c->cap;
  a.t0 = t0;
  a.t1 = t1;
  memcpy(a.xi, xi, 6 * sizeof(double));
  memcpy(a.origin, c->cfg.lidar_origin, 3 * sizeof(double));
  a.tau = c->cfg.tau;
  a.bin_dirs = c->d_bin_dirs;
  a.n_bins = c->B;
  a.knn = c->d_knn;
  a.k = c->K;
  a.pools = c->d_pools;
  a.pool_bound = c->d_pool_bound;
  a.bin_ref = c->d_bin_ref;
  a.pool_width = c->pool_width;
  a.grid = c->G;
  a.recs = c->d_recs;
  a.keys = c->d_keys;
  a.slots = c->d_slots;
  a.counts = c->d_counts;
  if (c->use_direct) {
    a.members = c->d_members;
    a.capb = c->capb_eff;
    a.flags = c->d_flags;
    a.tile_shift = c->tile_shift;
    a.overflow = c->d_err + 2;
  }
  a.budget_partials = c->budget_self ? nullptr : c->d_partials;
  a.budget_blocks = c->budget_self ? 0 : c->budget_blocks;
  a.mass_rows = c->budget_self ? c->d_mass_rows : nullptr;
  c->recs_deferred = c->budget_self && c->cfg.mode == GCS_MODE_SCALE && !deskew_only;
  a.scalars = c->d_scalars;
  a.p0_out = p0_out;
  a.w_out = w_out;
  a.w_budget_out = wb_out;
  a.nearest_out = c->d_nearest;  // device ids
  a.iz_out = iz_out;
  a.t_out = t_out;
  if (c->gate_next) {  // pre-launched by the scan front: k_gate waits for the twist, k_points reads it
    HIPCHK(c, launch_gate(c->d_gate, c->gate_next, c->d_gate_xi, c->d_err + 3, s));
    a.xi_dev = c->d_gate_xi;
    c->gate_next = 0;
  } else if (c->preint_pending) {  // k_preint, queued by the prologue on this stream, wrote the twist
    a.xi_dev = c->d_gate_xi;
    c->preint_pending = false;
  }
  c->iz_valid = false;
  const bool scale = c->cfg.mode == GCS_MODE_SCALE && !deskew_only;
  if (deskew_only) {
    a.n_bins = 0;  // k_points<false, 0, 1>: no soft assign, no record, no bucketing
    a.nearest_out = nullptr;
    a.members = nullptr;
  }
  c->pts_blocks = points_blocks(c->cap, scale);
  c->pts_fold_pending = scale && fold_later;
  MirrorArgs mir{};
  if (to_host && !c->pts_fold_pending) {  // the fold hands the scalars and error words to the host mirror
    mir.mirror = c->d_scalars_mirror;
    mir.err = c->d_err;
    mir.seq = ++c->mirror_seq;
    mir.torn = c->mirror_torn;
  }
  HIPCHK(c, launch_points(a, scale, c->d_part_pts, c->pts_blocks, !c->pts_fold_pending, s, ev.e0, ev.e1,
                          c->legacy_points, mir));
  return GCS_OK;
}

BinKernelArgs bin_args(gcs_ctx* c) {
  BinKernelArgs b{};
  b.recs = c->d_recs;
  b.perm = c->d_perm;
  if (c->use_direct) {
    b.members = c->d_members;
    b.capb = c->capb_eff;
  }
  b.starts = c->d_starts;
  b.counts = c->d_counts;
  b.flags = c->d_flags;
  b.tile_dirty = c->d_tile_dirty;
  b.tile_order = c->d_tile_order;
  b.tile_work = c->d_tile_work;
  b.rknn_off = c->d_rknn_off;
  b.rknn = c->d_rknn;
  b.rknn_local = c->d_rknn_local;
  b.tile_src_off = c->d_tile_src_off;
  b.tile_src = c->d_tile_src;
  b.bin_dirs = c->d_bin_dirs;
  b.map = c->d_map;
  b.n_bins = c->B;
  b.cap = c->cap;
  b.tile_bins = c->tile_bins;
  b.raw = c->d_bins_raw;
  memcpy(b.origin, c->cfg.lidar_origin, 3 * sizeof(double));
  b.tau = c->cfg.tau;
  b.scan = c->d_scan;
  b.scalars = c->d_scalars;
  if (c->pts_fold_pending) {
    b.pts_partials = c->d_part_pts;
    b.pts_blocks = c->pts_blocks;
  }
  if (c->recs_deferred) {  // the self-budget point stage's mass rows (one per k_points block)
    b.mass_rows = c->d_mass_rows;
    b.mass_nrows = c->pts_blocks;
  }
  if (c->d_counts) {
    b.zero_after = c->d_counts + c->B;
    b.n_zero_after = c->n_counts_words - c->B;
  }
  return b;
}

int flush_tile_order(gcs_ctx* c, hipStream_t s, gcs_ctx* ec);
int stage_bins(gcs_ctx* c) {
  hipStream_t s = c->stream;
  if (int rc = flush_tile_order(c, s, c)) return rc;  // (a tile order no pushforward took)
  BinKernelArgs b = bin_args(c);
  if (c->cfg.mode == GCS_MODE_SCALE) {
    if (!c->use_direct) {  // sorted bucketing (direct buckets: k_points placed and flagged them)
      StageEv ev = stage_ev(c, ST_SORT);
      BucketArgs ba{};
      ba.n_bins = c->B;
      ba.k = c->K;
      ba.counts = c->d_counts;
      ba.keys = c->d_keys;
      ba.slots = c->d_slots;
      ba.knn = c->d_knn;
      ba.starts = c->d_starts;
      ba.scan_status = c->d_counts + c->B + 2;
      ba.scan_ticket = c->d_tickets;
      ba.slot_idx = c->d_sorted;
      ba.perm = c->d_perm;
      ba.flags = c->d_flags;
      ba.tile_shift = c->tile_shift;
      ba.err = c->d_err;
      ba.spin_limit = c->spin_limit;
      ba.inject_scan_fail = c->inject_scan_fail;
      HIPCHK(c, launch_bucketing(ba, c->cap, s, ev.e0, ev.e1));
    }
    StageEv ev = stage_ev(c, ST_BINS), evf = stage_ev(c, ST_BINS_FOLD);
    // stage = the bin kernel itself; ST_BINS_FOLD = its partial-row fold (+ R_mf)
    HIPCHK(c, launch_bins_scale(b, c->d_bins_part, s, ev.e0, ev.e1, evf.e0, evf.e1));
    c->pts_fold_pending = false;
  } else {
    StageEv ev = stage_ev(c, ST_BINS);
    HIPCHK(c, launch_dense(b, c->d_bin_partials, c->d_partials, s, ev.e0, ev.e1));
  }
  return GCS_OK;
}

int stage_mf(gcs_ctx* c) {
  StageEv ev = stage_ev(c, ST_MF);
  HIPCHK(c, launch_mf(c->d_scan, c->d_map, c->B, c->d_partials, red_blocks(c->B), c->d_scalars, c->stream, ev.e0,
                      ev.e1));
  return GCS_OK;
}

// a validated mirror's error words into h_err (a word stays set until the check that reads it clears it)
void take_mirror_err(gcs_ctx* c) {
  const uint64_t* m = reinterpret_cast<const uint64_t*>(c->h_scalars);
  for (int k = 0; k < 2; ++k) {
    c->h_err[2 * k] |= (uint32_t)(m[MIR_ERR + k] & 0xffffffffu);
    c->h_err[2 * k + 1] |= (uint32_t)(m[MIR_ERR + k] >> 32);
  }
}

// Wait for a stamped host buffer: words [0, n) of data, [n] the sequence number of the launch that
// writes it, [n + 1] the checksum sum_i mirror_word_hash(w_i, i) + mirror_word_hash(seq, n) (k_final's
// scan mirror, k_payload_out's all-reduce sum).  The host polls the sequence word (a stream
// synchronize returns some microseconds after the kernel ends) and accepts the buffer only when the
// checksum of what it reads matches: a buffer whose data words have not all reached host memory when
// the sequence word has is re-read (*rereads), never consumed.  Without a valid buffer after 20 ms (a
// fault, or a stalled queue) the stream synchronize waits and reports the asynchronous error (*syncs),
// and the buffer must then be complete.  GCSLAM_SYNC_WAIT=stream: synchronize only.
uint64_t stamped_sum(const volatile uint64_t* m, int n) {
  uint64_t s = 0;
  for (int i = 0; i < n; ++i) s += mirror_word_hash(m[i], (uint32_t)i);
  return s + mirror_word_hash(m[n], (uint32_t)n);
}

int wait_stamped(gcs_ctx* c, const double* buf, int n, uint64_t seq, hipStream_t stream, int64_t* rereads,
                 int64_t* syncs, const char* what) {
  static const bool spin = [] {
    const char* e = getenv("GCSLAM_SYNC_WAIT");
    return !(e && strcmp(e, "stream") == 0);
  }();
  const volatile uint64_t* m = reinterpret_cast<const volatile uint64_t*>(buf);
  if (spin) {
    const auto t0 = clk::now();
    bool reread = false;
    for (;;) {
      if (m[n] == seq) {
        std::atomic_thread_fence(std::memory_order_acquire);
        if (stamped_sum(m, n) == m[n + 1]) {
          std::atomic_thread_fence(std::memory_order_acquire);
          if (reread) ++*rereads;
          return GCS_OK;
        }
        reread = true;  // the sequence word is here, some data word is not yet: read again
      }
      __builtin_ia32_pause();
      if (clk::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    ++*syncs;
  }
  HIPCHK(c, hipStreamSynchronize(stream));
  if (m[n] != seq || stamped_sum(m, n) != m[n + 1])
    return fail(c, GCS_ERR_HIP, std::string(what) + ": sequence " + std::to_string((unsigned long long)m[n]) +
                                    " / checksum do not match launch " + std::to_string((unsigned long long)seq) +
                                    " after the stream synchronized");
  return GCS_OK;
}

// Wait for the scan's device stages: the PT fold's scan mirror (k_final; gcs_layout.h Mirror) through
// wait_stamped.  Nothing later in the scan reads device memory outside stream order.
int wait_mirror(gcs_ctx* c) {
  if (int rc = wait_stamped(c, c->h_scalars, MIR_SEQ, c->mirror_seq, c->stream, &c->mirror_rereads, &c->mirror_syncs,
                            "scan mirror"))
    return rc;
  take_mirror_err(c);
  ++c->mirror_scans;
  c->stages_done = true;
  return GCS_OK;
}

// clear_next (gcs_scan): k_pt also zeroes the bucket counts (the bin kernel, their last reader, is
// behind it on this stream) and the other flag buffer -- the next scan's -- whose last reader, the
// previous scan's pushforward, completed before this scan's bin kernel (join_push); the next
// k_budget then only sums the weights.  Measured: DESIGN.md section 5 (round 4).
int stage_pt(gcs_ctx* c, bool to_host = false, bool clear_next = false) {
  StageEv ev = stage_ev(c, ST_PT);
  MirrorArgs mir{};
  if (to_host) {
    mir.mirror = c->d_scalars_mirror;
    mir.err = c->d_err;
    mir.seq = ++c->mirror_seq;
    mir.torn = c->mirror_torn;
  }
  PtClear clr{};
  if (clear_next && c->pt_clear && c->d_counts && c->d_flags_buf[0]) {
    clr.c32 = c->d_counts;
    clr.n32 = c->B;
    clr.c8 = c->d_flags_buf[c->flags_cur ^ 1];
    clr.n8 = c->B + bins_scale_blocks(c->B, c->tile_bins);
  }
  HIPCHK(c, launch_pt(c->d_scan, c->d_map, c->d_derived, c->B, c->d_partials, pt_blocks(c->B), c->d_scalars,
                      mir, c->d_flags, c->d_touched, c->stream, ev.e0, ev.e1, clr));
  if (clr.c32) {
    c->counts_clean = true;
    c->flags_clean[c->flags_cur ^ 1] = true;
  }
  if (to_host) HIPCHK(c, hipEventRecord(c->ev_stages, c->stream));
  c->stages_done = false;
  return GCS_OK;
}

// the next scan's bin-tile dispatch order from this scan's bin kernel (d_tile_dirty / d_tile_work ->
// d_tile_order; read only by the next bin kernel, written by nothing else), queued on the main stream
// behind the scan's stages: the device runs it while the host runs the tail (the next bin kernel is
// behind it in stream order).  Deferred (GCSLAM_TILE_ORDER_PUSH=1, measured slower): the scan's
// pushforward takes it onto the push stream behind itself (stage_push, after the stages) and the next
// bin kernel is ordered after it by join_push; a scan whose pushforward does not go out on its own
// stream leaves it pending, and the next stage_bins queues it on the main stream.
int flush_tile_order(gcs_ctx* c, hipStream_t s, gcs_ctx* ec) {
  if (!c->tile_order_pending) return GCS_OK;
  c->tile_order_pending = false;
  HIPCHK(ec, launch_tile_order(c->d_tile_dirty, c->d_tile_work, bins_scale_blocks(c->B, c->tile_bins), c->d_tile_order,
                               s));
  return GCS_OK;
}
int stage_tile_order(gcs_ctx* c) {
  if (!c->tile_order_on) return GCS_OK;
  c->tile_order_pending = true;
  if (c->tile_order_defer && !c->push_main && c->push_stream) return GCS_OK;
  return flush_tile_order(c, c->stream, c);
}

// on_worker: called by the push worker; errors are returned, not written to the context's message
int stage_push(gcs_ctx* c, const double* z_t, const double* Sig6, double gamma, hipStream_t s, double* partials,
               uint8_t* flags, bool on_worker = false) {
  gcs_ctx* ec = on_worker ? nullptr : c;
  PushArgs pa{};
  so3_exp(z_t + 3, pa.R);
  pa.t[0] = z_t[0];
  pa.t[1] = z_t[1];
  pa.t[2] = 0.0;  // t_z := 0 before the map update (CHANGELOG.md:575-578)
  double Srt[9], Srr[9], RS[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      pa.Stt[3 * i + j] = Sig6[6 * i + j];
      Srt[3 * i + j] = Sig6[6 * (3 + i) + j];
      Srr[3 * i + j] = Sig6[6 * (3 + i) + 3 + j];
    }
  mat3_mul(pa.R, Srt, pa.F);
  mat3_mul(pa.R, Srr, RS);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) pa.G[3 * i + j] = RS[3 * i] * pa.R[3 * j] + RS[3 * i + 1] * pa.R[3 * j + 1] + RS[3 * i + 2] * pa.R[3 * j + 2];
  pa.gamma = gamma;
  StageEv ev = stage_ev(c, ST_PUSH);
  // the main stream's stages are complete once wait_mirror saw the fold's ready word (the fold is
  // the stream's last kernel before it): only the other paths order the push stream by the event.
  // k_tile_order runs on the main stream after that fold, where it may run beside this pushforward
  // (or behind it on the same stream, GCSLAM_TILE_ORDER_PUSH=1): it reads d_tile_dirty / d_tile_work
  // and writes d_tile_order, and the pushforward reads d_scan / d_flags and writes d_map / d_derived /
  // d_touched / its partials and map-total scalars -- disjoint buffers, which the two must keep.  A fault in k_tile_order is reported by the
  // next call that synchronises its stream.
  if (s != c->stream && !c->stages_done) HIPCHK(ec, hipStreamWaitEvent(s, c->ev_stages, 0));
  HIPCHK(ec, launch_pushforward(c->d_scan, c->d_map, c->d_derived, c->B, pa, partials, c->d_scalars, flags,
                               c->d_touched, s, ev.e0, ev.e1));
  // the deferred tile order behind it (the stages it reads are complete, as for the pushforward)
  if (int rc = flush_tile_order(c, s, ec)) return rc;
  if (s != c->stream) {
    HIPCHK(ec, hipEventRecord(c->ev_push, s));
    c->push_pending = true;
  }
  return GCS_OK;
}

// The push worker: waits (spin, then sleep) for a submitted job and makes its launch calls with the
// job's captured arguments (the flags buffer of that scan; the context's device buffers are fixed).
int scan_front(gcs_ctx* c, const gcs_scan_inputs* in, uint64_t seq);

void push_worker(gcs_ctx* c) {
  (void)hipSetDevice(c->cfg.device);
  c->worker_tid.store((int64_t)syscall(SYS_gettid));
  t_on_worker = true;
  uint64_t seen = 0;
  for (;;) {
    // spin for up to 2 ms after the last job (a scan every 0.1-0.3 ms keeps the worker awake: a
    // futex wake-up costs tens of microseconds, which at C3 delayed the pushforward behind the
    // next scan's bin kernel), then sleep until the next submission
    int spins = 0;
    auto t_idle = std::chrono::steady_clock::now();
    while (c->push_req.load() == seen && !c->push_stop.load()) {
      __builtin_ia32_pause();
      if ((++spins & 255) != 0 || std::chrono::steady_clock::now() - t_idle < std::chrono::milliseconds(2))
        continue;
      std::unique_lock<std::mutex> lk(c->push_mu);
      c->push_sleeping.store(true);
      c->push_cv.wait(lk, [&] { return c->push_req.load() != seen || c->push_stop.load(); });
      c->push_sleeping.store(false);
      t_idle = std::chrono::steady_clock::now();
    }
    const uint64_t r = c->push_req.load(std::memory_order_acquire);
    if (r == seen) return;  // stop requested, nothing pending
    for (; seen < r; ++seen) {  // the queued jobs in submission order
      const gcs_ctx::PushJob& j = c->push_jobs[seen & 1];
      int rc = GCS_OK;
      std::string msg;
      if (j.kind == 1) {
        const hipError_t e = launch_budget(j.ba, j.nblk, j.s, nullptr, nullptr);
        if (e != hipSuccess) {
          rc = GCS_ERR_HIP;
          msg = "k_budget launch (worker): " + std::string(hipGetErrorString(e));
        }
      } else if (j.kind == 2) {
        rc = scan_front(c, j.in, j.seq);
        if (rc) msg = "scan front launch (worker): " + t_fail_msg;
      } else if (j.kind == 3) {
        for (int k = 0; k < j.ncl && !rc; ++k) rc = live::pmap_clear_tile_launch(j.pm, j.clear12[k]);
        if (!rc)
          rc = live::pmap_update_launch(j.pm, j.tiles12, j.tids12, j.n12, j.z_t, j.ts12, j.seq12, j.next12, &j.ucfg,
                                        &j.uin);
        if (rc) msg = "gcs_pmap_map_update (live path, worker): " + std::string(gcs_pmap_last_error(j.pm));
      } else {
        rc = stage_push(c, j.z_t, j.Sig6, j.gamma, j.s, j.partials, j.flags, true);
        if (rc) msg = "pushforward launch (worker): " + t_fail_msg;
      }
      if (rc && !c->push_rc) {  // the first failure is the one push_wait reports
        c->push_err = msg;
        c->push_rc = rc;
      }
      c->push_done.store(seen + 1, std::memory_order_release);
    }
  }
}

// launch the scan's pushforward: on the worker (default) or inline (timing the push stage, or
// GCSLAM_PUSH_THREAD=0)
int submit_push(gcs_ctx* c, const double* z_t, const double* Sig6, double gamma, hipStream_t s, double* partials) {
  const bool timed = (c->timing_mask >> ST_PUSH) & 1u;
  if (!c->push_async || timed) {
    if (int rc = push_wait(c)) return rc;
    return stage_push(c, z_t, Sig6, gamma, s, partials, c->d_flags);
  }
  if (!c->push_thread.joinable()) c->push_thread = std::thread(push_worker, c);
  gcs_ctx::PushJob& j = claim_job(c);
  j.kind = 0;
  memcpy(j.z_t, z_t, sizeof(j.z_t));
  memcpy(j.Sig6, Sig6, sizeof(j.Sig6));
  j.gamma = gamma;
  j.s = s;
  j.partials = partials;
  j.flags = c->d_flags;
  c->push_req.fetch_add(1);
  if (c->push_sleeping.load()) {
    std::lock_guard<std::mutex> lk(c->push_mu);
    c->push_cv.notify_one();
  }
  return GCS_OK;
}

// k_budget's launch call on the worker too (gcs_scan queues it before its host prologue): the main
// thread goes straight to PredictDiffusion; stage_points waits for the worker (push_wait) before it
// queues k_points behind it on the same stream, so the device order is the synchronous one.
int submit_budget(gcs_ctx* c, const BudgetArgs& ba, int nblk, hipStream_t s) {
  if (!c->push_thread.joinable()) c->push_thread = std::thread(push_worker, c);
  gcs_ctx::PushJob& j = claim_job(c);  // (queued behind the last scan's pushforward launches)
  j.kind = 1;
  j.ba = ba;
  j.nblk = nblk;
  j.s = s;
  c->push_req.fetch_add(1);
  if (c->push_sleeping.load()) {
    std::lock_guard<std::mutex> lk(c->push_mu);
    c->push_cv.notify_one();
  }
  return GCS_OK;
}

// The scan's device front, queued by the worker while the main thread runs the host prologue:
// k_budget, k_points behind the launch gate (it waits on the device for the twist), the join with
// the last pushforward, the bin kernel + fold, k_pt + fold (mirror, ready word) and k_tile_order --
// the launch calls and the dispatch latency of the point stage leave the scan's critical path.
int scan_front(gcs_ctx* c, const gcs_scan_inputs* in, uint64_t seq) {
  static const double kNoTwist[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  c->budget_pending = false;
  c->gate_next = seq;
  if (int rc = stage_points(c, in->xyz_dev, in->point_step, in->timestamps_dev, in->weights_dev, in->n_points,
                            in->scan_start_time, in->scan_end_time, kNoTwist, nullptr, nullptr, nullptr,
                            /*fold_later=*/true, in->xyz_format == 1))
    return rc;
  if (int rc = join_push(c)) return rc;
  if (int rc = stage_bins(c)) return rc;
  if (int rc = stage_pt(c, /*to_host=*/true, /*clear_next=*/true)) return rc;
  return stage_tile_order(c);
}

int submit_front(gcs_ctx* c, const gcs_scan_inputs* in, uint64_t seq) {
  if (!c->push_thread.joinable()) c->push_thread = std::thread(push_worker, c);
  gcs_ctx::PushJob& j = claim_job(c);  // (queued behind the last scan's pushforward launches)
  j.kind = 2;
  j.in = in;
  j.seq = seq;
  c->push_req.fetch_add(1);
  if (c->push_sleeping.load()) {
    std::lock_guard<std::mutex> lk(c->push_mu);
    c->push_cv.notify_one();
  }
  return GCS_OK;
}

// the twist, then the sequence word (x86 stores are ordered; the fence keeps the compiler's order)
void open_gate(gcs_ctx* c, const double* xi) {
  volatile uint64_t* g = c->h_gate;
  for (int k = 0; k < 6; ++k) {
    uint64_t u;
    memcpy(&u, xi + k, sizeof(u));
    g[1 + k] = u;
  }
  std::atomic_thread_fence(std::memory_order_release);
  __atomic_store_n(c->h_gate, c->gate_seq, __ATOMIC_RELEASE);
}

// On every early return of a pre-launched scan: opens the gate (zero twist), so no point block waits
// for its timeout, and waits for the worker's launch calls, which read the context's per-scan state
struct GateGuard {
  gcs_ctx* c;
  bool open = false, joined = false;
  ~GateGuard() {
    static const double kNoTwist[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (!open && !c->gate_withhold) open_gate(c, kNoTwist);
    if (!joined) {
      const std::string keep = c->err;  // the scan's own failure is the message to report
      (void)push_wait(c);
      c->err = keep;
    }
  }
};

// after a stream sync: a k_scan whose look-back bound ran out left wrong bucket starts
int check_bucket_err(gcs_ctx* c) {
  if (c->h_err[0]) {
    c->h_err[0] = 0u;
    return fail(c, GCS_ERR_HIP, "k_scan: decoupled look-back exceeded its spin bound; bucket starts invalid, scan failed");
  }
  return GCS_OK;
}

// the device error words into h_err after the stream's work (paths without the scan mirror), re-armed
int pull_err(gcs_ctx* c) {
  uint32_t e[4];
  HIPCHK(c, hipMemcpyAsync(e, c->d_err, sizeof(e), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(e), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < 4; ++k) c->h_err[k] |= e[k];
  return GCS_OK;
}

int pull_scalars(gcs_ctx* c) {
  HIPCHK(c, hipMemcpyAsync(c->h_scalars, c->d_scalars, SC_COUNT * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  return pull_err(c);
}

// The IMU/odometry branch from the quantities the reference reads (pipeline.py:442-566,595-776):
// dt_int, dt_imu, omega_avg and the scan-to-scan preintegration, then the eleven factors.
// extra = [dt_int, dt_imu, omega_avg(3)]
void run_imu_odom(const gcs_imu_odom_inputs& in, host::ImuOdomOut& io, double* extra) {
  const double dt_int = host::imu_integration_time(in.m, in.stamps, in.t_last_scan, in.t_scan);
  double dt_imu, om[3];
  host::imu_rate_stats(in.m, in.stamps, in.gyro, in.w_int, in.mu_inc + 9, &dt_imu, om);
  host::PreintOut pre;
  host::preintegrate_imu(in.m, in.stamps, in.gyro, in.accel, in.w_int, in.pose0 + 3, in.mu_inc + 9, in.mu_inc + 12,
                         in.gravity_W, pre);
  host::ImuOdomInputs a{};
  a.m = in.m;
  a.stamps = in.stamps; a.gyro = in.gyro; a.accel = in.accel; a.w_int = in.w_int;
  a.dt_imu = dt_imu; a.dt_int = dt_int; a.dt_sec = in.dt_sec;
  a.omega_avg = om;
  a.drot_int = pre.delta_pose + 3; a.dp_int = pre.delta_pose; a.dv_int = pre.delta_v;
  a.pose0 = in.pose0; a.pose_pred = in.pose_pred; a.mu_prev = in.mu_prev; a.mu_inc = in.mu_inc;
  a.accel_bias = in.mu_inc + 12;
  a.gravity = in.gravity_W;
  a.Sigma_g = in.Sigma_g; a.Sigma_a = in.Sigma_a;
  a.odom_pose = in.odom_pose; a.odom_cov = in.odom_cov_se3; a.odom_twist = in.odom_twist;
  a.odom_twist_cov = in.odom_twist_cov;
  a.planar_z_ref = in.planar_z_ref; a.planar_z_sigma = in.planar_z_sigma; a.planar_vz_sigma = in.planar_vz_sigma;
  host::imu_odom_branch(a, io);
  if (extra) { extra[0] = dt_int; extra[1] = dt_imu; extra[2] = om[0]; extra[3] = om[1]; extra[4] = om[2]; }
}

// node defaults when no odometry has arrived (backend_node.py:939-940,2047-2051)
const double kZero6[6] = {0, 0, 0, 0, 0, 0};
struct BigCov6 {
  double v[36];
  BigCov6() { for (int i = 0; i < 36; ++i) v[i] = (i % 7 == 0) ? 1e12 : 0.0; }
};
const BigCov6 kBigCov6;

double trig(double lift, double psd, double nu, double mer, double rho, double dts, double exs, double alpha, double beta) {
  return lift + psd + nu + mer + rho + fabs(1.0 - dts) + fabs(1.0 - exs) + fabs(1.0 - alpha) + fabs(1.0 - beta);
}

}  // namespace

extern "C" {

const char* gcs_version(void) { return "gcslam-mi355x 0.1.0 (gfx950)"; }
int gcs_abi_version(void) { return GCS_ABI_VERSION; }
// a failed gcs_ctx_create leaves no context: its message is kept per thread for gcs_last_error(NULL)
thread_local std::string t_create_msg;
const char* gcs_last_error(const gcs_ctx* ctx) {
  return ctx ? ctx->err.c_str() : (t_create_msg.empty() ? "null context" : t_create_msg.c_str());
}

int gcs_config_defaults(gcs_config* c) {
  if (!c) return GCS_ERR_ARG;
  memset(c, 0, sizeof(*c));
  c->n_bins = 48;            // legacy B_BINS (CHANGELOG.md:492)
  c->n_points_cap = 8192;    // constants.py:64
  c->max_raw_points = 1 << 16;
  c->mode = GCS_MODE_DENSE;
  c->k_cand = 16;
  c->tau = 0.1;              // DECLARED tau at B = 48
  c->forgetting_factor = 0.99;
  c->gravity_W[2] = -9.81;   // constants.py:80
  c->use_imu_odom = 1;
  c->imu_gravity_scale = 1.0;
  c->planar_z_ref = 0.0;
  c->planar_z_sigma = 0.1;
  c->planar_vz_sigma = 0.01;
  c->alpha_min = 1.0;
  c->alpha_max = 1.0;
  c->c0_cond = 1e6;
  return GCS_OK;
}

int gcs_ctx_create(const gcs_config* cfg, gcs_ctx** out) {
  if (!cfg || !out) return GCS_ERR_ARG;
  *out = nullptr;
  if (!(cfg->planar_z_sigma > 0.0) || !(cfg->planar_vz_sigma > 0.0) || !(cfg->alpha_min <= cfg->alpha_max) ||
      !(cfg->c0_cond > 0.0))
    return GCS_ERR_ARG;  // gcs_config_defaults() fills these
  if (cfg->n_bins < 1 || cfg->n_points_cap < 1 || cfg->max_raw_points < 0) return GCS_ERR_ARG;
  // scale mode: the point kernel is instantiated for K = 8, 16, 32 and the bucketing reads kNN rows as int4
  if (cfg->mode == GCS_MODE_SCALE && ((cfg->k_cand != 8 && cfg->k_cand != 16 && cfg->k_cand != 32) || cfg->k_cand > cfg->n_bins))
    return GCS_ERR_ARG;
  if (!(cfg->tau > 0.0)) return GCS_ERR_ARG;
  t_create_msg.clear();
  gcs_ctx* c = new gcs_ctx();
  c->scan_st = new gcs_scan_state();
  c->live_out = new gcs_scan_outputs();
  c->cfg = *cfg;
  c->B = cfg->n_bins;
  c->cap = cfg->n_points_cap;
  c->tile_bins = bins_tile_for(c->cap, c->B);
  c->tile_shift = __builtin_ctz((unsigned)c->tile_bins);
  c->K = cfg->mode == GCS_MODE_SCALE ? cfg->k_cand : 0;
  c->max_raw = cfg->max_raw_points;
  for (int k = 0; k < 3; ++k) c->grav[k] = cfg->gravity_W[k] * cfg->imu_gravity_scale;
  auto bad = [&](hipError_t e) {
    if (e != hipSuccess) {
      gcs_ctx_destroy(c);
      return true;
    }
    return false;
  };
  if (bad(hipSetDevice(cfg->device))) return GCS_ERR_HIP;
  // GCSLAM_STREAM_PRIO=1: the scan stages' stream at the device's highest priority and the pushforward's
  // at its lowest, so the next scan's front takes the CUs the previous pushforward frees (A/B knob)
  {
    const char* e = getenv("GCSLAM_STREAM_PRIO");
    int lo = 0, hi = 0;
    if (e && atoi(e) != 0 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
      if (bad(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi))) return GCS_ERR_HIP;
      c->own_stream = true;
      if (bad(hipStreamCreateWithPriority(&c->push_stream, hipStreamNonBlocking, lo))) return GCS_ERR_HIP;
    } else {
      if (bad(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking))) return GCS_ERR_HIP;
      c->own_stream = true;
      if (bad(hipStreamCreateWithFlags(&c->push_stream, hipStreamNonBlocking))) return GCS_ERR_HIP;
    }
  }
  if (bad(hipEventCreateWithFlags(&c->ev_push, hipEventDisableTiming))) return GCS_ERR_HIP;
  if (bad(hipEventCreateWithFlags(&c->ev_stages, hipEventDisableTiming))) return GCS_ERR_HIP;
  if (const char* pm = getenv("GCSLAM_PUSH_MAIN")) c->push_main = atoi(pm) != 0;
  if (const char* pt = getenv("GCSLAM_PUSH_THREAD")) c->push_async = atoi(pt) != 0;
  if (const char* sb = getenv("GCSLAM_SORTED_BUCKETS")) c->direct_buckets = atoi(sb) == 0;
  const size_t B = c->B, cap = c->cap;
  if (bad(hipMalloc(&c->d_bin_dirs, B * 4 * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_recs, cap * sizeof(PointRec)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_iz, cap * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_live_p0, 3 * cap * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_live_w, cap * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_live_t, cap * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_nearest, cap * sizeof(int)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_scan, B * SF_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_map, B * MF_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_derived, B * MD_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMemset(c->d_map, 0, B * MF_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMemset(c->d_scan, 0, B * SF_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_touched, B))) return GCS_ERR_HIP;
  c->partials_len = std::max<size_t>({partials_need(kRedBlocks, 24), partials_need(pt_blocks(c->B), 13), partials_need(bins_scale_blocks(c->B, c->tile_bins), bins_partial_nv()),
                                      partials_need(push_blocks(c->B), 10)});
  if (bad(hipMalloc(&c->d_partials, c->partials_len * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_part_pts, partials_need(std::max(kRedBlocks, points_max_blocks()), 5) * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_mass_rows, (size_t)points_max_blocks() * sizeof(double2)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_part_push, partials_need(push_blocks(c->B), 10) * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_scalars, SC_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  if (bad(hipMemset(c->d_scalars, 0, SC_COUNT * sizeof(double)))) return GCS_ERR_HIP;
  // [0] k_scan's ticket, [1] k_pt's last-block fold ticket (each re-armed by its last block)
  if (bad(hipMalloc(&c->d_tickets, 4 * sizeof(uint32_t)))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_parse_flag, sizeof(uint32_t)))) return GCS_ERR_HIP;
  if (bad(hipMemset(c->d_tickets, 0, 4 * sizeof(uint32_t)))) return GCS_ERR_HIP;
  // the scan mirror (gcs_layout.h Mirror; k_final writes it, wait_mirror validates it): coherent, so
  // the device's stores go to host memory uncached instead of waiting in an XCD's L2
  if (bad(hipHostMalloc(&c->h_scalars, (MIR_WORDS + 4) * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent)))
    return GCS_ERR_HIP;
  memset(c->h_scalars, 0, (MIR_WORDS + 4) * sizeof(double));  // sequence 0: no scan's
  if (bad(hipHostGetDevicePointer((void**)&c->d_scalars_mirror, c->h_scalars, 0))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_err, 4 * sizeof(uint32_t)))) return GCS_ERR_HIP;
  if (bad(hipMemset(c->d_err, 0, 4 * sizeof(uint32_t)))) return GCS_ERR_HIP;
  if (bad(hipHostMalloc(&c->h_gate, 8 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent)))
    return GCS_ERR_HIP;
  for (int k = 0; k < 8; ++k) c->h_gate[k] = 0u;
  if (bad(hipHostGetDevicePointer((void**)&c->d_gate, c->h_gate, 0))) return GCS_ERR_HIP;
  if (bad(hipMalloc(&c->d_gate_xi, 8 * sizeof(double)))) return GCS_ERR_HIP;
  if (const char* g = getenv("GCSLAM_GATE")) c->gate_on = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_DEVICE_PREINT")) c->device_preint = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_DEVICE_IMU_ODOM")) c->device_imu_odom = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_PT_CLEAR")) c->pt_clear = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_BEGIN_MIRROR")) c->begin_mirror = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_LIVE_ASYNC")) c->live_async = atoi(g) != 0;
  if (const char* g = getenv("GCSLAM_BUDGET_BLOCKS")) c->budget_max = std::max(1, std::min(1024, atoi(g)));
  if (bad(hipHostMalloc(&c->h_preint_out, 16 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent)))
    return GCS_ERR_HIP;
  if (cfg->mode == GCS_MODE_SCALE) {
    if (bad(hipMalloc(&c->d_knn, B * c->K * sizeof(int)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_rknn_off, (B + 1) * sizeof(int)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_rknn, B * c->K * sizeof(int)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_keys, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_slots, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_sorted, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    c->n_counts_words = (int)B + 2 + scan_tiles(c->B);
    if (bad(hipMalloc(&c->d_counts, (size_t)c->n_counts_words * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMemset(c->d_counts, 0, (size_t)c->n_counts_words * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_starts, B * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_perm, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMalloc(&c->d_members, B * (size_t)c->capb * sizeof(uint32_t)))) return GCS_ERR_HIP;
    // zeroed so every slot holds a valid point index even when a failed scan leaves holes
    if (bad(hipMemset(c->d_perm, 0, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    if (bad(hipMemset(c->d_sorted, 0, cap * sizeof(uint32_t)))) return GCS_ERR_HIP;
    // bin flags, then one flag per k_bins_scale tile (both cleared by k_budget every scan)
    const size_t nflags = B + bins_scale_blocks(c->B, c->tile_bins);
    const size_t nflags16 = (nflags + 15) & ~(size_t)15;  // both buffers 16-B aligned (k_budget's clear)
    if (bad(hipMalloc(&c->d_flags_buf[0], 2 * nflags16))) return GCS_ERR_HIP;
    if (bad(hipMemset(c->d_flags_buf[0], 0, 2 * nflags16))) return GCS_ERR_HIP;
    c->d_flags_buf[1] = c->d_flags_buf[0] + nflags16;
    c->d_flags = c->d_flags_buf[0];
    // every tile starts dirty: the first scan writes all ScanBinStats rows and partial rows
    if (bad(hipMalloc(&c->d_tile_dirty, bins_scale_blocks(c->B, c->tile_bins)))) return GCS_ERR_HIP;
    if (bad(hipMemset(c->d_tile_dirty, 1, bins_scale_blocks(c->B, c->tile_bins)))) return GCS_ERR_HIP;
    {
      const int nt = bins_scale_blocks(c->B, c->tile_bins);
      const char* e = getenv("GCSLAM_TILE_ORDER");
      c->tile_order_on = nt > 2048 && !(e && atoi(e) == 0);
      const char* ep = getenv("GCSLAM_TILE_ORDER_PUSH");
      c->tile_order_defer = ep && atoi(ep) == 1;
      if (c->tile_order_on) {
        std::vector<int> ident(nt);
        for (int i = 0; i < nt; ++i) ident[i] = i;
        if (bad(hipMalloc(&c->d_tile_order, nt * sizeof(int)))) return GCS_ERR_HIP;
        if (bad(hipMemcpy(c->d_tile_order, ident.data(), nt * sizeof(int), hipMemcpyHostToDevice))) return GCS_ERR_HIP;
        if (bad(hipMalloc(&c->d_tile_work, nt * sizeof(uint32_t)))) return GCS_ERR_HIP;
        if (bad(hipMemset(c->d_tile_work, 0, nt * sizeof(uint32_t)))) return GCS_ERR_HIP;
      }
    }
    if (bad(hipMalloc(&c->d_bins_part, partials_need(bins_scale_blocks(c->B, c->tile_bins), bins_partial_nv()) * sizeof(double))))
      return GCS_ERR_HIP;
    // the split bin path's raw sums (128-bin tiles, GCSLAM_BINS_SPLIT=1; default: the fused phase D).
    // Same-box A/B at C3 (profiles/r06/split/): split 94 us (gather + finalize) against 84 us fused --
    // the 19 raw sums of every active bin written and read back (~2 x 90 MB) cost more than the
    // two-wave finalize they free
    static const bool split = [] {
      const char* e = getenv("GCSLAM_BINS_SPLIT");
      return e && atoi(e) == 1;
    }();
    if (split && c->tile_bins == 128 && bad(hipMalloc(&c->d_bins_raw, (size_t)19 * B * sizeof(double))))
      return GCS_ERR_HIP;
  } else {
    size_t nchunks = (cap + 255) / 256;
    if (bad(hipMalloc(&c->d_bin_partials, nchunks * 19 * B * sizeof(double)))) return GCS_ERR_HIP;
  }
  c->dirs_host.assign(B * 3, 0.0);
  atlas::fibonacci(c->B, c->dirs_host.data());
  if (int rc = upload_atlas(c)) {
    t_create_msg = "gcs_ctx_create: " + c->err;
    gcs_ctx_destroy(c);
    return rc;
  }
  // the hipMemset / hipMemcpy calls above ran on the null stream, which does not order the context's
  // non-blocking streams: they may still be in flight when hipMemset or a pageable hipMemcpy returns,
  // so the first kernels would race them (a 218 MB ScanBinStats clear overwrote rows the first C3
  // scan's bin kernel had written -- run-to-run differences of the zero bins' Sigma, tools/
  // determinism_check.py at C3).  Drain the null stream first.
  if (bad(hipStreamSynchronize(nullptr))) return GCS_ERR_HIP;
  if (bad(launch_map_derive(c->d_map, c->d_derived, c->B, c->d_partials, c->d_scalars, c->d_touched,
                            c->stream)))
    return GCS_ERR_HIP;
  if (bad(hipStreamSynchronize(c->stream))) return GCS_ERR_HIP;
  // identity prior (belief.py:320-358) and datasheet IW state
  memset(&c->belief, 0, sizeof(Belief));
  for (int i = 0; i < DZ; ++i) c->belief.L[i * DZ + i] = 1e-6;
  host::datasheet_iw_state(c->iw_nu, c->iw_Psi);
  host::process_noise_Q(c->iw_nu, c->iw_Psi, c->Q);
  host::datasheet_meas_iw_state(c->meas_nu, c->meas_Psi);
  *out = c;
  return GCS_OK;
}

int gcs_ctx_destroy(gcs_ctx* c) {
  if (!c) return GCS_OK;
  if (c->push_thread.joinable()) {
    (void)push_wait(c);
    {
      std::lock_guard<std::mutex> lk(c->push_mu);
      c->push_stop.store(true);
    }
    c->push_cv.notify_one();
    c->push_thread.join();
  }
  if (c->push_stream) (void)hipStreamSynchronize(c->push_stream);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* ptrs[] = {c->d_gate_xi, c->d_members, c->d_bin_dirs, c->d_knn, c->d_rknn_off, c->d_rknn, c->d_pools, c->d_pool_bound, c->d_recs, c->d_iz, c->d_live_p0, c->d_live_w, c->d_live_t, c->d_keys, c->d_slots,
                  c->d_sorted, c->d_nearest, c->d_counts, c->d_starts, c->d_perm, c->d_flags_buf[0], c->d_touched,
                  c->d_tile_dirty, c->d_tile_order, c->d_tile_work, c->d_bins_part, c->d_bins_raw, c->d_tickets,
                  c->d_bin_ref, c->d_tile_src_off, c->d_tile_src, c->d_rknn_local, c->d_part_pts, c->d_mass_rows, c->d_part_push, c->d_parse_flag,
                  c->d_scan, c->d_map, c->d_derived, c->d_bin_partials, c->d_partials, c->d_scalars};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_scalars) (void)hipHostFree(c->h_scalars);
  if (c->d_err) (void)hipFree(c->d_err);
  if (c->h_gate) (void)hipHostFree(c->h_gate);
  if (c->h_preint_in) (void)hipHostFree(c->h_preint_in);
  if (c->h_preint_out) (void)hipHostFree(c->h_preint_out);
  if (c->comm_stream) {
    (void)hipStreamSynchronize(c->comm_stream);
    (void)hipStreamDestroy(c->comm_stream);
  }
  if (c->d_pay_seq) (void)hipFree(c->d_pay_seq);
  if (c->h_payload) (void)hipHostFree(c->h_payload);
  if (c->h_psum) (void)hipHostFree(c->h_psum);
  if (c->d_payload) (void)hipFree(c->d_payload);
  if (c->d_payload_in) (void)hipFree(c->d_payload_in);
  for (int st = 0; st < kStages; ++st)
    for (hipEvent_t e : c->ev[st]) (void)hipEventDestroy(e);
  if (c->ev_push) (void)hipEventDestroy(c->ev_push);
  if (c->ev_stages) (void)hipEventDestroy(c->ev_stages);
  if (c->ev_preint) (void)hipEventDestroy(c->ev_preint);
  if (c->io_stream) {
    (void)hipStreamSynchronize(c->io_stream);
    (void)hipStreamDestroy(c->io_stream);
  }
  if (c->h_io_stage) (void)hipHostFree(c->h_io_stage);
  if (c->h_io_out) (void)hipHostFree(c->h_io_out);
  if (c->d_io_win) (void)hipFree(c->d_io_win);
  if (c->d_io_out) (void)hipFree(c->d_io_out);
  if (c->d_io_seq) (void)hipFree(c->d_io_seq);
  if (c->push_stream) (void)hipStreamDestroy(c->push_stream);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c->scan_st;
  delete c->live_out;
  delete c;
  return GCS_OK;
}

int gcs_ctx_set_stream(gcs_ctx* c, void* s) {
  if (!c) return GCS_ERR_ARG;
  if (int rc = push_wait(c)) return rc;
  HIPCHK(c, hipStreamSynchronize(c->push_stream));
  c->push_pending = false;
  if (c->stream) HIPCHK(c, hipStreamSynchronize(c->stream));  // work queued on the old stream completes first
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  c->stream = (hipStream_t)s;
  c->own_stream = false;
  return GCS_OK;
}

int gcs_ctx_synchronize(gcs_ctx* c) {
  if (!c) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GCS_OK;
}

int gcs_ctx_set_debug(gcs_ctx* c, int32_t key, int64_t value) {
  if (!c) return GCS_ERR_ARG;
  switch (key) {
    case GCS_DEBUG_SORTED_BUCKETS:
      c->direct_buckets = value == 0;
      return GCS_OK;
    case GCS_DEBUG_BUCKET_CAPACITY:
      if (value < 4 || value > c->capb || (value & 3)) return fail(c, GCS_ERR_ARG, "bucket capacity: a multiple of 4 in [4, 32]");
      c->capb_eff = (int)value;
      c->sorted_sticky = false;
      return GCS_OK;
    case GCS_DEBUG_SCAN_SPIN_LIMIT:
      if (value < 0 || value > 0xffffffffLL) return fail(c, GCS_ERR_ARG, "spin limit out of range");
      c->spin_limit = (uint32_t)value;
      return GCS_OK;
    case GCS_DEBUG_INJECT_SCAN_FAIL:
      c->inject_scan_fail = value ? 1 : 0;
      return GCS_OK;
    case GCS_DEBUG_POINT_KERNEL:
      c->legacy_points = value != 0;
      return GCS_OK;
    case GCS_DEBUG_DEVICE_PREINT:
      c->device_preint = value != 0;
      return GCS_OK;
    case GCS_DEBUG_DEVICE_IMU_ODOM:
      c->device_imu_odom = value != 0;
      return GCS_OK;
    case GCS_DEBUG_PT_CLEAR:
      c->pt_clear = value != 0;
      return GCS_OK;
    case GCS_DEBUG_LAUNCH_GATE:
      if (value < -1 || value > 1) return fail(c, GCS_ERR_ARG, "launch gate: -1, 0 or 1");
      c->gate_on = value != 0;
      c->gate_withhold = value < 0;
      return GCS_OK;
    case GCS_DEBUG_MIRROR_TORN:
      if (value < 0 || value > 10000) return fail(c, GCS_ERR_ARG, "mirror torn delay: 0..10000 us");
      c->mirror_torn = (int)value;
      return GCS_OK;
    case GCS_DEBUG_COMBINE_DELAY:
      if (value < 0 || value > 1000000) return fail(c, GCS_ERR_ARG, "combine delay: 0..1000000 us");
      c->combine_delay_us = (int)value;
      return GCS_OK;
    case GCS_DEBUG_SENDBUF:
      if (value < -1 || value > 1) return fail(c, GCS_ERR_ARG, "send buffer: -1 (by world size), 0 host, 1 device");
      c->sendbuf_mode = (int)value;
      return GCS_OK;
    default:
      return fail(c, GCS_ERR_ARG, "unknown debug key");
  }
}

int gcs_ctx_host_split(gcs_ctx* c, double* ms_sum, int64_t* n, int32_t reset) {
  if (!c || !ms_sum || !n) return GCS_ERR_ARG;
  memcpy(ms_sum, c->host_sums, sizeof(c->host_sums));
  n[0] = c->host_n[0];
  n[1] = c->host_n[1];
  if (reset) {
    memset(c->host_sums, 0, sizeof(c->host_sums));
    c->host_n[0] = c->host_n[1] = 0;
  }
  return GCS_OK;
}

int gcs_ctx_host_split_history(gcs_ctx* c, float* out, int32_t n_max, int32_t* n_out) {
  if (!c || !out || !n_out || n_max < 0) return GCS_ERR_ARG;
  const int64_t have = std::min<int64_t>(c->host_n[0], gcs_ctx::kHostHist);
  const int64_t n = std::min<int64_t>(have, n_max);
  for (int64_t i = 0; i < n; ++i) {  // the latest n scans, oldest first
    const int64_t k = c->host_n[0] - n + i;
    memcpy(out + 6 * i, c->host_hist.data() + (size_t)(k % gcs_ctx::kHostHist) * 6, 6 * sizeof(float));
  }
  *n_out = (int32_t)n;
  return GCS_OK;
}

int64_t gcs_ctx_worker_tid(gcs_ctx* c) { return c ? c->worker_tid.load() : 0; }

int gcs_ctx_mirror_stats(gcs_ctx* c, int64_t* out) {
  if (!c || !out) return GCS_ERR_ARG;
  out[0] = c->mirror_scans;
  out[1] = c->mirror_rereads;
  out[2] = c->mirror_syncs;
  out[3] = (int64_t)c->pay_seq;
  out[4] = c->pay_rereads;
  out[5] = c->pay_syncs;
  return GCS_OK;
}

namespace {
uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ULL) {
  const uint8_t* b = (const uint8_t*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ULL;
  return h;
}
// checksum of n bytes of device memory (synchronous copy)
int dev_fnv(gcs_ctx* c, const void* d, size_t n, uint64_t* out) {
  *out = 0;
  if (!d || !n) return GCS_OK;
  std::vector<uint8_t> h(n);
  HIPCHK(c, hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost));
  *out = fnv1a(h.data(), n);
  return GCS_OK;
}
}  // namespace

int gcs_debug_state_checksums(gcs_ctx* c, uint64_t* out) {
  if (!c || !out) return GCS_ERR_ARG;
  if (int rc = push_wait(c)) return rc;
  if (c->push_stream) HIPCHK(c, hipStreamSynchronize(c->push_stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t B = c->B;
  int rc = 0;
  if ((rc = dev_fnv(c, c->d_scan, B * SF_COUNT * sizeof(double), &out[0]))) return rc;
  if ((rc = dev_fnv(c, c->d_map, B * MF_COUNT * sizeof(double), &out[1]))) return rc;
  if ((rc = dev_fnv(c, c->d_derived, B * MD_COUNT * sizeof(double), &out[2]))) return rc;
  if ((rc = dev_fnv(c, c->d_touched, B, &out[3]))) return rc;
  const size_t nflags = c->d_flags_buf[0] ? 2 * ((B + bins_scale_blocks(c->B, c->tile_bins) + 15) & ~(size_t)15) : 0;
  if ((rc = dev_fnv(c, c->d_flags_buf[0], nflags, &out[4]))) return rc;
  const size_t npart = c->d_bins_part ? (size_t)bins_scale_blocks(c->B, c->tile_bins) * partial_stride(bins_partial_nv()) : 0;
  if ((rc = dev_fnv(c, c->d_bins_part, npart * sizeof(double), &out[5]))) return rc;
  if ((rc = dev_fnv(c, c->d_scalars, SC_COUNT * sizeof(double), &out[6]))) return rc;
  out[7] = fnv1a(c->h_scalars, SC_COUNT * sizeof(double));
  return GCS_OK;
}

int gcs_ctx_enable_timing(gcs_ctx* c, int32_t stage_mask) {
  if (!c) return GCS_ERR_ARG;
  if (stage_mask && c->ev[0].empty())
    for (int st = 0; st < kStages; ++st) {
      c->ev[st].resize(2 * gcs_ctx::kEvRing, nullptr);
      // timing only: no system-scope fence when a stamp completes (the fence's cache write-back and
      // invalidate measured ~8 us per stamped scan at C2, profiles/r05/stamp/)
      static const unsigned fl = [] {  // A/B knob GCSLAM_STAMP_EVENT=default|device (fence-free by default)
        const char* e = getenv("GCSLAM_STAMP_EVENT");
        if (e && strcmp(e, "default") == 0) return (unsigned)hipEventDefault;
        if (e && strcmp(e, "device") == 0) return (unsigned)hipEventReleaseToDevice;
        return (unsigned)hipEventDisableSystemFence;
      }();
      for (hipEvent_t& e : c->ev[st]) HIPCHK(c, hipEventCreateWithFlags(&e, fl));
    }
  c->timing_mask = (uint32_t)stage_mask;
  return GCS_OK;
}

int gcs_ctx_stage_times(gcs_ctx* c, double* ms_sum, int64_t* counts, int32_t reset) {
  if (!c) return GCS_ERR_ARG;
  if (int rc = push_wait(c)) return rc;  // the worker queues stage events of the scan front
  harvest(c);
  for (int st = 0; st < kStages; ++st) {
    if (ms_sum) ms_sum[st] = c->stage_ms_sum[st];
    if (counts) counts[st] = c->stage_count[st];
    if (reset) { c->stage_ms_sum[st] = 0.0; c->stage_count[st] = 0; }
  }
  return GCS_OK;
}

int gcs_ctx_set_atlas(gcs_ctx* c, const double* dirs) {
  if (!c || !dirs) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->dirs_host.assign(dirs, dirs + (size_t)c->B * 3);
  return upload_atlas(c);
}

int gcs_ctx_get_atlas(gcs_ctx* c, double* dirs, int32_t* knn) {
  if (!c) return GCS_ERR_ARG;
  if (dirs) memcpy(dirs, c->dirs_host.data(), c->dirs_host.size() * sizeof(double));
  if (knn && !c->knn_host.empty()) memcpy(knn, c->knn_host.data(), c->knn_host.size() * sizeof(int));
  return GCS_OK;
}

int gcs_ctx_set_belief(gcs_ctx* c, const gcs_belief* b) {
  if (!c || !b) return GCS_ERR_ARG;
  to_host_belief(*b, c->belief);
  c->prev_fac_valid = false;
  return GCS_OK;
}

int gcs_ctx_get_belief(gcs_ctx* c, gcs_belief* b) {
  if (!c || !b) return GCS_ERR_ARG;
  from_host_belief(c->belief, *b);
  return GCS_OK;
}

int gcs_ctx_set_map(gcs_ctx* c, const double* map) {
  if (!c || !map) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<double> dev((size_t)c->B * MF_COUNT);
  to_device_order(c, MF_COUNT, map, dev.data());
  HIPCHK(c, hipMemcpy(c->d_map, dev.data(), dev.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipStreamSynchronize(nullptr));  // a pageable copy may return before its DMA lands
  HIPCHK(c, launch_map_derive(c->d_map, c->d_derived, c->B, c->d_partials, c->d_scalars, c->d_touched,
                              c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GCS_OK;
}

int pull_rows(gcs_ctx* c, const double* dev_src, int F, double* ref_out) {
  if (int rc_ = join_push(c)) return rc_;
  std::vector<double> dev((size_t)c->B * F);
  HIPCHK(c, hipMemcpyAsync(dev.data(), dev_src, dev.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  to_reference_order(c, F, dev.data(), ref_out);
  return GCS_OK;
}

int gcs_ctx_get_map(gcs_ctx* c, double* map, double* derived) {
  if (!c) return GCS_ERR_ARG;
  if (map)
    if (int rc = pull_rows(c, c->d_map, MF_COUNT, map)) return rc;
  if (derived)
    if (int rc = pull_rows(c, c->d_derived, MD_COUNT, derived)) return rc;
  return GCS_OK;
}

int gcs_ctx_get_scan_stats(gcs_ctx* c, double* scan) {
  if (!c || !scan) return GCS_ERR_ARG;
  return pull_rows(c, c->d_scan, SF_COUNT, scan);
}

int gcs_ctx_get_bin_order(gcs_ctx* c, int32_t* order) {
  if (!c || !order) return GCS_ERR_ARG;
  for (int i = 0; i < c->B; ++i) order[i] = c->order[i];
  return GCS_OK;
}

int gcs_ctx_device_arrays(gcs_ctx* c, double** scan, double** map, double** derived) {
  if (!c) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the arrays are final when the pointers are handed out
  if (scan) *scan = c->d_scan;
  if (map) *map = c->d_map;
  if (derived) *derived = c->d_derived;
  return GCS_OK;
}

int gcs_ctx_set_iw_state(gcs_ctx* c, const double* nu, const double* Psi) {
  if (!c || !nu || !Psi) return GCS_ERR_ARG;
  memcpy(c->iw_nu, nu, sizeof(c->iw_nu));
  memcpy(c->iw_Psi, Psi, sizeof(c->iw_Psi));
  host::process_noise_Q(c->iw_nu, c->iw_Psi, c->Q);
  return GCS_OK;
}

int gcs_ctx_get_iw_state(gcs_ctx* c, double* nu, double* Psi, double* Q) {
  if (!c) return GCS_ERR_ARG;
  if (nu) memcpy(nu, c->iw_nu, sizeof(c->iw_nu));
  if (Psi) memcpy(Psi, c->iw_Psi, sizeof(c->iw_Psi));
  if (Q) memcpy(Q, c->Q, sizeof(c->Q));
  return GCS_OK;
}

int gcs_ctx_set_meas_iw_state(gcs_ctx* c, const double* nu, const double* Psi) {
  if (!c || !nu || !Psi) return GCS_ERR_ARG;
  memcpy(c->meas_nu, nu, sizeof(c->meas_nu));
  memcpy(c->meas_Psi, Psi, sizeof(c->meas_Psi));
  return GCS_OK;
}

int gcs_ctx_get_meas_iw_state(gcs_ctx* c, double* nu, double* Psi, double* cert2) {
  if (!c) return GCS_ERR_ARG;
  if (nu) memcpy(nu, c->meas_nu, sizeof(c->meas_nu));
  if (Psi) memcpy(Psi, c->meas_Psi, sizeof(c->meas_Psi));
  if (cert2) memcpy(cert2, c->meas_cert, sizeof(c->meas_cert));
  return GCS_OK;
}

// ---------------------------------------------------------------- per-operator entry points
namespace {
__global__ void k_ref_ids(const int* dev_ids, const int* bin_ref, int n, int* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = bin_ref[dev_ids[i]];
}
}  // namespace

int gcs_parse_pointcloud2(gcs_ctx* c, const void* data_dev, const gcs_pointcloud2_layout* L, double* points_dev,
                          double* t_dev, double* w_dev, uint8_t* ring_dev) {
  if (!c || !L || (L->n_points > 0 && (!data_dev || !points_dev || !t_dev || !w_dev))) return GCS_ERR_ARG;
  if (L->n_points < 0 || L->point_step < 1) return GCS_ERR_ARG;
  auto fits = [&](int off, int bytes) { return off >= 0 && off + bytes <= L->point_step; };
  auto width = [](int dt) { return dt <= 2 ? 1 : dt <= 4 ? 2 : dt <= 7 ? 4 : 8; };
  if (!fits(L->off_x, 4) || !fits(L->off_y, 4) || !fits(L->off_z, 4))
    return fail(c, GCS_ERR_ARG, "PointCloud2 x/y/z FLOAT32 fields outside point_step");
  if (L->ring_datatype < 1 || L->ring_datatype > 8 || !fits(L->off_ring, width(L->ring_datatype)))
    return fail(c, GCS_ERR_ARG, "PointCloud2 (VLP-16 layout) ring field missing or outside point_step");
  if (L->off_t >= 0 && (L->t_datatype < 1 || L->t_datatype > 8 || !fits(L->off_t, width(L->t_datatype))))
    return fail(c, GCS_ERR_ARG, "PointCloud2 time field outside point_step");
  if (int rc_ = join_push(c)) return rc_;
  ParseArgs a{};
  a.data = (const uint8_t*)data_dev;
  a.n = L->n_points;
  a.point_step = L->point_step;
  a.off_x = L->off_x; a.off_y = L->off_y; a.off_z = L->off_z;
  a.off_ring = L->off_ring; a.ring_datatype = L->ring_datatype;
  a.off_t = L->off_t; a.t_datatype = L->t_datatype;
  a.header_stamp = L->header_stamp_sec;
  memcpy(a.R, L->R_base_lidar, sizeof(a.R));
  memcpy(a.tb, L->t_base_lidar, sizeof(a.tb));
  a.points = points_dev; a.t = t_dev; a.w = w_dev; a.ring = ring_dev;
  a.ns_flag = c->d_parse_flag;
  HIPCHK(c, launch_parse(a, c->stream));
  return GCS_OK;
}

int gcs_point_stage(gcs_ctx* c, const void* xyz, int32_t point_step, const double* t, const double* w, int32_t n,
                    double t0, double t1, const double* xi, double* p0_dev, double* w_out_dev, double* w_budget_dev,
                    int32_t* nearest_dev, double* cert) {
  if (!c || !xi) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  c->budget_pending = false;  // a k_budget queued by a gcs_scan that failed later is stale
  int rc = stage_points(c, xyz, point_step, t, w, n, t0, t1, xi, p0_dev, w_out_dev, w_budget_dev, false, false,
                        c->d_iz);
  if (rc) return rc;
  c->iz_valid = true;
  if (nearest_dev) {  // reported in reference bin ids
    hipLaunchKernelGGL(k_ref_ids, dim3((c->cap + 255) / 256), dim3(256), 0, c->stream, (const int*)c->d_nearest,
                       (const int*)c->d_bin_ref, c->cap, nearest_dev);
    HIPCHK(c, hipGetLastError());
  }
  if ((rc = pull_scalars(c))) return rc;
  if (cert)
    for (int k = 0; k < 8; ++k) cert[k] = c->h_scalars[k];
  return GCS_OK;
}

namespace {
__global__ void k_materialize(const PointRec* recs, const double* iz, const int* nearest, const int* knn,
                              const double* bin_dirs, const int* bin_ref, int cap, int B, int K, bool scale, double ox,
                              double oy, double oz, double tau, int* ids, double* r) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const double izi = iz[i];
  double it = 1.0 / tau;
  if (scale) {
    // the 32-B record: d and m re-derived as the bin kernel's staging does (gcs_layout.h PointRec32)
    const double4 p = reinterpret_cast<const double4*>(recs)[i];
    const double o[3] = {ox, oy, oz};
    double d[3];
    ray_dir(p.x, p.y, p.z, o, d);
    const double* nb = bin_dirs + 4 * (size_t)nearest[i];  // d_nearest holds device ids
    const double m = dot3_exact(d[0], d[1], d[2], nb[0], nb[1], nb[2]);
    const int* row = knn + (size_t)nearest[i] * K;
    for (int k = 0; k < K; ++k) {
      const double* bd = bin_dirs + 4 * (size_t)row[k];
      double s = dot3_exact(d[0], d[1], d[2], bd[0], bd[1], bd[2]);
      if (ids) ids[(size_t)i * K + k] = bin_ref[row[k]];
      if (r) r[(size_t)i * K + k] = exp((s - m) * it) * izi;
    }
  } else {
    PointRec pr = recs[i];
    double d0 = pr.dx, d1 = pr.dy, d2 = pr.dz;
    for (int b = 0; b < B; ++b) {
      const double* bd = bin_dirs + 4 * (size_t)b;
      double s = dot3_exact(d0, d1, d2, bd[0], bd[1], bd[2]);
      if (r) r[(size_t)i * B + b] = exp((s - pr.m) * it) * izi;
    }
  }
}
}  // namespace

int gcs_bin_soft_assign(gcs_ctx* c, int32_t* ids, double* r) {
  if (!c) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  if (!c->iz_valid) return fail(c, GCS_ERR_STATE, "gcs_bin_soft_assign needs gcs_point_stage first");
  bool scale = c->cfg.mode == GCS_MODE_SCALE;
  hipLaunchKernelGGL(k_materialize, dim3((c->cap + 255) / 256), dim3(256), 0, c->stream, (const PointRec*)c->d_recs,
                     (const double*)c->d_iz, (const int*)c->d_nearest, (const int*)c->d_knn, (const double*)c->d_bin_dirs,
                     (const int*)c->d_bin_ref, c->cap, c->B, c->K,
                     scale, c->cfg.lidar_origin[0], c->cfg.lidar_origin[1], c->cfg.lidar_origin[2], c->cfg.tau, ids, r);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GCS_OK;
}

int gcs_scan_bin_moment_match(gcs_ctx* c, double* cert) {
  if (!c) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  int rc = stage_bins(c);
  if (rc) return rc;
  if ((rc = pull_scalars(c))) return rc;
  if ((rc = check_bucket_err(c))) return rc;
  if (cert)
    for (int k = 0; k < 5; ++k) cert[k] = c->h_scalars[SC_BIN_NSUM + k];
  return GCS_OK;
}

int gcs_matrix_fisher_rotation(gcs_ctx* c, double* mf) {
  if (!c) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  int rc = stage_mf(c);
  if (rc) return rc;
  if ((rc = pull_scalars(c))) return rc;
  if (mf) {
    int k = 0;
    for (int i = 0; i < 9; ++i) mf[k++] = c->h_scalars[SC_MF_H + i];
    mf[k++] = c->h_scalars[SC_MF_NEFF];
    for (int i = 0; i < 9; ++i) mf[k++] = c->h_scalars[SC_MF_MAPSCAT + i];
    mf[k++] = c->h_scalars[SC_MF_MAPND];
    mf[k++] = c->h_scalars[SC_MF_SCANN];
    for (int i = 0; i < 9; ++i) mf[k++] = c->h_scalars[SC_MF_R + i];
    double U[9], s[3], V[9];
    svd3(c->h_scalars + SC_MF_H, U, s, V);
    for (int i = 0; i < 3; ++i) mf[k++] = s[i];
    for (int i = 0; i < 9; ++i) mf[k++] = V[i];
  }
  return GCS_OK;
}

int gcs_planar_translation(gcs_ctx* c, const double* R_hat, double* pt) {
  if (!c || !R_hat) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  HIPCHK(c, hipMemcpyAsync(c->d_scalars + SC_MF_R, R_hat, 9 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  int rc = stage_pt(c);
  if (rc) return rc;
  if ((rc = pull_scalars(c))) return rc;
  if (pt) {
    for (int i = 0; i < 9; ++i) pt[i] = c->h_scalars[SC_PT_L + i];
    for (int i = 0; i < 3; ++i) pt[9 + i] = c->h_scalars[SC_PT_H + i];
    pt[12] = c->h_scalars[SC_PT_NEFF];
  }
  return GCS_OK;
}

int gcs_pushforward(gcs_ctx* c, const double* z_t, const double* Sig6, double gamma) {
  if (!c || !z_t || !Sig6) return GCS_ERR_ARG;
  if (int rc_ = join_push(c)) return rc_;
  int rc = stage_push(c, z_t, Sig6, gamma, c->stream, c->d_partials, c->d_flags);
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GCS_OK;
}

// ---------------------------------------------------------------- the per-scan pipeline
// gcs_scan runs the whole bin-path scan in one call.  gcs_scan_begin / gcs_scan_finish split the
// same steps around the caller's LiDAR evidence for the live primitive path (pipeline.py:778-1011:
// surfels, recency, view, association and visual pose evidence run between them on the device
// through their own entry points).  The pieces below are shared, so both forms run one code path.

namespace {

// LiDAR evidence of step 9 and its certificate terms: the bin path's MF + planar blocks, or the live
// path's visual pose evidence (the caller's gcs_lidar_evidence)
struct LidarTerms {
  double L[DZ * DZ] = {}, h[DZ] = {};
  double ev_ess = 0.0;  // support.ess_total of aggregate(LiDAR certs)
  double ev_nll = 0.0;  // mismatch.nll_per_ess of aggregate(LiDAR certs)
};

// 1 (launch), 2 PredictDiffusion, 3 IMU membership window + preintegration -> deskew twist
// (pipeline.py:399-483)
// Device preintegration (k_preint): the window is staged in pinned memory (the trailing run of
// repeated stamps -- the zero padding -- trimmed to its first sample: its steps are exact identities
// and only their weights enter ess), the kernel is queued on the scan stream, and the point stage
// reads the twist from the device word.  st.xi / st.pre arrive after the scan's sync (finish_preint).
int launch_device_preint(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_state& st) {
  const int m = in->imu_len;
  int r = m - 1;
  while (r > 0 && in->imu_stamps[r - 1] == in->imu_stamps[r]) --r;
  const int me = r + 1;
  // the previous k_preint may still read the window (a scan that failed after queuing it): wait for it
  // before the window is rewritten or freed
  if (c->ev_preint_pending) {
    HIPCHK(c, hipEventSynchronize(c->ev_preint));
    c->ev_preint_pending = false;
  }
  if (c->preint_in_cap < 7 * (int64_t)me) {
    if (c->h_preint_in) (void)hipHostFree(c->h_preint_in);
    c->h_preint_in = nullptr;
    c->preint_in_cap = 0;
    const int64_t cap = 7 * (int64_t)std::max(me, 512);
    HIPCHK(c, hipHostMalloc(&c->h_preint_in, cap * sizeof(double), hipHostMallocMapped));
    c->preint_in_cap = cap;
  }
  double* hin = c->h_preint_in;
  memcpy(hin, in->imu_stamps, me * sizeof(double));
  memcpy(hin + me, in->imu_gyro, 3 * me * sizeof(double));
  memcpy(hin + 4 * me, in->imu_accel, 3 * me * sizeof(double));
  PreintArgs a{};
  a.imu = hin;
  a.m = me;
  a.n_tail = m - me;
  a.tail_stamp = in->imu_stamps[r];
  a.t0 = in->scan_start_time;
  a.t1 = in->scan_end_time;
  a.sigma = st.sigma_warp;
  for (int k = 0; k < 3; ++k) {
    a.rotvec[k] = st.pose0[3 + k];
    a.gb[k] = st.mu_inc[9 + k];
    a.ab[k] = st.mu_inc[12 + k];
    a.g[k] = c->grav[k];
  }
  a.rotation_only = c->cfg.deskew_rotation_only ? 1 : 0;
  a.xi_dev = c->d_gate_xi;
  a.host_out = c->h_preint_out;
  HIPCHK(c, launch_preint(a, c->stream));
  if (!c->ev_preint) HIPCHK(c, hipEventCreateWithFlags(&c->ev_preint, hipEventDisableTiming));
  HIPCHK(c, hipEventRecord(c->ev_preint, c->stream));
  c->ev_preint_pending = true;
  c->preint_pending = true;
  c->preint_host_pending = true;
  return GCS_OK;
}

// after the scan's sync: the device preintegration's record into the scan state
void finish_preint(gcs_ctx* c, gcs_scan_state& st) {
  if (!c->preint_host_pending) return;
  c->preint_host_pending = false;
  // k_preint's record is read after its own completion event (the mirror that precedes this call is
  // a later kernel's; the event makes the order explicit and costs a query once it has fired)
  if (c->ev_preint_pending) {
    if (hipEventQuery(c->ev_preint) != hipSuccess) (void)hipEventSynchronize(c->ev_preint);
    c->ev_preint_pending = false;
  }
  const volatile double* o = c->h_preint_out;
  for (int k = 0; k < 6; ++k) st.xi[k] = o[k];
  st.pre.ess = o[6];
  for (int k = 0; k < 6; ++k) st.pre.delta_pose[k] = o[7 + k];
  for (int k = 0; k < 3; ++k) st.pre.delta_v[k] = o[13 + k];
  st.cert[10] = st.pre.ess;
}

int scan_prologue(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_state& st, bool budget = true) {
  st.T0 = clk::now();
  c->preint_pending = c->preint_host_pending = false;  // (a failed scan may have left them set)
  if (budget) {  // (the pre-launched front queues k_budget itself)
    c->budget_pending = false;
    if (int rc0 = stage_budget(c, in->weights_dev, in->n_points, true,
                               c->self_budget && c->cfg.mode == GCS_MODE_SCALE))  // runs during the prologue
      return rc0;
  }
  const double* Q = in->Q ? in->Q : c->Q;
  double* cert = st.cert;
  memset(cert, 0, sizeof(st.cert));
  st.Tsum = 0.0;
  if (in->L_ext) memcpy(st.Lext, in->L_ext, sizeof(st.Lext)); else memset(st.Lext, 0, sizeof(st.Lext));
  if (in->h_ext) memcpy(st.hext, in->h_ext, sizeof(st.hext)); else memset(st.hext, 0, sizeof(st.hext));
  // 2 PredictDiffusion
  st.prev = c->belief;
  double pinfl[3];
  host::predict_diffusion(st.prev, Q, in->dt_sec, st.pred, pinfl, st.mu_prev,
                          c->prev_fac_valid ? &c->prev_fac : nullptr, c->prev_cov);
  cert[6] = pinfl[0]; cert[7] = pinfl[1]; cert[8] = pinfl[2];
  st.Tsum += trig(pinfl[0], pinfl[1], 0, 0, 0, pinfl[2], 1, 1, 1);
  st.Tp = clk::now();
  // 3 IMU membership window + preintegration -> deskew twist (pipeline.py:432-483)
  host::SpdFactor fpred;  // one factor of the predicted information for every solve below
  host::spd_factor_lifted(DZ, st.pred.L, kEpsLift, fpred);
  double e15[DZ] = {}, col15[DZ];
  e15[15] = 1.0;
  host::spd_factor_solve(fpred, e15, col15);  // column 15 of the predicted covariance
  st.sigma_warp = std::max(sqrt(col15[15]), 0.01);
  cert[38] = st.sigma_warp;
  host::spd_factor_solve(fpred, st.pred.h, st.mu_inc);
  host::world_pose_from_increment(st.prev, st.mu_prev, st.pose0);
  if (budget && c->device_preint) {  // k_preint on the stream ahead of the point stage
    if (int rc = launch_device_preint(c, in, st)) return rc;
    st.T1 = clk::now();
    return GCS_OK;
  }
  std::vector<double>& wimu = c->wimu;
  wimu.resize(in->imu_len);
  for (int i = 0; i < in->imu_len; ++i)  // a repeated stamp (the window's zero padding) reuses its value
    wimu[i] = i > 0 && in->imu_stamps[i] == in->imu_stamps[i - 1]
                  ? wimu[i - 1]
                  : smooth_window(in->imu_stamps[i], in->scan_start_time, in->scan_end_time, st.sigma_warp);
  host::preintegrate_imu(in->imu_len, in->imu_stamps, in->imu_gyro, in->imu_accel, wimu.data(), st.pose0 + 3,
                         st.mu_inc + 9, st.mu_inc + 12, c->grav, st.pre);
  host::se3_log(st.pre.delta_pose, st.xi);
  if (c->cfg.deskew_rotation_only) st.xi[0] = st.xi[1] = st.xi[2] = 0.0;
  cert[10] = st.pre.ess;
  st.T1 = clk::now();
  return GCS_OK;
}

// The IMU / odometry branch on the device (k_imu_odom): the window and the small inputs packed into pinned
// memory, one H2D copy and the one-workgroup kernel on the context's io_stream (beside the bin path's
// kernels); finish_imu_odom_dev reads the stamped record (wait_stamped: sequence + checksum).
int launch_imu_odom_dev(gcs_ctx* c, const gcs_imu_odom_inputs& in) {
  const int m = in.m;
  if (m < 2 || m > kImuOdomMaxM)
    return fail(c, GCS_ERR_ARG, "device IMU/odometry branch: the window holds 2 .. " + std::to_string(kImuOdomMaxM) +
                                    " samples");
  const size_t words = (size_t)8 * kImuOdomMaxM + kIoSmallLen;
  if (!c->d_io_win) {
    HIPCHK(c, hipHostMalloc(&c->h_io_stage, words * sizeof(double), hipHostMallocDefault));
    HIPCHK(c, hipMalloc(&c->d_io_win, words * sizeof(double)));
    HIPCHK(c, hipMalloc(&c->d_io_out, (kIoOutWords + kImuOdomStatWords) * sizeof(double)));
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    HIPCHK(c, hipHostMalloc(&c->h_io_out, (kIoOutWords + 2) * sizeof(double), fl));
    memset(c->h_io_out, 0, (kIoOutWords + 2) * sizeof(double));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->dh_io_out, c->h_io_out, 0));
    HIPCHK(c, hipMalloc(&c->d_io_seq, sizeof(uint64_t)));
    HIPCHK(c, hipMemset(c->d_io_seq, 0, sizeof(uint64_t)));
    HIPCHK(c, hipStreamSynchronize(nullptr));  // (the null stream does not order io_stream)
    HIPCHK(c, hipStreamCreateWithFlags(&c->io_stream, hipStreamNonBlocking));
    c->io_seq = 0;
  }
  // the previous call's copy out of the staging buffer has completed (its record was read after it; a
  // scan that failed before reading it leaves it pending: drain the stream first)
  if (c->io_dev_pending) {
    HIPCHK(c, hipStreamSynchronize(c->io_stream));
    c->io_dev_pending = false;
  }
  double* w = c->h_io_stage;
  memcpy(w, in.stamps, m * sizeof(double));
  memcpy(w + m, in.gyro, 3 * m * sizeof(double));
  memcpy(w + 4 * m, in.accel, 3 * m * sizeof(double));
  memcpy(w + 7 * m, in.w_int, m * sizeof(double));
  double* sm = w + 8 * m;
  memcpy(sm + kIoPose0, in.pose0, 6 * sizeof(double));
  memcpy(sm + kIoPosePred, in.pose_pred, 6 * sizeof(double));
  memcpy(sm + kIoMuPrev, in.mu_prev, DZ * sizeof(double));
  memcpy(sm + kIoMuInc, in.mu_inc, DZ * sizeof(double));
  memcpy(sm + kIoGravity, in.gravity_W, 3 * sizeof(double));
  memcpy(sm + kIoSigmaG, in.Sigma_g, 9 * sizeof(double));
  memcpy(sm + kIoSigmaA, in.Sigma_a, 9 * sizeof(double));
  memcpy(sm + kIoOdomPose, in.odom_pose, 6 * sizeof(double));
  memcpy(sm + kIoOdomCov, in.odom_cov_se3, 36 * sizeof(double));
  memcpy(sm + kIoOdomTwist, in.odom_twist, 6 * sizeof(double));
  memcpy(sm + kIoOdomTwistCov, in.odom_twist_cov, 36 * sizeof(double));
  HIPCHK(c, hipMemcpyAsync(c->d_io_win, w, ((size_t)8 * m + kIoSmallLen) * sizeof(double), hipMemcpyHostToDevice,
                           c->io_stream));
  ImuOdomDevArgs a{};
  a.win = c->d_io_win;
  a.m = m;
  a.t_last_scan = in.t_last_scan;
  a.t_scan = in.t_scan;
  a.dt_sec = in.dt_sec;
  a.planar_z_ref = in.planar_z_ref;
  a.planar_z_sigma = in.planar_z_sigma;
  a.planar_vz_sigma = in.planar_vz_sigma;
  a.out = c->d_io_out;
  a.host = c->dh_io_out;
  a.dseq = c->d_io_seq;
  HIPCHK(c, launch_imu_odom(a, c->io_stream));
  ++c->io_seq;
  c->io_dev_pending = true;
  return GCS_OK;
}

int finish_imu_odom_dev(gcs_ctx* c, host::ImuOdomOut& io, double* extra) {
  if (!c->io_dev_pending) return GCS_OK;
  c->io_dev_pending = false;
  if (int rc = wait_stamped(c, c->h_io_out, kIoOutWords, c->io_seq, c->io_stream, &c->io_rereads, &c->io_syncs,
                            "device IMU/odometry evidence"))
    return rc;
  memcpy(&io, c->h_io_out, sizeof(host::ImuOdomOut));
  if (extra) memcpy(extra, c->h_io_out + kIoOutWords - 5, 5 * sizeof(double));
  for (int k = 0; k < DZ * DZ; ++k)
    if (!std::isfinite(io.L[k])) return fail(c, GCS_ERR_NONFINITE, "IMU/odometry evidence contains NaN");
  return GCS_OK;
}

// 13 measurement-noise IW statistics over the scan-to-scan IMU window (pipeline.py:448-453, 522-566)
// and 9 the IMU/odometry evidence branch (pipeline.py:595-776), computed while the device stages
// run (they need no device result); padded samples (stamp <= 0) carry weight 0 (the reference's
// valid mask).  w_imu_int unmasked as in the reference (padding gets the 1e-12 floor); the IW
// statistics mask stamps <= 0 themselves.
int scan_imu_odom(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_state& st, gcs_scan_outputs* out) {
  std::vector<double>& wint = c->wint;
  wint.resize(in->imu_len);
  for (int i = 0; i < in->imu_len; ++i)
    wint[i] = i > 0 && in->imu_stamps[i] == in->imu_stamps[i - 1]
                  ? wint[i - 1]
                  : smooth_window(in->imu_stamps[i], in->t_last_scan, in->t_scan, st.sigma_warp);
  host::imu_meas_iw_suffstats(in->imu_len, in->imu_stamps, in->imu_gyro, in->imu_accel, wint.data(), st.mu_inc + 9,
                              st.mu_inc + 12, st.pose0 + 3, c->grav, out->iw_meas_dPsi, out->iw_meas_dnu);
  host::world_pose_from_increment(st.pred, st.mu_inc, st.pose_pred);
  st.use_io = c->cfg.use_imu_odom != 0;
  memset(st.io_extra, 0, sizeof(st.io_extra));
  if (st.use_io) {
    if (in->imu_len < 2) return fail(c, GCS_ERR_ARG, "IMU window of at least 2 samples required");
    double Sg[9], Sa[9];
    if (in->Sigma_g) memcpy(Sg, in->Sigma_g, sizeof(Sg)); else host::meas_iw_mode(c->meas_nu, c->meas_Psi, 0, Sg);
    if (in->Sigma_a) memcpy(Sa, in->Sigma_a, sizeof(Sa)); else host::meas_iw_mode(c->meas_nu, c->meas_Psi, 1, Sa);
    gcs_imu_odom_inputs ii{};
    ii.m = in->imu_len;
    ii.stamps = in->imu_stamps; ii.gyro = in->imu_gyro; ii.accel = in->imu_accel; ii.w_int = wint.data();
    ii.t_last_scan = in->t_last_scan; ii.t_scan = in->t_scan; ii.dt_sec = in->dt_sec;
    ii.pose0 = st.pose0; ii.pose_pred = st.pose_pred; ii.mu_prev = st.mu_prev; ii.mu_inc = st.mu_inc;
    ii.gravity_W = c->grav;
    ii.Sigma_g = Sg; ii.Sigma_a = Sa;
    ii.odom_pose = in->odom_pose ? in->odom_pose : kZero6;
    ii.odom_cov_se3 = in->odom_cov_se3 ? in->odom_cov_se3 : kBigCov6.v;
    ii.odom_twist = in->odom_twist ? in->odom_twist : kZero6;
    ii.odom_twist_cov = in->odom_twist_cov ? in->odom_twist_cov : kBigCov6.v;
    ii.planar_z_ref = c->cfg.planar_z_ref; ii.planar_z_sigma = c->cfg.planar_z_sigma;
    ii.planar_vz_sigma = c->cfg.planar_vz_sigma;
    if (c->device_imu_odom) {  // k_imu_odom beside the device stages; finish_imu_odom_dev reads it
      if (int rc = launch_imu_odom_dev(c, ii)) return rc;
    } else {
      run_imu_odom(ii, c->io, st.io_extra);
      for (int k = 0; k < DZ * DZ; ++k)
        if (!std::isfinite(c->io.L[k])) return fail(c, GCS_ERR_NONFINITE, "IMU/odometry evidence contains NaN");
    }
  } else {
    memset(c->io.L, 0, sizeof(c->io.L));
    memset(c->io.h, 0, sizeof(c->io.h));
  }
  for (int k = 0; k < 27; ++k)
    if (!std::isfinite(out->iw_meas_dPsi[k])) return fail(c, GCS_ERR_NONFINITE, "omega_avg / IMU residuals non-finite");
  memcpy(c->last_meas_dPsi, out->iw_meas_dPsi, sizeof(c->last_meas_dPsi));
  memcpy(c->last_meas_dnu, out->iw_meas_dnu, sizeof(c->last_meas_dnu));
  return GCS_OK;
}

// budget (point_budget.py:182-212) and deskew certificates from the point stage's scalars
int scan_point_certs(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_state& st) {
  const double* S = c->h_scalars;
  double* cert = st.cert;
  double mass_in = S[SC_MASS_IN];
  double budget_ess = 1.0 / (S[SC_BUDGET_W2] + (double)c->cap * kEpsMass);
  double budget_mer = kEpsMass / (mass_in + kEpsMass);
  cert[0] = budget_ess;
  cert[1] = std::min(1.0, c->cap / (in->n_points + kEpsMass));
  cert[2] = budget_mer;
  cert[3] = mass_in;
  cert[4] = c->last_n_sel;
  cert[5] = c->last_stride;
  st.Tsum += budget_mer;
  if (!std::isfinite(mass_in)) return fail(c, GCS_ERR_NONFINITE, "non-finite point weights");
  cert[9] = S[SC_DESKEW_WOUT] / (S[SC_DESKEW_WIN] + kEpsMass);
  return GCS_OK;
}

// soft assign, moment match, 7 MatrixFisherRotation and 8 PlanarTranslationEvidence tails
// (binning.py:71-75,118-125,193-196; matrix_fisher_evidence.py:240-256,310-394,565-671) and the
// combined 22-D LiDAR evidence (build_combined_lidar_evidence_22d, :729-756)
void scan_bin_lidar(gcs_ctx* c, gcs_scan_state& st, LidarTerms& lt, gcs_scan_outputs* out) {
  const double* S = c->h_scalars;
  double* cert = st.cert;
  double avg_ent = S[SC_ENTROPY] / ((double)c->cap + kEpsMass);
  cert[11] = avg_ent;
  cert[12] = exp(avg_ent);
  cert[13] = S[SC_MAXRESP];
  double mm_ess = S[SC_BIN_NSUM] * S[SC_BIN_NSUM] / (S[SC_BIN_N2SUM] + kEpsMass);
  cert[14] = mm_ess;
  cert[15] = S[SC_BIN_SUPP] / (double)c->B;
  cert[16] = S[SC_BIN_PSD];
  cert[17] = S[SC_BIN_EPSR];
  st.Tsum += S[SC_BIN_PSD] + S[SC_BIN_EPSR];
  double R_pred[9];
  so3_exp(st.pose_pred + 3, R_pred);
  double Umf[9], sv[3], V[9];
  svd3(S + SC_MF_H, Umf, sv, V);  // L_rot needs s and V (host, same 3x3 SVD code as the device)
  const double* Rmf = S + SC_MF_R;
  double Lrot_raw[9], Lrot[9];
  double dg[3] = {sv[1] + sv[2], sv[0] + sv[2], sv[0] + sv[1]};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Lrot_raw[3 * i + j] = V[3 * i] * dg[0] * V[3 * j] + V[3 * i + 1] * dg[1] * V[3 * j + 1] + V[3 * i + 2] * dg[2] * V[3 * j + 2];
  double mf_delta = host::psd_project(3, Lrot_raw, kEpsPsd, Lrot);
  double Rerr[9], drot[3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rerr[3 * i + j] = R_pred[i] * Rmf[j] + R_pred[3 + i] * Rmf[3 + j] + R_pred[6 + i] * Rmf[6 + j];
  so3_log(Rerr, drot);
  double hrot[3];
  for (int i = 0; i < 3; ++i) hrot[i] = Lrot[3 * i] * drot[0] + Lrot[3 * i + 1] * drot[1] + Lrot[3 * i + 2] * drot[2];
  double mf_neff = S[SC_MF_NEFF];
  double mf_mer = kEpsMass / (mf_neff + kEpsMass);
  cert[18] = mf_delta; cert[19] = mf_mer; cert[20] = mf_neff;
  cert[21] = sv[0]; cert[22] = sv[1]; cert[23] = sv[2];
  cert[24] = 0.5 * (drot[0] * hrot[0] + drot[1] * hrot[1] + drot[2] * hrot[2]);
  st.Tsum += mf_delta + mf_mer;
  double Tmap[9], ev[3], Vt[9];
  double nd = S[SC_MF_MAPND] + kEpsMass;
  for (int k = 0; k < 9; ++k) Tmap[k] = S[SC_MF_MAPSCAT + k] / nd;
  double Tsym[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Tsym[3 * i + j] = 0.5 * (Tmap[3 * i + j] + Tmap[3 * j + i]);
  host::jacobi_eigh(3, Tsym, ev, Vt);
  std::sort(ev, ev + 3);
  double lam1 = std::max(ev[2], kEpsMass), lam3 = std::max(ev[0], 0.0);
  double zs = lam3 / lam1;
  double Lf[9], hf[3], Lreg[9], twls[3];
  for (int k = 0; k < 9; ++k) Lf[k] = S[SC_PT_L + k];
  for (int k = 0; k < 3; ++k) hf[k] = S[SC_PT_H + k];
  memcpy(Lreg, Lf, sizeof(Lreg));
  Lreg[0] += kEpsMass; Lreg[4] += kEpsMass; Lreg[8] += kEpsMass;
  host::solve3(Lreg, hf, twls);
  double mask[3] = {1.0, 1.0, zs};
  double Ltr_raw[9], Ltr[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ltr_raw[3 * i + j] = Lf[3 * i + j] * mask[i] * mask[j];
  double pt_delta = host::psd_project(3, Ltr_raw, kEpsPsd, Ltr);
  double dtr[3] = {twls[0] - st.pose_pred[0], twls[1] - st.pose_pred[1], twls[2] - st.pose_pred[2]};
  double htr[3];
  for (int i = 0; i < 3; ++i) htr[i] = Ltr[3 * i] * dtr[0] + Ltr[3 * i + 1] * dtr[1] + Ltr[3 * i + 2] * dtr[2];
  double pt_neff = S[SC_PT_NEFF];
  double pt_mer = kEpsMass / (pt_neff + kEpsMass);
  cert[25] = pt_delta; cert[26] = pt_mer; cert[27] = pt_neff; cert[28] = zs;
  cert[29] = 0.5 * (dtr[0] * htr[0] + dtr[1] * htr[1] + dtr[2] * htr[2]);
  st.Tsum += pt_delta + pt_mer;
  memcpy(out->R_mf, Rmf, sizeof(out->R_mf));
  memcpy(out->t_wls, twls, sizeof(out->t_wls));
  memset(lt.L, 0, sizeof(lt.L));
  memset(lt.h, 0, sizeof(lt.h));
  for (int i = 0; i < 3; ++i) {
    lt.h[i] = htr[i];
    lt.h[3 + i] = hrot[i];
    for (int j = 0; j < 3; ++j) {
      lt.L[i * DZ + j] = Ltr[3 * i + j];
      lt.L[(3 + i) * DZ + 3 + j] = Lrot[3 * i + j];
    }
  }
  // aggregate of the LiDAR certs [deskew, soft assign, moment match, MF, planar] (pipeline.py:1057)
  lt.ev_ess = (st.pre.ess + cert[12] + mm_ess + 0.0 + 0.0) / 5.0;
  lt.ev_nll = cert[24] / (mf_neff + kEpsMass) + cert[29] / (pt_neff + kEpsMass);
}

// 9 evidence sum + power tempering + excitation scaling, 10 FusionScaleFromCertificates, 11
// InfoFusionAdditive, 12 PoseUpdateFrobeniusRecompose, process IW statistics, 13 the bin map's
// PoseCovInflationPushforward (push: the bin path; the live path's map update is the caller's step
// 12b), 14 AnchorDriftUpdate (pipeline.py:1038-1230, 1494-1502)
int scan_tail(gcs_ctx* c, gcs_scan_state& st, const LidarTerms& lt, gcs_scan_outputs* out, bool push) {
  if (int rc = finish_imu_odom_dev(c, c->io, st.io_extra)) return rc;  // (the device branch, when it ran)
  double* cert = st.cert;
  Belief& pred = st.pred;
  double Lraw[DZ * DZ], hraw[DZ];
  for (int i = 0; i < DZ * DZ; ++i) Lraw[i] = st.Lext[i] + c->io.L[i];
  for (int i = 0; i < DZ; ++i) hraw[i] = st.hext[i] + c->io.h[i];
  memcpy(out->L_imu_odom, c->io.L, sizeof(out->L_imu_odom));
  {
    const host::EvCert* cs[11] = {&c->io.odom, &c->io.imu, &c->io.dep, &c->io.gyro, &c->io.preint, &c->io.planar,
                                  &c->io.vz, &c->io.vel, &c->io.wz, &c->io.kin, &c->io.odom_dep};
    for (int k = 0; k < 11; ++k) {
      double* o = out->imu_odom_certs + 7 * k;
      if (!st.use_io) { for (int j = 0; j < 7; ++j) o[j] = 0.0; continue; }
      o[0] = cs[k]->ess; o[1] = cs[k]->support; o[2] = cs[k]->nll; o[3] = cs[k]->lift; o[4] = cs[k]->psd;
      o[5] = cs[k]->mer; o[6] = cs[k]->trust_alpha;
    }
  }
  memcpy(out->h_imu_odom, c->io.h, sizeof(out->h_imu_odom));
  if (st.use_io) st.Tsum += c->io.trigger;  // the eleven IMU/odometry certs are in all_certs (pipeline.py:964)
  for (int i = 0; i < DZ * DZ; ++i) Lraw[i] += lt.L[i];
  for (int i = 0; i < DZ; ++i) hraw[i] += lt.h[i];
  auto nrm = [](const double* v, int n, int stride) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += v[i * stride] * v[i * stride];
    return sqrt(s);
  };
  double dt_pose = nrm(Lraw + 15 * DZ, 6, 1) + nrm(Lraw + 15, 6, DZ);
  double dt_vel = nrm(Lraw + 15 * DZ + 6, 3, 1) + nrm(Lraw + 6 * DZ + 15, 3, DZ);
  double dt_asym = fabs(dt_vel - dt_pose) / (dt_vel + dt_pose + kEpsMass);
  dt_asym = std::min(std::max(dt_asym, 0.0), 1.0);
  double z_to_xy = fabs(Lraw[2 * DZ + 2]) / (0.5 * (fabs(Lraw[0]) + fabs(Lraw[DZ + 1])) + kEpsMass);
  // combined evidence cert (pipeline.py:1057-1067): aggregate([aggregate(LiDAR certs), odom, imu,
  // gyro]); ExcitationCert is never filled -> 0
  const double ess_total = st.use_io ? (lt.ev_ess + c->io.odom.ess + c->io.imu.ess + c->io.gyro.ess) / 4.0 : lt.ev_ess;
  const double nll_total = st.use_io ? lt.ev_nll + c->io.odom.nll + c->io.imu.nll + c->io.gyro.nll : lt.ev_nll;
  double ess_to_exc = ess_total / (0.0 + kEpsMass);
  double s_z = z_to_xy / (z_to_xy + 1.0);
  double s_exc = 1.0 / (1.0 + ess_to_exc / 50.0);
  double sc = std::min(std::max(dt_asym * s_z * s_exc, 0.0), 1.0);
  double beta = 0.25 + 0.75 * sc;
  beta = std::min(std::max(beta, 0.25), 1.0);
  cert[30] = beta; cert[39] = dt_asym; cert[40] = z_to_xy;
  st.Tsum += fabs(1.0 - beta);
  double Lev[DZ * DZ], hev[DZ];
  for (int i = 0; i < DZ * DZ; ++i) Lev[i] = beta * Lraw[i];
  for (int i = 0; i < DZ; ++i) hev[i] = beta * hraw[i];
  // excitation prior scaling (excitation.py:15-64)
  double e_dt = Lev[15 * DZ + 15], e_ex = 0.0, p_dt = pred.L[15 * DZ + 15], p_ex = 0.0;
  for (int i = 16; i < 22; ++i) { e_ex += Lev[i * DZ + i]; p_ex += pred.L[i * DZ + i]; }
  double s_dt = e_dt / (e_dt + p_dt + 1e-12), s_ex = e_ex / (e_ex + p_ex + 1e-12);
  double a_dt = 1.0 - s_dt, a_ex = 1.0 - s_ex;
  for (int j = 0; j < DZ; ++j) { pred.L[15 * DZ + j] *= a_dt; }
  for (int i = 0; i < DZ; ++i) { pred.L[i * DZ + 15] *= a_dt; }
  pred.h[15] *= a_dt;
  for (int r = 16; r < 22; ++r) for (int j = 0; j < DZ; ++j) pred.L[r * DZ + j] *= a_ex;
  for (int i = 0; i < DZ; ++i) for (int r = 16; r < 22; ++r) pred.L[i * DZ + r] *= a_ex;
  for (int r = 16; r < 22; ++r) pred.h[r] *= a_ex;
  cert[31] = s_dt; cert[32] = s_ex;
  st.Tsum += fabs(s_dt) + fabs(s_ex);
  // 10 FusionScaleFromCertificates on the pose-6 conditioning of the tempered evidence
  // (pipeline.py:1150-1192, fusion.py:46-142)
  double c6min, c6max, c6cond, c6nn, quality;
  host::pose6_conditioning(Lev, &c6min, &c6max, &c6cond, &c6nn);
  const double alpha = host::fusion_scale(c6cond, ess_total, nll_total, beta, dt_asym, z_to_xy, 0.0, c->cfg.alpha_min,
                                          c->cfg.alpha_max, c->cfg.c0_cond, &quality);
  cert[33] = alpha;
  st.Tsum += fabs(1.0 - alpha);
  cert[42] = st.use_io ? c->io.trigger : 0.0;
  cert[43] = st.io_extra[0];         // dt_int
  cert[44] = st.io_extra[1];         // dt_imu
  cert[45] = c->io.transport_sigma;
  cert[46] = c->io.kappa;            // IMU gravity vMF kappa
  cert[47] = c->io.imu_scale;        // imu_dependence_inflation scale
  cert[48] = c->io.odom_scale;       // odom_dependence_inflation scale
  cert[49] = c6cond;                 // pose-6 conditioning
  cert[50] = c6nn;
  cert[51] = ess_total;
  cert[52] = quality;
  cert[53] = c->io.ess_weighted;
  cert[54] = c->io.mean_reliability;
  cert[55] = nll_total;
  cert[56] = st.io_extra[4];         // omega_avg z
  // 11 InfoFusionAdditive (fusion.py:186-191)
  Belief post = pred;
  double Lsum[DZ * DZ];
  for (int i = 0; i < DZ * DZ; ++i) Lsum[i] = pred.L[i] + alpha * Lev[i];
  double fdelta = host::psd_project(DZ, Lsum, kEpsPsd, post.L);
  for (int i = 0; i < DZ; ++i) post.h[i] = pred.h[i] + alpha * hev[i];
  cert[34] = fdelta;
  st.Tsum += fdelta;
  // 12 PoseUpdateFrobeniusRecompose (recompose.py:94-205)
  cert[35] = st.Tsum;
  double fs = st.Tsum / (st.Tsum + 1.0);
  cert[36] = fs;
  double dz[DZ], corr[6], dpc[6], e6[6];
  host::SpdFactor fpost;  // recompose keeps L: one factor serves post, rec and the anchor drift
  host::spd_factor_lifted(DZ, post.L, kEpsLift, fpost);
  host::spd_factor_solve(fpost, post.h, dz);
  host::bch3(post.z_lin, dz, corr);
  for (int i = 0; i < 6; ++i) dpc[i] = dz[i] + fs * corr[i];
  Belief rec = post;
  se3_exp(dpc, e6);
  host::se3_compose(post.X_anchor, e6, rec.X_anchor);
  for (int i = 0; i < 6; ++i) rec.z_lin[i] = post.z_lin[i] - dpc[i];
  for (int i = 0; i < DZ; ++i) {
    double s = 0.0;
    for (int j = 0; j < 6; ++j) s += post.L[i * DZ + j] * dpc[j];
    rec.h[i] = post.h[i] - s;
  }
  double mu_pred_x[DZ], mu_rec[DZ], covr[DZ * DZ];
  host::spd_solve_lifted(DZ, pred.L, pred.h, kEpsLift, mu_pred_x);  // pred after excitation scaling
  host::spd_factor_solve(fpost, rec.h, mu_rec);
  host::spd_factor_inverse(fpost, covr);
  host::process_iw_suffstats_from(mu_pred_x, mu_rec, covr, out->iw_process_dPsi, out->iw_process_dnu);
  memcpy(c->last_dPsi, out->iw_process_dPsi, sizeof(c->last_dPsi));
  memcpy(c->last_dnu, out->iw_process_dnu, sizeof(c->last_dnu));
  // 13 PoseCovInflationPushforward with z_t (pipeline.py:1244-1246)
  double z_t[6], Sig6[36];
  host::world_pose_from_increment(rec, mu_rec, z_t);
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) Sig6[6 * i + j] = covr[i * DZ + j];
  memcpy(c->map_rec, st.xi, 6 * sizeof(double));
  memcpy(c->map_rec + 6, z_t, 6 * sizeof(double));
  memcpy(c->map_rec + 12, Sig6, 36 * sizeof(double));
  auto Tq = clk::now();
  if (push && c->map_mode != GCS_MAP_FOLLOW)  // a follower's map takes the lead's update (gcs_map_follow)
    if (int rc = submit_push(c, z_t, Sig6, c->cfg.forgetting_factor, c->push_main ? c->stream : c->push_stream,
                             c->d_part_push))
      return rc;
  auto Tr = clk::now();
  memcpy(out->z_t, z_t, sizeof(out->z_t));
  // 14 AnchorDriftUpdate (anchor_drift.py:93-191)
  const double* dz2 = mu_rec;  // mean_increment(rec)
  double dm = sqrt(dz2[0] * dz2[0] + dz2[1] * dz2[1] + dz2[2] * dz2[2]);
  double dr = sqrt(dz2[3] * dz2[3] + dz2[4] * dz2[4] + dz2[5] * dz2[5]);
  double rho = std::min(std::max(std::max(dm / 0.5, dr / 0.2), 0.0), 1.0);
  Belief fin = rec;
  double sd[6];
  for (int i = 0; i < 6; ++i) sd[i] = rho * dz2[i];
  se3_exp(sd, e6);
  host::se3_compose(rec.X_anchor, e6, fin.X_anchor);
  for (int i = 0; i < DZ; ++i) fin.z_lin[i] = (1.0 - rho) * dz2[i];
  for (int i = 0; i < DZ; ++i) {
    double s = 0.0;
    for (int j = 0; j < DZ; ++j) s += rec.L[i * DZ + j] * fin.z_lin[j];
    fin.h[i] = s;
  }
  cert[37] = rho;
  for (int i = 0; i < DZ * DZ; ++i) out->L_evidence[i] = Lev[i];
  for (int i = 0; i < DZ; ++i) out->h_evidence[i] = hev[i];
  for (int i = 0; i < DZ; ++i)
    if (!std::isfinite(fin.h[i])) return fail(c, GCS_ERR_NONFINITE, "non-finite belief after scan");
  c->belief = fin;
  c->prev_fac = fpost;  // fin.L == post.L: recompose and the anchor drift change h, not L
  memcpy(c->prev_cov, covr, sizeof(c->prev_cov));
  c->prev_fac_valid = true;
  from_host_belief(fin, out->belief);
  c->have_last = true;
  memcpy(out->cert, cert, sizeof(out->cert));
  auto T3 = clk::now();
  out->stage_ms[0] = ms_between(st.T0, st.T1);
  out->stage_ms[1] = ms_between(st.T1, st.T2);
  out->stage_ms[2] = ms_between(st.T2, T3);
  out->stage_ms[3] = ms_between(st.T0, T3);
  out->stage_ms[4] = ms_between(st.T0, st.Tp);  // of [0]: budget launch + PredictDiffusion
  out->stage_ms[5] = ms_between(st.T1, st.Ts);  // of [1]: the device stages' launch calls
  out->stage_ms[6] = ms_between(st.T2, Tq);     // of [2]: tail numerics up to the pushforward launch
  out->stage_ms[7] = ms_between(Tq, Tr);        // of [2]: pushforward launch calls
  for (int k = 0; k < 8; ++k) c->host_sums[k] += out->stage_ms[k];
  float* hh = c->host_hist.data() + (size_t)(c->host_n[0] % gcs_ctx::kHostHist) * 6;
  for (int k = 0; k < 4; ++k) hh[k] = (float)out->stage_ms[k];
  hh[4] = hh[5] = 0.0f;
  ++c->host_n[0];
  return GCS_OK;
}

}  // namespace

int gcs_scan(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_outputs* out) {
  if (!c || !in || !out) return fail(c, GCS_ERR_ARG, "null argument");
  if (in->imu_len < 1 || !in->imu_stamps || !in->imu_gyro || !in->imu_accel) return fail(c, GCS_ERR_ARG, "IMU window required");
  c->live_pending = false;
  // this scan's device error words arrive with its own mirror: none of an earlier, failed call's stays
  memset(c->h_err, 0, sizeof(c->h_err));
  // direct buckets for this call's stages (scale mode, unless a bucket overflowed before)
  c->use_direct = c->cfg.mode == GCS_MODE_SCALE && c->direct_buckets && !c->sorted_sticky && c->d_members;
  struct DirectOff {
    gcs_ctx* c;
    ~DirectOff() { c->use_direct = false; }  // per-operator entry points always take the sorted path
  } direct_off{c};
  gcs_scan_state& st = *c->scan_st;
  int rc = 0;
  // pre-launched front (direct buckets, worker thread, budget / point stages not event-timed): the
  // device stages are queued now and the point kernel waits on the device for the prologue's twist
  const uint32_t front_timed = (1u << ST_BUDGET) | (1u << ST_POINTS);
  if (c->gate_on && c->push_async && c->use_direct && c->h_gate && !(c->timing_mask & front_timed)) {
    GateGuard guard{c};
    ++c->gate_seq;
    st.T0 = clk::now();
    if ((rc = submit_front(c, in, c->gate_seq))) return rc;
    if ((rc = scan_prologue(c, in, st, /*budget=*/false))) return rc;
    if (!c->gate_withhold) open_gate(c, st.xi);
    guard.open = true;
    st.Ts = clk::now();
    if ((rc = scan_imu_odom(c, in, st, out))) return rc;
    guard.joined = true;
    if ((rc = push_wait(c))) return rc;  // the front's launch calls (and their errors)
    if ((rc = wait_mirror(c))) return rc;
    if (c->h_err[3]) {
      c->h_err[3] = 0u;
      return fail(c, GCS_ERR_HIP, "k_points: launch gate not opened within its timeout");
    }
  } else {
    if ((rc = scan_prologue(c, in, st))) return rc;
    // 1,3,4-6 device: budget, deskew, soft assign, moment match; 7,8 MF + planar reductions
    rc = stage_points(c, in->xyz_dev, in->point_step, in->timestamps_dev, in->weights_dev, in->n_points,
                      in->scan_start_time, in->scan_end_time, st.xi, nullptr, nullptr, nullptr, /*fold_later=*/true,
                      in->xyz_format == 1);
    if (rc) return rc;
    if (int rc_ = join_push(c)) return rc_;  // the bin kernel reads the map the previous scan's pushforward wrote
    if ((rc = stage_bins(c))) return rc;  // scale mode: Matrix-Fisher reduction + R_mf fused in
    if (c->cfg.mode != GCS_MODE_SCALE && (rc = stage_mf(c))) return rc;
    if ((rc = stage_pt(c, /*to_host=*/true, /*clear_next=*/true))) return rc;
    if ((rc = stage_tile_order(c))) return rc;
    st.Ts = clk::now();
    if ((rc = scan_imu_odom(c, in, st, out))) return rc;
    if ((rc = wait_mirror(c))) return rc;  // the PT fold has written the scalars to h_scalars
    finish_preint(c, st);
  }
  if ((rc = check_bucket_err(c))) return rc;
  bool redone = false;
  if (c->use_direct && c->h_err[2]) {
    // a bucket exceeded the direct rows: redo the device stages with the sorted bucketing (same
    // flags buffer: the previous scan's pushforward may still read the other), and keep it
    c->h_err[2] = 0u;
    c->sorted_sticky = true;
    c->use_direct = false;
    redone = true;
    if ((rc = stage_budget(c, in->weights_dev, in->n_points, /*toggle=*/false,
                           c->self_budget && c->cfg.mode == GCS_MODE_SCALE)))
      return rc;
    if ((rc = stage_points(c, in->xyz_dev, in->point_step, in->timestamps_dev, in->weights_dev, in->n_points,
                           in->scan_start_time, in->scan_end_time, st.xi, nullptr, nullptr, nullptr, true,
                           in->xyz_format == 1)))
      return rc;
    if ((rc = stage_bins(c))) return rc;
    if ((rc = stage_pt(c, /*to_host=*/true, /*clear_next=*/true))) return rc;
    if ((rc = stage_tile_order(c))) return rc;
    if ((rc = wait_mirror(c))) return rc;
    if ((rc = check_bucket_err(c))) return rc;
  }
  st.cert[41] = c->h_err[1] ? 1.0 : 0.0;  // a bucket above the ranking capacity took the compaction path
  st.cert[57] = redone ? 1.0 : 0.0;       // a bucket overflowed the direct rows: redone sorted
  c->h_err[1] = 0u;
  st.T2 = clk::now();
  if ((rc = scan_point_certs(c, in, st))) return rc;
  LidarTerms lt;
  scan_bin_lidar(c, st, lt, out);
  return scan_tail(c, st, lt, out, /*push=*/true);
}

// ---------------------------------------------------------------- live primitive path: begin / finish
int gcs_scan_begin(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_begin_outputs* out) {
  if (!c || !in || !out) return fail(c, GCS_ERR_ARG, "null argument");
  if (in->imu_len < 1 || !in->imu_stamps || !in->imu_gyro || !in->imu_accel) return fail(c, GCS_ERR_ARG, "IMU window required");
  c->live_pending = false;
  // this scan's device error words arrive with its own mirror: none of an earlier, failed call's stays
  memset(c->h_err, 0, sizeof(c->h_err));
  c->use_direct = false;
  gcs_scan_state& st = *c->scan_st;
  if (int rc = scan_prologue(c, in, st)) return rc;
  // 1 + 3 on the device: budget gather, deskew, window weights (no soft assign, no bins)
  double* p0 = out->points_dev ? out->points_dev : c->d_live_p0;
  double* tt = out->timestamps_dev ? out->timestamps_dev : c->d_live_t;
  double* ww = out->weights_dev ? out->weights_dev : c->d_live_w;
  int rc = stage_points(c, in->xyz_dev, in->point_step, in->timestamps_dev, in->weights_dev, in->n_points,
                        in->scan_start_time, in->scan_end_time, st.xi, p0, ww, nullptr,
                        /*fold_later=*/false, in->xyz_format == 1, nullptr, /*deskew_only=*/true, tt,
                        /*to_host=*/c->begin_mirror);
  if (rc) return rc;
  st.Ts = clk::now();
  if ((rc = scan_imu_odom(c, in, st, c->live_out))) return rc;
  if (c->begin_mirror) {  // the point fold's stamped mirror: its scalars and error words, no D2H copies
    if ((rc = wait_mirror(c))) return rc;
  } else {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = pull_scalars(c))) return rc;
  }
  finish_preint(c, st);
  st.T2 = clk::now();
  if ((rc = scan_point_certs(c, in, st))) return rc;
  if ((rc = finish_imu_odom_dev(c, c->io, st.io_extra))) return rc;  // (the device branch, when it ran)
  // the map branch's linearisation point: z_lin = solve(PSD(L_pred + L_imu_odom), h_pred + h_imu_odom),
  // its pose block (pipeline.py:751-755); read by visual_pose_evidence as [t, rotvec] (:318-322)
  double Lf[DZ * DZ], Lp[DZ * DZ], hf[DZ], zl[DZ];
  for (int i = 0; i < DZ * DZ; ++i) Lf[i] = st.pred.L[i] + c->io.L[i];
  for (int i = 0; i < DZ; ++i) hf[i] = st.pred.h[i] + c->io.h[i];
  host::psd_project(DZ, Lf, kEpsPsd, Lp);
  host::spd_solve_lifted(DZ, Lp, hf, kEpsLift, zl);
  memcpy(out->z_lin_pose, zl, sizeof(out->z_lin_pose));
  memcpy(out->pose_pred, st.pose_pred, sizeof(out->pose_pred));
  out->n_points = c->cap;
  out->n_selected = c->last_n_sel;
  out->points_dev = p0;
  out->timestamps_dev = tt;
  out->weights_dev = ww;
  out->deskew_ess = st.pre.ess;  // the deskew certificate's support (deskew_constant_twist.py:95-104)
  out->deskew_support = st.cert[9];
  memcpy(out->cert, st.cert, sizeof(out->cert));
  c->live_pending = true;
  return GCS_OK;
}

int gcs_scan_finish(gcs_ctx* c, const gcs_lidar_evidence* ev, gcs_scan_outputs* out) {
  if (!c || !ev || !out || !ev->L_lidar || !ev->h_lidar) return fail(c, GCS_ERR_ARG, "null argument");
  if (!c->live_pending) return fail(c, GCS_ERR_STATE, "gcs_scan_finish without gcs_scan_begin");
  c->live_pending = false;
  gcs_scan_state& st = *c->scan_st;
  memcpy(out->iw_meas_dPsi, c->live_out->iw_meas_dPsi, sizeof(out->iw_meas_dPsi));
  memcpy(out->iw_meas_dnu, c->live_out->iw_meas_dnu, sizeof(out->iw_meas_dnu));
  memset(out->R_mf, 0, sizeof(out->R_mf));
  memset(out->t_wls, 0, sizeof(out->t_wls));
  LidarTerms lt;
  for (int i = 0; i < DZ * DZ; ++i) {
    lt.L[i] = ev->L_lidar[i];
    if (!std::isfinite(lt.L[i])) return fail(c, GCS_ERR_NONFINITE, "L_lidar contains NaN");
  }
  memcpy(lt.h, ev->h_lidar, sizeof(lt.h));
  // aggregate(LiDAR certs) = aggregate([deskew, surfel, association, visual]) (pipeline.py:1049-1056):
  // mean ess_total, summed nll_per_ess (the deskew cert has neither a mismatch term)
  lt.ev_ess = (st.pre.ess + ev->ess_sum) / (1.0 + (double)ev->n_certs);
  lt.ev_nll = ev->nll_sum;
  st.Tsum += ev->trigger_sum;  // the map branch's and the visual certs in all_certs (pipeline.py:964-1002)
  st.cert[58] = ev->trigger_sum;
  return scan_tail(c, st, lt, out, /*push=*/false);
}

// ---------------------------------------------------------------- live primitive path: one call
namespace {
// tiling.py:167-209 (ma_hex_stencil_tile_ids): the packed ids of the hex disk (radius_xy, axial order
// sorted by (q, r)) x the z slab (radius_z, outer loop) around the cell of center; -1 past cap
int ma_hex_stencil(const double* ctr, double h_tile, int rxy, int rz, int64_t* out, int cap) {
#pragma clang fp contract(off)
  const double x = ctr[0], y = ctr[1], z = ctr[2];
  const double h = std::max(h_tile, 1e-12);
  const int64_t c1 = (int64_t)std::floor(x / h);
  const int64_t c2 = (int64_t)std::floor((x * 0.5 + y * (std::sqrt(3.0) * 0.5)) / h);
  const int64_t cz = (int64_t)std::floor(z / h);
  constexpr int64_t bias = int64_t(1) << 20, mask = (int64_t(1) << 21) - 1;
  auto pack = [&](int64_t a, int64_t b, int64_t c) {
    return (((a + bias) & mask) << 42) | (((b + bias) & mask) << 21) | ((c + bias) & mask);
  };
  if (rxy < 0 || rz < 0) return -1;
  int n = 0;
  for (int dz = -rz; dz <= rz; ++dz)
    for (int q = -rxy; q <= rxy; ++q)
      for (int r = std::max(-rxy, -q - rxy); r <= std::min(rxy, -q + rxy); ++r) {
        if (n >= cap) return -1;
        out[n++] = pack(c1 + q, c2 + r, cz + dz);
      }
  return n;
}

int sub_fail(gcs_ctx* c, int rc, const char* what, const char* msg) {
  return fail(c, rc, std::string(what) + ": " + (msg ? msg : ""));
}
}  // namespace

int gcs_ma_hex_stencil(const double* center3, double h_tile, int32_t radius_xy, int32_t radius_z, int64_t* out,
                       int32_t cap) {
  if (!center3 || !out || cap < 0) return GCS_ERR_ARG;
  const int n = ma_hex_stencil(center3, h_tile, radius_xy, radius_z, out, cap);
  return n < 0 ? GCS_ERR_ARG : n;
}

int gcs_live_scan(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_begin_outputs* bo, const gcs_live_args* a,
                  gcs_live_outputs* lo, gcs_scan_outputs* out) {
  if (!c || !bo || !a || !lo || !out) return fail(c, GCS_ERR_ARG, "null argument");
  if (!a->surfels || !a->assoc || !a->map || !a->assoc_cfg || !a->update_cfg || !a->surfel_out || !a->view ||
      !a->view_tile_ids_dev || !a->assoc_out || !a->vpe_out || !a->lidar_sources_dev ||
      !a->assoc_out->candidate_pool_indices || !a->assoc_out->candidate_tile_ids || !a->assoc_out->candidate_slots)
    return fail(c, GCS_ERR_ARG, "gcs_live_scan: missing context, output or association array");
  if (a->n_tiles < 0 || a->n_free < 0 || (a->n_tiles > 0 && (!a->tile_ids || !a->tile_slots)) ||
      (a->n_free > 0 && !a->free_slots))
    return fail(c, GCS_ERR_ARG, "gcs_live_scan: bad tile directory");
  if (c->live_map) return fail(c, GCS_ERR_STATE, "gcs_live_scan: the previous scan's step 12b was not collected");
  memset(lo, 0, sizeof(*lo));
  const clk::time_point t_in = clk::now();
  auto mark = [&](int k) { lo->phase_us[k] = 1e3 * ms_between(t_in, clk::now()); };
  int rc;
  if (in) {
    if ((rc = gcs_scan_begin(c, in, bo))) return rc;
  } else if (!c->live_pending) {
    return fail(c, GCS_ERR_STATE, "gcs_live_scan without gcs_scan_begin");
  }
  mark(0);
  // the scan's tiles around the predicted position (pipeline.py:783-797)
  const int na = ma_hex_stencil(bo->pose_pred, a->h_tile, a->r_active_xy, a->r_active_z, lo->active_ids,
                                GCS_LIVE_MAX_TILES);
  const int ns = ma_hex_stencil(bo->pose_pred, a->h_tile, a->r_stencil_xy, a->r_stencil_z, lo->stencil_ids,
                                GCS_LIVE_MAX_TILES);
  if (na < 0 || ns < 0) return fail(c, GCS_ERR_ARG, "gcs_live_scan: a stencil exceeds GCS_LIVE_MAX_TILES tiles");
  if (na != a->n_active_expected)
    return fail(c, GCS_ERR_ARG, "active tile stencil size mismatch: expected N_ACTIVE_TILES=" +
                                    std::to_string(a->n_active_expected) + ", got " + std::to_string(na));
  if (ns != a->n_stencil_expected)
    return fail(c, GCS_ERR_ARG, "stencil tile size mismatch: expected N_STENCIL_TILES=" +
                                    std::to_string(a->n_stencil_expected) + ", got " + std::to_string(ns));
  lo->n_active = na;
  lo->n_stencil = ns;
  // the AtlasMap directory: present tiles for the recency inflation and the view, new tiles for step 12b
  std::vector<std::pair<int64_t, int32_t>> dir((size_t)a->n_tiles);
  for (int i = 0; i < a->n_tiles; ++i) dir[i] = {a->tile_ids[i], a->tile_slots[i]};
  std::sort(dir.begin(), dir.end());
  auto find = [&](int64_t id) -> int32_t {
    auto it = std::lower_bound(dir.begin(), dir.end(), std::make_pair(id, (int32_t)INT32_MIN));
    return (it != dir.end() && it->first == id) ? it->second : -1;
  };
  int32_t rec[GCS_LIVE_MAX_TILES], vs[GCS_LIVE_MAX_TILES];
  int nrec = 0;
  for (int i = 0; i < na; ++i) {
    const int32_t s = find(lo->active_ids[i]);
    if (s >= 0) rec[nrec++] = s;
  }
  lo->n_present_active = nrec;
  for (int i = 0; i < ns; ++i) vs[i] = find(lo->stencil_ids[i]);  // -1: viewed as empty
  gcs_surfel_ctx* sf = a->surfels;
  gcs_assoc_ctx* as = a->assoc;
  gcs_pmap* pm = a->map;
  hipStream_t s = c->stream;
  if (live::surfel_bind_stream(sf, s)) return sub_fail(c, GCS_ERR_HIP, "surfels", gcs_surfel_last_error(sf));
  if (live::assoc_bind_stream(as, s)) return sub_fail(c, GCS_ERR_HIP, "association", gcs_assoc_last_error(as));
  if (live::pmap_bind_stream(pm, s)) return sub_fail(c, GCS_ERR_HIP, "map", gcs_pmap_last_error(pm));
  int32_t clear[GCS_LIVE_MAX_TILES];
  int ncl = 0, nfree = 0;
  for (int i = 0; i < na; ++i) {
    int32_t s = find(lo->active_ids[i]);
    if (s < 0) {  // AtlasMap.index(create=True): the first free slot (stencil ids are distinct)
      if (nfree >= a->n_free) {
        lo->n_created = 0;  // nothing was created: the caller adopts no tile
        return fail(c, GCS_ERR_STATE, "primitive map holds max_tiles tiles");
      }
      s = a->free_slots[nfree++];
      if (a->slot_written && a->slot_written[s]) clear[ncl++] = s;
      lo->created_ids[lo->n_created] = lo->active_ids[i];
      lo->created_slots[lo->n_created++] = s;
    }
    lo->active_slots[i] = s;
  }
  // a created tile on a written slot is cleared now, ahead of every launch that can fail: the caller
  // adopts the created tiles (slot written, count 0) whatever the call returns, so their device
  // storage must be empty from here on (index(create=True) of the per-operator path clears at once too)
  for (int k = 0; k < ncl; ++k)
    if ((rc = live::pmap_clear_tile_launch(pm, clear[k]))) {
      lo->n_created = 0;
      return sub_fail(c, rc, "gcs_pmap_clear_tile", gcs_pmap_last_error(pm));
    }
  ncl = 0;
  if (a->zero_dev && a->zero_bytes > 0) HIPCHK(c, hipMemsetAsync(a->zero_dev, 0, (size_t)a->zero_bytes, s));
  // surfels of the deskewed points (pipeline.py:778-782), the batch's LiDAR sources set on its valid
  // rows; the launches behind them read the surfel count on the device (no host wait here)
  gcs_surfel_outputs sfo = *a->surfel_out;
  sfo.sources = a->lidar_sources_dev;
  if ((rc = live::surfel_launch(sf, a->points_dev, a->timestamps_dev, a->weights_dev, a->n_points, &sfo)))
    return sub_fail(c, rc, "gcs_extract_lidar_surfels", gcs_surfel_last_error(sf));
  const int32_t* nv_dev = live::surfel_nvalid_dev(sf);
  mark(1);
  // recency inflation of the active tiles the map holds, then the view over the stencil (:800-815)
  if ((rc = live::pmap_recency_launch(pm, rec, nrec, a->scan_seq, a->recency_lambda, a->recency_min_scale)))
    return sub_fail(c, rc, "gcs_pmap_recency_inflate", gcs_pmap_last_error(pm));
  if ((rc = live::pmap_view_launch(pm, vs, lo->stencil_ids, ns, a->m_tile_view, a->eps_lift, a->eps_mass, a->view)))
    return sub_fail(c, rc, "gcs_pmap_extract_view", gcs_pmap_last_error(pm));
  if ((rc = live::pmap_copy_staged_ids(pm, a->view_tile_ids_dev, ns)))
    return sub_fail(c, rc, "gcs_pmap_extract_view", gcs_pmap_last_error(pm));
  // OT association (:816-878)
  gcs_assoc_meas m = a->meas;
  m.n_valid = 0;  // n_camera_valid (0: a LiDAR-only batch) + n_lidar_valid: read on the device (nv_dev)
  gcs_assoc_view v{};
  v.tile_ids = a->view_tile_ids_dev;
  v.n_tiles = ns;
  v.m_tile_view = a->m_tile_view;
  v.positions = a->view->positions;
  v.directions = a->view->directions;
  v.kappas = a->view->kappas;
  v.valid_mask = a->view->valid_mask;
  v.last_supported_scan_seq = a->view->last_supported_scan_seq;
  v.candidate_tile_ids = a->view->candidate_tile_ids;
  v.candidate_slots = a->view->candidate_slots;
  gcs_assoc_outputs* ao = a->assoc_out;
  if ((rc = live::assoc_launch(as, a->assoc_cfg, &m, &v, ao, nv_dev)))
    return sub_fail(c, rc, "gcs_associate_primitives_ot", gcs_assoc_last_error(as));
  // visual pose evidence at z_lin_pose (:980-1010); one wait for the surfels, the recency, the view, the
  // association and the pose evidence
  gcs_assoc_view vv{};
  vv.positions = v.positions;
  vv.directions = v.directions;
  vv.kappas = v.kappas;
  vv.valid_mask = v.valid_mask;
  vv.n_tiles = 1;
  vv.m_tile_view = ns * a->m_tile_view;
  gcs_vpe_outputs* vo = a->vpe_out;
  if ((rc = live::vpe_launch(as, &m, &vv, ao->responsibilities, ao->candidate_pool_indices, ao->row_masses,
                             a->assoc_cfg->k_assoc, bo->z_lin_pose, a->eps_lift, a->eps_mass, nv_dev)))
    return sub_fail(c, rc, "gcs_visual_pose_evidence", gcs_assoc_last_error(as));
  mark(3);
  HIPCHK(c, hipStreamSynchronize(s));
  live::surfel_collect(sf, &sfo);
  gcs_surfel_outputs* so = a->surfel_out;
  memcpy(so->center, sfo.center, sizeof(so->center));
  so->n_valid = sfo.n_valid;
  memcpy(so->cert, sfo.cert, sizeof(so->cert));
  const int nv = so->n_valid;
  live::assoc_collect(as, ao);
  live::pmap_recency_collect(pm, nrec, lo->recency_stats);
  live::vpe_collect(as, nv, a->assoc_cfg->k_assoc, bo->z_lin_pose, a->eps_lift, vo);
  mark(4);
  // the finish: trigger magnitudes of the surfel (identity influence), recency (exact), association
  // (mass_epsilon_ratio unless exact) and visual (lift_strength = eps_lift unless exact) certs; ESS of
  // the surfel (n_valid), association and visual certs; no mismatch terms (pipeline.py:1049-1056,1211)
  const double t_assoc = ao->exact ? 0.0 : ao->cert[GCS_ASSOC_CERT_MASS_EPS_RATIO];
  const double t_vis = vo->exact ? 0.0 : a->eps_lift;
  const double e_assoc = ao->exact ? 0.0 : ao->cert[GCS_ASSOC_CERT_ESS];
  const double e_vis = vo->exact ? 0.0 : vo->ess_total;
  gcs_lidar_evidence ev{};
  ev.L_lidar = vo->L_pose;
  ev.h_lidar = vo->h_pose;
  ev.trigger_sum = ((0.0 + 0.0) + t_assoc) + t_vis;  // the per-cert sums in the pipeline's order
  ev.ess_sum = ((0.0 + (double)nv) + e_assoc) + e_vis;
  ev.n_certs = 3;
  ev.nll_sum = 0.0;
  lo->trigger_sum = ev.trigger_sum;
  lo->ess_sum = ev.ess_sum;
  if ((rc = gcs_scan_finish(c, &ev, out))) return rc;
  mark(5);
  // step 12b at z_t over the active tiles (:1232-1492); new tiles on written slots start cleared
  if (c->live_async && c->push_async) {  // the launch calls on the worker: the caller builds its results meanwhile
    if (!c->push_thread.joinable()) c->push_thread = std::thread(push_worker, c);
    gcs_ctx::PushJob& j = claim_job(c);
    j.kind = 3;
    j.pm = pm;
    j.n12 = na;
    j.ncl = ncl;
    memcpy(j.tiles12, lo->active_slots, sizeof(int32_t) * na);
    memcpy(j.tids12, lo->active_ids, sizeof(int64_t) * na);
    memcpy(j.clear12, clear, sizeof(int32_t) * ncl);
    memcpy(j.z_t, out->z_t, sizeof(j.z_t));
    j.ts12 = a->timestamp;
    j.seq12 = a->scan_seq;
    j.next12 = a->next_global_id;
    j.ucfg = *a->update_cfg;
    gcs_pmap_update_inputs& ui = j.uin;
    ui = gcs_pmap_update_inputs{};
    ui.Lambdas = m.Lambdas;
    ui.thetas = m.thetas;
    ui.etas = m.etas;
    ui.weights = m.weights;
    ui.valid = m.valid_mask;
    ui.colors = a->batch_colors;
    ui.sources = a->batch_sources;
    ui.n_total = m.n_total;
    ui.n_lobes = m.n_lobes;
    ui.responsibilities = ao->responsibilities;
    ui.candidate_tile_ids = ao->candidate_tile_ids;
    ui.candidate_slots = ao->candidate_slots;
    ui.row_masses = ao->row_masses;
    ui.k_assoc = a->assoc_cfg->k_assoc;
    c->push_req.fetch_add(1);
    if (c->push_sleeping.load()) {
      std::lock_guard<std::mutex> lk(c->push_mu);
      c->push_cv.notify_one();
    }
    lo->next_global_id = a->next_global_id;
    c->live_map = pm;
    mark(6);
    return GCS_OK;
  }
  for (int k = 0; k < ncl; ++k)
    if ((rc = live::pmap_clear_tile_launch(pm, clear[k]))) return sub_fail(c, rc, "gcs_pmap_clear_tile", gcs_pmap_last_error(pm));
  gcs_pmap_update_inputs ui{};
  ui.Lambdas = m.Lambdas;
  ui.thetas = m.thetas;
  ui.etas = m.etas;
  ui.weights = m.weights;
  ui.valid = m.valid_mask;
  ui.colors = a->batch_colors;
  ui.sources = a->batch_sources;
  ui.n_total = m.n_total;
  ui.n_lobes = m.n_lobes;
  ui.responsibilities = ao->responsibilities;
  ui.candidate_tile_ids = ao->candidate_tile_ids;
  ui.candidate_slots = ao->candidate_slots;
  ui.row_masses = ao->row_masses;
  ui.k_assoc = a->assoc_cfg->k_assoc;
  if ((rc = live::pmap_update_launch(pm, lo->active_slots, lo->active_ids, na, out->z_t, a->timestamp, a->scan_seq,
                                     a->next_global_id, a->update_cfg, &ui)))
    return sub_fail(c, rc, "gcs_pmap_map_update", gcs_pmap_last_error(pm));
  lo->next_global_id = a->next_global_id;
  c->live_map = pm;
  mark(6);
  return GCS_OK;
}

int gcs_live_collect(gcs_ctx* c, gcs_live_outputs* lo) {
  if (!c || !lo) return fail(c, GCS_ERR_ARG, "null argument");
  if (!c->live_map) return fail(c, GCS_ERR_STATE, "gcs_live_collect without gcs_live_scan");
  gcs_pmap* pm = c->live_map;
  c->live_map = nullptr;
  const clk::time_point t_in = clk::now();
  if (int rc = push_wait(c)) return rc;  // step 12b's launch calls (worker)
  if (int rc = live::pmap_update_collect(pm, &lo->next_global_id, &lo->update, lo->counts))
    return sub_fail(c, rc, "gcs_pmap_map_update", gcs_pmap_last_error(pm));
  lo->phase_us[7] = 1e3 * ms_between(t_in, clk::now());
  return GCS_OK;
}

// ---------------------------------------------------------------- hypothesis payload / combine
namespace {
// Payload layout: [w_iw dPsi 252 | w_iw dnu 7 | w_iw dPsi_meas 27 | w_iw dnu_meas 3 |
// w L 484 | w h 22 | w z 22 | w mu 22 | w |mu|^2 1]
// fac (may be null): the lifted factor of b.L, already computed (the context's last tail)
void pack_payload(const Belief& b, const double* dPsi, const double* dnu, const double* mdPsi, const double* mdnu,
                  double w_iw, double w_bary, double* p, const host::SpdFactor* fac = nullptr) {
  int k = 0;
  for (int i = 0; i < 252; ++i) p[k++] = w_iw * (dPsi ? dPsi[i] : 0.0);
  for (int i = 0; i < 7; ++i) p[k++] = w_iw * (dnu ? dnu[i] : 0.0);
  for (int i = 0; i < 27; ++i) p[k++] = w_iw * (mdPsi ? mdPsi[i] : 0.0);
  for (int i = 0; i < 3; ++i) p[k++] = w_iw * (mdnu ? mdnu[i] : 0.0);
  for (int i = 0; i < DZ * DZ; ++i) p[k++] = w_bary * b.L[i];
  for (int i = 0; i < DZ; ++i) p[k++] = w_bary * b.h[i];
  for (int i = 0; i < DZ; ++i) p[k++] = w_bary * b.z_lin[i];
  double mu[DZ], n2 = 0.0;
  if (fac) host::spd_factor_solve(*fac, b.h, mu);  // mean_increment with the factor already at hand
  else host::mean_increment(b, mu);
  for (int i = 0; i < DZ; ++i) { p[k++] = w_bary * mu[i]; n2 += mu[i] * mu[i]; }
  p[k++] = w_bary * n2;
}

// The summed payload -> barycenter (PSD of L, hypothesis.py:92-115) + process IW apply with
// weight min(1, scan_count) + Q rebuild + measurement IW apply with weight 1 (backend_node.py:2102-2119)
void apply_payload(const double* p, int32_t scan_count, const double* X_anchor, double stamp, const double* nu7,
                   const double* Psi, const double* mnu, const double* mPsi, Belief& out, double* nu_out,
                   double* Psi_out, double* Q_out, double* mnu_out, double* mPsi_out, double* cert4,
                   double* meas_cert2) {
  const double* dPsi = p;
  const double* dnu = p + 252;
  const double* L = p + 289;
  const double* h = L + 484;
  const double* z = h + 22;
  const double* mu = z + 22;
  const double n2 = mu[22];
  memset(&out, 0, sizeof(out));
  const double delta = host::psd_project(DZ, L, kEpsPsd, out.L);
  memcpy(out.h, h, sizeof(out.h));
  memcpy(out.z_lin, z, sizeof(out.z_lin));
  memcpy(out.X_anchor, X_anchor, sizeof(out.X_anchor));
  out.stamp = stamp;
  double m2 = 0.0;
  for (int i = 0; i < DZ; ++i) m2 += mu[i] * mu[i];
  const double wp = std::min(1, scan_count);
  double dP[252], dn[7], c2[2];
  for (int i = 0; i < 252; ++i) dP[i] = wp * dPsi[i];
  for (int i = 0; i < 7; ++i) dn[i] = wp * dnu[i];
  host::process_iw_apply(nu7, Psi, dP, dn, nu_out, Psi_out, c2);
  host::process_noise_Q(nu_out, Psi_out, Q_out);
  double mc[2];
  host::meas_iw_apply(mnu, mPsi, p + 259, p + 286, mnu_out, mPsi_out, mc);
  if (meas_cert2) { meas_cert2[0] = mc[0]; meas_cert2[1] = mc[1]; }
  if (cert4) { cert4[0] = delta; cert4[1] = n2 - m2; cert4[2] = c2[0]; cert4[3] = c2[1]; }
}

int combine_into_ctx(gcs_ctx* c, const double* p, int32_t scan_count, gcs_belief* comb, double* cert) {
  Belief out;
  double nu2[7], Psi2[252], Q2[DZ * DZ], mnu2[3], mPsi2[27], c4[4];
  apply_payload(p, scan_count, c->belief.X_anchor, c->belief.stamp, c->iw_nu, c->iw_Psi, c->meas_nu, c->meas_Psi,
                out, nu2, Psi2, Q2, mnu2, mPsi2, c4, c->meas_cert);
  memcpy(c->iw_nu, nu2, sizeof(nu2));
  memcpy(c->iw_Psi, Psi2, sizeof(Psi2));
  memcpy(c->Q, Q2, sizeof(Q2));
  memcpy(c->meas_nu, mnu2, sizeof(mnu2));
  memcpy(c->meas_Psi, mPsi2, sizeof(mPsi2));
  if (comb) from_host_belief(out, *comb);
  if (cert) memcpy(cert, c4, sizeof(c4));
  return GCS_OK;
}
}  // namespace

int gcs_hypothesis_payload(gcs_ctx* c, double w_iw, double w_bary, double* p) {
  if (!c || !p) return GCS_ERR_ARG;
  const bool h = c->have_last;
  pack_payload(c->belief, h ? c->last_dPsi : nullptr, h ? c->last_dnu : nullptr, h ? c->last_meas_dPsi : nullptr,
               h ? c->last_meas_dnu : nullptr, w_iw, w_bary, p, c->prev_fac_valid ? &c->prev_fac : nullptr);
  return GCS_OK;
}

int gcs_hypothesis_combine(gcs_ctx* c, const double* p, int32_t scan_count, gcs_belief* comb, double* cert) {
  if (!c || !p) return GCS_ERR_ARG;
  return combine_into_ctx(c, p, scan_count, comb, cert);
}

int gcs_payload_pack(const gcs_belief* b, const double* dPsi, const double* dnu, const double* mdPsi,
                     const double* mdnu, double w_iw, double w_bary, double* payload) {
  if (!b || !payload) return GCS_ERR_ARG;
  Belief hb;
  to_host_belief(*b, hb);
  pack_payload(hb, dPsi, dnu, mdPsi, mdnu, w_iw, w_bary, payload);
  return GCS_OK;
}

int gcs_datasheet_noise_states(double* nu7, double* Psi252, double* mnu3, double* mPsi27) {
  if (!nu7 || !Psi252 || !mnu3 || !mPsi27) return GCS_ERR_ARG;
  host::datasheet_iw_state(nu7, Psi252);
  host::datasheet_meas_iw_state(mnu3, mPsi27);
  return GCS_OK;
}

int gcs_payload_apply(const double* p, int32_t scan_count, const double* X_anchor, double stamp, const double* nu7,
                      const double* Psi, const double* mnu, const double* mPsi, gcs_belief* comb, double* nu_out,
                      double* Psi_out, double* Q_out, double* mnu_out, double* mPsi_out, double* cert4) {
  if (!p || !X_anchor || !nu7 || !Psi || !mnu || !mPsi || !nu_out || !Psi_out || !Q_out || !mnu_out || !mPsi_out)
    return GCS_ERR_ARG;
  Belief out;
  apply_payload(p, scan_count, X_anchor, stamp, nu7, Psi, mnu, mPsi, out, nu_out, Psi_out, Q_out, mnu_out, mPsi_out,
                cert4, nullptr);
  if (comb) from_host_belief(out, *comb);
  return GCS_OK;
}

// ---------------------------------------------------------------- RCCL
int gcs_rccl_get_unique_id(uint8_t* id) {
  if (!id) return GCS_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return GCS_ERR_HIP;
  static_assert(sizeof(u) == GCS_RCCL_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof(u));
  return GCS_OK;
}

int gcs_rccl_comm_init(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t* id, void** comm) {
  if (!id || !comm || n_ranks < 1 || rank < 0 || rank >= n_ranks) return GCS_ERR_ARG;
  *comm = nullptr;
  if (hipSetDevice(device) != hipSuccess) return GCS_ERR_HIP;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t cm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&cm, n_ranks, u, rank);
  if (r != ncclSuccess) {  // the reason, for gcs_last_error(NULL) (e.g. two ranks on one device)
    const char* last = ncclGetLastError(nullptr);
    t_create_msg = std::string("ncclCommInitRank: ") + ncclGetErrorString(r) + (last && *last ? std::string(": ") + last : "");
    return GCS_ERR_HIP;
  }
  *comm = (void*)cm;
  return GCS_OK;
}

int gcs_rccl_comm_destroy(void* comm) {
  if (!comm) return GCS_OK;

  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? GCS_OK : GCS_ERR_HIP;
}

int gcs_rccl_broadcast(void* comm, void* buf, int64_t bytes, int32_t root, void* stream) {
  if (!comm || (!buf && bytes > 0) || bytes < 0 || root < 0) return GCS_ERR_ARG;
  if (bytes == 0) return GCS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, (ncclComm_t)comm, s) != ncclSuccess) return GCS_ERR_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? GCS_OK : GCS_ERR_HIP;
}

int gcs_rccl_comm_count(void* comm, int32_t* count, int32_t* user_rank) {
  if (!comm || !count || !user_rank) return GCS_ERR_ARG;
  int n = 0, r = 0;
  if (ncclCommCount((ncclComm_t)comm, &n) != ncclSuccess) return GCS_ERR_HIP;
  if (ncclCommUserRank((ncclComm_t)comm, &r) != ncclSuccess) return GCS_ERR_HIP;
  *count = n;
  *user_rank = r;
  return GCS_OK;
}

int gcs_combine_allreduce(gcs_ctx* c, void* comm, double w_iw, double w_bary, int32_t scan_count,
                          gcs_belief* comb, double* cert);

int gcs_scan_combine(gcs_ctx* c, const gcs_scan_inputs* in, gcs_scan_outputs* out, void* comm, double w_iw,
                     double w_bary, int32_t scan_count, gcs_belief* comb, double* cert, double* combine_ms) {
  const clk::time_point tc = clk::now();
  if (int rc = gcs_scan(c, in, out)) return rc;
  const clk::time_point t0 = clk::now();
  const int rc = gcs_combine_allreduce(c, comm, w_iw, w_bary, scan_count, comb, cert);
  const clk::time_point t1 = clk::now();
  const double cm = ms_between(t0, t1);
  if (combine_ms) *combine_ms = cm;
  c->host_sums[8] += cm;
  c->host_sums[9] += ms_between(tc, t1);
  ++c->host_n[1];
  if (c->host_n[0] > 0) {
    float* hh = c->host_hist.data() + (size_t)((c->host_n[0] - 1) % gcs_ctx::kHostHist) * 6;
    hh[4] = (float)cm;
    hh[5] = (float)ms_between(tc, t1);
  }
  return rc;
}

int gcs_combine_allreduce(gcs_ctx* c, void* comm, double w_iw, double w_bary, int32_t scan_count,
                          gcs_belief* comb, double* cert) {
  if (!c) return GCS_ERR_ARG;
  constexpr int kLen = GCS_PAYLOAD_LEN + GCS_MAP_REC_LEN;
  if (!c->h_payload) {
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    HIPCHK(c, hipHostMalloc(&c->h_payload, kLen * sizeof(double), fl));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->dh_payload, c->h_payload, 0));
    HIPCHK(c, hipHostMalloc(&c->h_psum, (kLen + 2) * sizeof(double), fl));
    memset(c->h_psum, 0, (kLen + 2) * sizeof(double));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->dh_psum, c->h_psum, 0));
    HIPCHK(c, hipMalloc(&c->d_payload, kLen * sizeof(double)));
    HIPCHK(c, hipMalloc(&c->d_payload_in, kLen * sizeof(double)));
    HIPCHK(c, hipMalloc(&c->d_pay_seq, sizeof(uint64_t)));
    HIPCHK(c, hipMemset(c->d_pay_seq, 0, sizeof(uint64_t)));
    HIPCHK(c, hipStreamSynchronize(nullptr));  // (the null stream does not order the combine stream)
    c->pay_seq = 0;
  }
  if (int rc = gcs_hypothesis_payload(c, w_iw, w_bary, c->h_payload)) return rc;
  // one map (LEAD / FOLLOW): the lead's map-update record rides the same all-reduce (zeros elsewhere)
  const bool shared_map = c->map_mode != GCS_MAP_OWN;
  const int len = shared_map ? kLen : GCS_PAYLOAD_LEN;
  if (shared_map)
    for (int k = 0; k < GCS_MAP_REC_LEN; ++k)
      c->h_payload[GCS_PAYLOAD_LEN + k] = c->map_mode == GCS_MAP_LEAD ? c->map_rec[k] : 0.0;
  const double* sum = c->h_payload;
  if (comm) {
    // The reduction rides its own stream: nothing the scan queued on the context stream (k_tile_order
    // behind the PT fold) or the push stream (the pushforward) is ahead of it.  The payload needs no
    // device ordering: it is host data of the finished scan.  ncclAllReduce reads it from the pinned
    // host buffer, k_payload_out copies the sum back with the call's sequence number and a checksum,
    // and the host polls that (wait_stamped): no copy call and no stream synchronize.  Measured at world
    // size 1 (profiles/r05/combine/, rccl/): 16.5 us per call alone and 19 us inside the C2 pipeline,
    // against 3.3 us for the host-only combine; the stage-out kernel alone takes 16.7 alone (a kernel
    // round trip from an idle stream).  A separate stage-in kernel, a captured graph, the context
    // stream, the sum written straight to pinned memory with hipStreamQuery polled, and a device-side
    // gate queued ahead of the call (which also held every device-wide synchronize until its timeout)
    // gave nothing.
    if (!c->comm_stream) {
      // the device's highest priority: the combine's kernels are dispatched ahead of the pushforward
      // that was just queued on the push stream (same box, alternated, profiles/r05/rccl/: combine 32 ->
      // 19 us in the C2 pipeline, 0.1275-0.1295 -> 0.1154-0.1161 ms per step; GCSLAM_COMBINE_PRIO=0)
      static const bool prio = [] {
        const char* e = getenv("GCSLAM_COMBINE_PRIO");
        return !(e && atoi(e) == 0);
      }();
      int lo = 0, hi = 0;
      if (prio && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
        HIPCHK(c, hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, hi));
      else
        HIPCHK(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    }
    hipStream_t s = c->comm_stream;
    if (comm != c->comm_seen) {
      int n = 1;
      if (ncclCommCount((ncclComm_t)comm, &n) != ncclSuccess) return fail(c, GCS_ERR_HIP, "ncclCommCount");
      c->comm_seen = comm;
      c->comm_world = n;
    }
    // The send buffer: at world size 1 the collective is a local copy and reads the pinned host buffer
    // directly (measured above).  With more ranks RCCL's ring kernels would read it across PCIe inside
    // the collective (and a transport that registers user buffers expects device memory), so the
    // payload is first copied to device memory by the copy engine on the same stream.
    const bool dev_send = c->sendbuf_mode == 1 || (c->sendbuf_mode < 0 && c->comm_world > 1);
    const double* send = c->dh_payload;
    if (dev_send) {
      HIPCHK(c, hipMemcpyAsync(c->d_payload_in, c->h_payload, len * sizeof(double), hipMemcpyHostToDevice, s));
      send = c->d_payload_in;
    }
    if (c->combine_delay_us) HIPCHK(c, launch_delay(c->combine_delay_us, s));
    ncclResult_t r = ncclAllReduce(send, c->d_payload, len, ncclDouble, ncclSum, (ncclComm_t)comm, s);
    if (r != ncclSuccess) return fail(c, GCS_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    HIPCHK(c, launch_payload_out(c->d_payload, c->dh_psum, len, c->d_pay_seq, s));
    const uint64_t seq = ++c->pay_seq;
    if (int rc = wait_stamped(c, c->h_psum, len, seq, s, &c->pay_rereads, &c->pay_syncs, "hypothesis all-reduce"))
      return rc;
    sum = c->h_psum;
  }
  if (shared_map) {  // a single rank carries its own record (a follower then replays its own update)
    memcpy(c->lead_rec, comm ? sum + GCS_PAYLOAD_LEN : c->map_rec, sizeof(c->lead_rec));
    c->have_lead_rec = true;
  }
  return combine_into_ctx(c, sum, scan_count, comb, cert);
}

int gcs_ctx_set_map_mode(gcs_ctx* c, int32_t mode) {
  if (!c) return GCS_ERR_ARG;
  if (mode < GCS_MAP_OWN || mode > GCS_MAP_FOLLOW) return fail(c, GCS_ERR_ARG, "map mode: GCS_MAP_OWN, _LEAD or _FOLLOW");
  c->map_mode = mode;
  c->have_lead_rec = false;
  return GCS_OK;
}

int gcs_ctx_map_record(gcs_ctx* c, double* rec) {
  if (!c || !rec) return GCS_ERR_ARG;
  if (!c->have_last) return fail(c, GCS_ERR_STATE, "no scan yet: no map-update record");
  memcpy(rec, c->map_rec, sizeof(c->map_rec));
  return GCS_OK;
}

// The lead's map update replayed on this context: k_budget + k_points at the lead's twist (the raw
// scan is the same on every hypothesis), the bin kernel (ScanBinStats and active flags: the lead's,
// bit for bit -- same kernels, same inputs), then k_pushforward at the lead's z_t and covariance.
// Its certificates and the planar / Matrix-Fisher reductions are not needed and not run.
int gcs_map_follow(gcs_ctx* c, const gcs_scan_inputs* in, const double* rec) {
  if (!c || !in) return fail(c, GCS_ERR_ARG, "null argument");
  if (c->map_mode != GCS_MAP_FOLLOW) return fail(c, GCS_ERR_STATE, "gcs_map_follow needs GCS_MAP_FOLLOW");
  if (!rec) {
    if (!c->have_lead_rec) return fail(c, GCS_ERR_STATE, "no lead record: pass rec or combine first");
    rec = c->lead_rec;
  }
  for (int k = 0; k < GCS_MAP_REC_LEN; ++k)
    if (!std::isfinite(rec[k])) return fail(c, GCS_ERR_NONFINITE, "map-update record not finite");
  double r[GCS_MAP_REC_LEN];
  memcpy(r, rec, sizeof(r));  // (rec may be the context's own lead_rec)
  memset(c->h_err, 0, sizeof(c->h_err));  // (as gcs_scan: this call's error words only)
  c->use_direct = c->cfg.mode == GCS_MODE_SCALE && c->direct_buckets && !c->sorted_sticky && c->d_members;
  struct DirectOff {
    gcs_ctx* c;
    ~DirectOff() { c->use_direct = false; }
  } direct_off{c};
  for (int pass = 0; pass < 2; ++pass) {
    if (int rc = push_wait(c)) return rc;
    c->budget_pending = false;
    if (int rc = stage_points(c, in->xyz_dev, in->point_step, in->timestamps_dev, in->weights_dev, in->n_points,
                              in->scan_start_time, in->scan_end_time, r, nullptr, nullptr, nullptr,
                              /*fold_later=*/true, in->xyz_format == 1))
      return rc;
    if (int rc = join_push(c)) return rc;
    if (int rc = stage_bins(c)) return rc;
    if (int rc = stage_tile_order(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->stages_done = true;
    if (int rc = pull_err(c)) return rc;
    if (int rc = check_bucket_err(c)) return rc;
    if (!(c->use_direct && c->h_err[2])) break;
    // a bucket overflowed the direct rows (the lead's scan was redone sorted too): redo sorted
    c->h_err[2] = 0u;
    c->sorted_sticky = true;
    c->use_direct = false;
  }
  c->h_err[1] = 0u;
  return submit_push(c, r + 6, r + 12, c->cfg.forgetting_factor, c->push_main ? c->stream : c->push_stream,
                     c->d_part_push);
}

int gcs_hypothesis_barycenter(int32_t n, const double* Ls, const double* hs, const double* zs, const double* w,
                              double* Lo, double* ho, double* zo, double* cert) {
  if (n < 1 || !Ls || !hs || !zs || !w || !Lo || !ho || !zo) return GCS_ERR_ARG;
  std::vector<double> wn(n);
  double wsum = 0.0, floor_adj = 0.0;
  for (int k = 0; k < n; ++k) {  // weight floor + renormalise (hypothesis.py:83-87)
    const double wf = std::max(w[k], 0.0025);
    floor_adj += fabs(wf - w[k]);
    wn[k] = wf;
    wsum += wf;
  }
  for (int k = 0; k < n; ++k) wn[k] /= wsum;
  double Lr[DZ * DZ] = {};
  for (int i = 0; i < DZ; ++i) { ho[i] = 0.0; zo[i] = 0.0; }
  for (int k = 0; k < n; ++k) {  // barycenter (:92-99)
    for (int i = 0; i < DZ * DZ; ++i) Lr[i] += wn[k] * Ls[(size_t)k * DZ * DZ + i];
    for (int i = 0; i < DZ; ++i) {
      ho[i] += wn[k] * hs[(size_t)k * DZ + i];
      zo[i] += wn[k] * zs[(size_t)k * DZ + i];
    }
  }
  double c6[6];
  host::psd_project(DZ, Lr, kEpsPsd, Lo, c6);
  // spread proxy (:103-115): sum w ||mu_k - sum w mu||^2
  std::vector<double> mus((size_t)n * DZ);
  double mom[DZ] = {};
  for (int k = 0; k < n; ++k) {
    host::spd_solve_lifted(DZ, Ls + (size_t)k * DZ * DZ, hs + (size_t)k * DZ, kEpsLift, &mus[(size_t)k * DZ]);
    for (int i = 0; i < DZ; ++i) mom[i] += wn[k] * mus[(size_t)k * DZ + i];
  }
  double spread = 0.0, ess_den = 0.0, supp = 0.0;
  for (int k = 0; k < n; ++k) {
    double d2 = 0.0;
    for (int i = 0; i < DZ; ++i) {
      const double d = mus[(size_t)k * DZ + i] - mom[i];
      d2 += d * d;
    }
    spread += wn[k] * d2;
    ess_den += wn[k] * wn[k];
    supp += wn[k] > 0.0025 ? 1.0 : 0.0;
  }
  if (cert) {
    cert[0] = c6[0]; cert[1] = floor_adj; cert[2] = 1.0 / ess_den; cert[3] = supp / n; cert[4] = spread; cert[5] = c6[4];
  }
  return GCS_OK;
}

int gcs_process_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                         double* Psi_out, double* cert2) {
  if (!nu || !Psi || !dPsi || !dnu || !nu_out || !Psi_out) return GCS_ERR_ARG;
  double c2[2];
  host::process_iw_apply(nu, Psi, dPsi, dnu, nu_out, Psi_out, c2);
  if (cert2) { cert2[0] = c2[0]; cert2[1] = c2[1]; }
  return GCS_OK;
}

int gcs_process_noise_Q(const double* nu, const double* Psi, double* Q) {
  if (!nu || !Psi || !Q) return GCS_ERR_ARG;
  host::process_noise_Q(nu, Psi, Q);
  return GCS_OK;
}

int gcs_meas_iw_mode(const double* nu, const double* Psi, int32_t idx, double* Sigma) {
  if (!nu || !Psi || !Sigma || idx < 0 || idx > 2) return GCS_ERR_ARG;
  host::meas_iw_mode(nu, Psi, idx, Sigma);
  return GCS_OK;
}

int gcs_ctx_describe(gcs_ctx* c, char* buf, int32_t len) {
  if (!c || !buf || len < 1) return GCS_ERR_ARG;
  const gcs_config& f = c->cfg;
  const bool scale = f.mode == GCS_MODE_SCALE;
  char tile_desc[160];
  snprintf(tile_desc, sizeof(tile_desc), "%sk_bins_scale, %d-bin tiles x %d lanes per bin (HIP)",
           c->use_direct || c->direct_buckets ? "direct buckets + " : "bucketing + ", c->tile_bins, 256 / c->tile_bins);
  char tmp[2048];
  int n = snprintf(tmp, sizeof(tmp),
      "{\"library\": \"%s\", \"abi\": %d, \"device\": %d, \"arch\": \"gfx950\", \"N_POINTS_CAP\": %d, "
      "\"B_BINS\": %d, \"soft_assign_mode\": \"%s\", \"k_cand\": %d, \"tau_soft_assign\": %.17g, "
      "\"tau_rule\": \"tau_B = 0.1 * 48 / B (declared)\", \"candidate_rule\": \"%s\", "
      "\"map_mode\": \"per-hypothesis MapBinStats (declared; reference couples through hypothesis 0)\", "
      "\"pushforward_form\": \"gamma forgetting + N[R(Sigma_p + pbar pbar^T)R^T + J Sigma_pose J^T + q q^T - u u^T], t_z := 0 (declared)\", "
      "\"forgetting_factor\": %.17g, \"deskew_rotation_only\": %s, \"gravity_W\": [%.17g, %.17g, %.17g], "
      "\"imu_gravity_scale\": %.17g, \"use_imu_odom\": %s, \"planar_z_ref\": %.17g, \"planar_z_sigma\": %.17g, "
      "\"planar_vz_sigma\": %.17g, \"alpha_min\": %.17g, \"alpha_max\": %.17g, \"c0_cond\": %.17g, "
      "\"eps_psd\": 1e-12, \"eps_lift\": 1e-09, \"eps_mass\": 1e-12, \"eps_r\": 1e-06, "
      "\"power_beta_min\": 0.25, \"power_beta_exc_c\": 50, \"power_beta_z_c\": 1, \"c_frob\": 1, "
      "\"MAX_IMU_PREINT_LEN\": 512, \"precision\": \"f64 state and accumulation, f32 xyz stream\", "
      "\"backends\": {\"points\": \"k_points (HIP)\", \"moment_match\": \"%s\", \"pushforward\": \"k_pushforward (HIP)\", "
      "\"tail_22d\": \"host C++\", \"imu_odom_evidence\": \"host C++ (gcs_evidence.cpp)\", "
      "\"hypothesis_combine\": \"payload sum all-reduce (RCCL) + host apply\"}}",
      gcs_version(), GCS_ABI_VERSION, f.device, f.n_points_cap, f.n_bins, scale ? "scale" : "dense", scale ? f.k_cand : 0,
      f.tau, scale ? "K nearest atlas bins of the exact nearest bin, ties -> lower id (declared)" : "dense N x B softmax (reference)",
      f.forgetting_factor, f.deskew_rotation_only ? "true" : "false", f.gravity_W[0], f.gravity_W[1], f.gravity_W[2],
      f.imu_gravity_scale, f.use_imu_odom ? "true" : "false", f.planar_z_ref, f.planar_z_sigma, f.planar_vz_sigma,
      f.alpha_min, f.alpha_max, f.c0_cond, scale ? tile_desc : "k_dense_accum + k_dense_finalize (HIP)");
  if (n < 0 || n >= len) return fail(c, GCS_ERR_ARG, "describe buffer too short");
  memcpy(buf, tmp, (size_t)n + 1);
  return GCS_OK;
}

// ---------------------------------------------------------------- host numerics
int gcs_psd_project(int32_t n, const double* M, double eps, double* out, double* cert6) {
  if (n < 1 || n > host::kMaxN || !M || !out) return GCS_ERR_ARG;
  host::psd_project(n, M, eps, out, cert6);
  return GCS_OK;
}
int gcs_spd_solve_lifted(int32_t n, const double* L, const double* b, double eps, double* x) {
  if (n < 1 || n > host::kMaxN || !L || !b || !x) return GCS_ERR_ARG;
  host::spd_solve_lifted(n, L, b, eps, x);
  return GCS_OK;
}
int gcs_spd_inverse_lifted(int32_t n, const double* L, double eps, double* Li) {
  if (n < 1 || n > host::kMaxN || !L || !Li) return GCS_ERR_ARG;
  host::spd_inverse_lifted(n, L, eps, Li);
  return GCS_OK;
}
int gcs_svd3(const double* H, double* U, double* s, double* V) {
  if (!H || !U || !s || !V) return GCS_ERR_ARG;
  svd3(H, U, s, V);
  return GCS_OK;
}
int gcs_imu_odom_evidence(const gcs_imu_odom_inputs* in, double* L, double* h, double* cert) {
  if (!in || !L || !h || in->m < 2 || !in->stamps || !in->gyro || !in->accel || !in->w_int || !in->pose0 ||
      !in->pose_pred || !in->mu_prev || !in->mu_inc || !in->gravity_W || !in->Sigma_g || !in->Sigma_a ||
      !in->odom_pose || !in->odom_cov_se3 || !in->odom_twist || !in->odom_twist_cov || !(in->planar_z_sigma > 0.0) ||
      !(in->planar_vz_sigma > 0.0))
    return GCS_ERR_ARG;
  host::ImuOdomOut* io = new host::ImuOdomOut();
  double ex[5];
  run_imu_odom(*in, *io, ex);
  memcpy(L, io->L, sizeof(io->L));
  memcpy(h, io->h, sizeof(io->h));
  if (cert) {
    const double v[GCS_IMU_ODOM_CERT_LEN] = {io->trigger, io->ess_weighted, io->kappa, io->transport_sigma,
                                             io->imu_scale, io->odom_scale, io->mean_reliability, io->odom.nll,
                                             io->imu.nll, io->gyro.nll, ex[0], ex[1], ex[2], ex[3], ex[4]};
    memcpy(cert, v, sizeof(v));
  }
  delete io;
  return GCS_OK;
}

int gcs_imu_odom_evidence_device(gcs_ctx* c, const gcs_imu_odom_inputs* in, double* L, double* h, double* cert) {
  if (!c) return GCS_ERR_ARG;
  if (!in || !L || !h || in->m < 2 || !in->stamps || !in->gyro || !in->accel || !in->w_int || !in->pose0 ||
      !in->pose_pred || !in->mu_prev || !in->mu_inc || !in->gravity_W || !in->Sigma_g || !in->Sigma_a ||
      !in->odom_pose || !in->odom_cov_se3 || !in->odom_twist || !in->odom_twist_cov || !(in->planar_z_sigma > 0.0) ||
      !(in->planar_vz_sigma > 0.0))
    return fail(c, GCS_ERR_ARG, "gcs_imu_odom_evidence_device: missing input");
  if (int rc = launch_imu_odom_dev(c, *in)) return rc;
  host::ImuOdomOut* io = new host::ImuOdomOut();
  double ex[5];
  const int rc = finish_imu_odom_dev(c, *io, ex);
  if (rc == GCS_OK) {
    memcpy(L, io->L, sizeof(io->L));
    memcpy(h, io->h, sizeof(io->h));
    if (cert) {
      const double v[GCS_IMU_ODOM_CERT_LEN] = {io->trigger, io->ess_weighted, io->kappa, io->transport_sigma,
                                               io->imu_scale, io->odom_scale, io->mean_reliability, io->odom.nll,
                                               io->imu.nll, io->gyro.nll, ex[0], ex[1], ex[2], ex[3], ex[4]};
      memcpy(cert, v, sizeof(v));
    }
  }
  delete io;
  return rc;
}

int gcs_imu_meas_iw_suffstats(int32_t m, const double* stamps, const double* gyro, const double* accel,
                              const double* w_int, const double* gb, const double* ab, const double* rv,
                              const double* g, double* dPsi, double* dnu) {
  if (m < 0 || !stamps || !gyro || !accel || !w_int || !gb || !ab || !rv || !g || !dPsi || !dnu) return GCS_ERR_ARG;
  host::imu_meas_iw_suffstats(m, stamps, gyro, accel, w_int, gb, ab, rv, g, dPsi, dnu);
  return GCS_OK;
}
int gcs_meas_iw_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double* nu_out,
                      double* Psi_out, double* cert2) {
  if (!nu || !Psi || !dPsi || !dnu || !nu_out || !Psi_out) return GCS_ERR_ARG;
  double c2[2];
  host::meas_iw_apply(nu, Psi, dPsi, dnu, nu_out, Psi_out, c2);
  if (cert2) { cert2[0] = c2[0]; cert2[1] = c2[1]; }
  return GCS_OK;
}
int gcs_debug_tile_order(int32_t device, const uint8_t* active, const uint32_t* work, int32_t n, int32_t xcd,
                         int32_t* order) {
  if (!active || !work || !order || n < 1) return GCS_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return GCS_ERR_HIP;
  uint8_t* da = nullptr;
  uint32_t* dw = nullptr;
  int* dord = nullptr;
  int rc = GCS_OK;
  if (hipMalloc(&da, n) != hipSuccess || hipMalloc(&dw, n * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&dord, n * sizeof(int)) != hipSuccess ||
      hipMemcpy(da, active, n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dw, work, n * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(dord, 0xff, n * sizeof(int)) != hipSuccess ||
      launch_tile_order_variant(da, dw, n, dord, xcd != 0, nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(order, dord, n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    rc = GCS_ERR_HIP;
  if (da) (void)hipFree(da);
  if (dw) (void)hipFree(dw);
  if (dord) (void)hipFree(dord);
  return rc;
}
int gcs_debug_preintegrate(int32_t device, int32_t m, const double* stamps, const double* gyro, const double* accel,
                           double t0, double t1, double sigma, const double* rotvec, const double* gyro_bias,
                           const double* accel_bias, const double* gravity, int32_t rotation_only, double* out) {
  if (m < 1 || !stamps || !gyro || !accel || !rotvec || !gyro_bias || !accel_bias || !gravity || !out)
    return GCS_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return GCS_ERR_HIP;
  double *hin = nullptr, *hout = nullptr, *dxi = nullptr;
  int rc = GCS_OK;
  if (hipHostMalloc(&hin, 7 * (size_t)m * sizeof(double), hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc(&hout, 16 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipMalloc(&dxi, 8 * sizeof(double)) != hipSuccess) {
    rc = GCS_ERR_HIP;
  } else {
    int r = m - 1;  // the same trailing-run trim as the scan prologue
    while (r > 0 && stamps[r - 1] == stamps[r]) --r;
    const int me = r + 1;
    memcpy(hin, stamps, me * sizeof(double));
    memcpy(hin + me, gyro, 3 * me * sizeof(double));
    memcpy(hin + 4 * me, accel, 3 * me * sizeof(double));
    PreintArgs a{};
    a.imu = hin;
    a.m = me;
    a.n_tail = m - me;
    a.tail_stamp = stamps[r];
    a.t0 = t0;
    a.t1 = t1;
    a.sigma = sigma;
    for (int k = 0; k < 3; ++k) {
      a.rotvec[k] = rotvec[k];
      a.gb[k] = gyro_bias[k];
      a.ab[k] = accel_bias[k];
      a.g[k] = gravity[k];
    }
    a.rotation_only = rotation_only;
    a.xi_dev = dxi;
    a.host_out = hout;
    double xi_dev[8];
    if (launch_preint(a, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(xi_dev, dxi, 6 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = GCS_ERR_HIP;
    } else {
      memcpy(out, hout, 16 * sizeof(double));
      for (int k = 0; k < 6; ++k)  // the device word k_points reads must equal the host record
        if (memcmp(&xi_dev[k], &hout[k], sizeof(double)) != 0) rc = GCS_ERR_HIP;
    }
  }
  if (hin) (void)hipHostFree(hin);
  if (hout) (void)hipHostFree(hout);
  if (dxi) (void)hipFree(dxi);
  return rc;
}
int gcs_psd_project3(const double* M, double* out, double* delta) {
  if (!M || !out) return GCS_ERR_ARG;
  const double d = psd_project3(M, out);
  if (delta) *delta = d;
  return GCS_OK;
}
int gcs_mf_rotation(const double* H, double* R) {
  if (!H || !R) return GCS_ERR_ARG;
  mf_rotation(H, R);
  return GCS_OK;
}
int gcs_predict_diffusion(const gcs_belief* prev, const double* Q, double dt, gcs_belief* pred, double* cert) {
  if (!prev || !Q || !pred) return GCS_ERR_ARG;
  Belief a, b;
  to_host_belief(*prev, a);
  double infl[3];
  host::predict_diffusion(a, Q, dt, b, infl);
  from_host_belief(b, *pred);
  if (cert) { cert[0] = infl[0]; cert[1] = infl[1]; cert[2] = infl[2]; cert[3] = 0.0; }
  return GCS_OK;
}
int gcs_info_fusion_additive(const gcs_belief* pred, const double* L_ev, const double* h_ev, double alpha,
                             gcs_belief* post, double* delta) {
  if (!pred || !L_ev || !h_ev || !post) return GCS_ERR_ARG;
  Belief a, b;
  to_host_belief(*pred, a);
  b = a;
  double Ls[DZ * DZ];
  for (int i = 0; i < DZ * DZ; ++i) Ls[i] = a.L[i] + alpha * L_ev[i];
  double d = host::psd_project(DZ, Ls, kEpsPsd, b.L);
  for (int i = 0; i < DZ; ++i) b.h[i] = a.h[i] + alpha * h_ev[i];
  from_host_belief(b, *post);
  if (delta) *delta = d;
  return GCS_OK;
}
int gcs_preintegrate_imu(int32_t m, const double* st, const double* gy, const double* ac, const double* w,
                         const double* rv, const double* gb, const double* ab, const double* g, double* dp, double* ess) {
  if (m < 1 || !st || !gy || !ac || !w || !rv || !gb || !ab || !g || !dp) return GCS_ERR_ARG;
  host::PreintOut o;
  host::preintegrate_imu(m, st, gy, ac, w, rv, gb, ab, g, o);
  memcpy(dp, o.delta_pose, 6 * sizeof(double));
  if (ess) *ess = o.ess;
  return GCS_OK;
}
int gcs_belief_world_pose(const gcs_belief* b, double* pose6) {
  if (!b || !pose6) return GCS_ERR_ARG;
  Belief a;
  to_host_belief(*b, a);
  host::mean_world_pose(a, pose6);
  return GCS_OK;
}
int gcs_fibonacci_atlas(int32_t B, double* dirs) {
  if (B < 1 || !dirs) return GCS_ERR_ARG;
  atlas::fibonacci(B, dirs);
  return GCS_OK;
}
int gcs_knn_table(int32_t B, const double* dirs, int32_t k, int32_t* knn) {
  if (B < 1 || k < 1 || k > B || !dirs || !knn) return GCS_ERR_ARG;
  atlas::knn(dirs, B, k, knn);
  return GCS_OK;
}
int gcs_nearest_bins(int32_t B, const double* dirs, int32_t nq, const double* q, int32_t* out) {
  if (B < 1 || nq < 0 || !dirs || (nq && (!q || !out))) return GCS_ERR_ARG;
  atlas::nearest(dirs, B, nq, q, out);
  return GCS_OK;
}

}  // extern "C"
