// Kernel argument blocks and launcher prototypes (internal; the public C-ABI is include/gcslam_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gcs_layout.h"

namespace gcs {

struct PointKernelArgs {
  // raw PointCloud2-like input (device)
  const uint8_t* xyz;  // float x,y,z at byte offsets 0,4,8 of each record
  int point_step;      // bytes per record
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
  const int* pools;        // ncell x pool_width, ascending ids, -1 padded
  int pool_width, grid;
  // outputs
  PointRec* recs;
  uint32_t* keys;
  uint32_t* slots;
  uint32_t* counts;  // per-bin bucket sizes (zeroed before the launch)
  uint8_t* flags;    // active-bin flags (zeroed before the launch)
  double* scalars;
  // optional debug/parity outputs (may be null)
  double* p0_out;
  double* w_out;
  double* w_budget_out;
  int* nearest_out;
};

struct BinKernelArgs {
  const PointRec* recs;
  const uint32_t* sorted_vals;
  const uint32_t* starts;
  const uint32_t* counts;
  const uint8_t* flags;
  const int* rknn_off;
  const int* rknn;
  const double* bin_dirs;
  int n_bins, cap;
  double origin[3];
  double tau;
  double* scan;  // 26 x B field-major
};

struct PushArgs {
  double R[9];
  double t[3];
  double Stt[9];  // translation block of the pose covariance
  double F[9];    // R S_rt   (rotation rows, translation columns)
  double G[9];    // R S_rr R^T
  double gamma;
};

hipError_t launch_budget(const double* w, int n_raw, int stride, double* partials, int nblk, double* scalars,
                         hipStream_t s);
hipError_t launch_points(const PointKernelArgs& a, bool scale, double* partials, int nblk, hipStream_t s);
hipError_t launch_bucketing(uint32_t* counts, uint32_t* starts, uint32_t* tile_sums, const uint32_t* keys,
                            const uint32_t* slots, int n, int n_bins, uint32_t* sorted, uint32_t* big_list,
                            uint32_t* big_n, hipStream_t s);
int bins_scale_blocks(int n_bins);
hipError_t launch_bins_scale(const BinKernelArgs& a, double* partials, hipStream_t s);
hipError_t launch_dense(const BinKernelArgs& a, double* bin_partials, double* partials, hipStream_t s);
hipError_t launch_bin_cert_final(const double* partials, int nblk, double* scalars, hipStream_t s);
hipError_t launch_mf(const double* scan, const double* map, int B, double* partials, int nblk, double* scalars,
                     hipStream_t s);
hipError_t launch_pt(const double* scan, const double* map, const double* derived, int B, double* partials, int nblk,
                     double* scalars, hipStream_t s);
hipError_t launch_pushforward(const double* scan, double* map, double* derived, int B, const PushArgs& pa,
                              hipStream_t s);
hipError_t launch_map_derive(const double* map, double* derived, int B, hipStream_t s);

}  // namespace gcs
