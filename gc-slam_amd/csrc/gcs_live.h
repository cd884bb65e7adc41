// Split forms of the per-operator entry points for the one-call live primitive path (gcs_live_scan,
// gcs_capi.cpp): each *_launch queues an operator's kernels on its context's stream without the host
// wait of the public entry point, each *_collect reads the host results after the caller's stream
// synchronize.  The public entry points are launch + synchronize + collect, so both paths run the
// same kernels on the same arguments.  Internal to libgcslam_hip.so.
#pragma once
#include <cstdint>

#include "gcslam_hip.h"

namespace gcs {
namespace live {

// gcs_extract_lidar_surfels (lidar_surfel_extraction.py:339-431)
int surfel_launch(gcs_surfel_ctx* c, const double* points, const double* timestamps, const double* weights,
                  int32_t n, gcs_surfel_outputs* o);
void surfel_collect(gcs_surfel_ctx* c, gcs_surfel_outputs* o);
// the surfel count on the device (written by the extraction's slot kernel), for launches queued behind it
const int32_t* surfel_nvalid_dev(gcs_surfel_ctx* c);
// queue the context's work on stream s (the null stream allowed), after what it queued before
int surfel_bind_stream(gcs_surfel_ctx* c, void* s);

// gcs_associate_primitives_ot (primitive_association.py:239-553)
// n_valid_dev (may be null): the measurement count on the device, read by the kernels instead of m->n_valid
int assoc_launch(gcs_assoc_ctx* c, const gcs_assoc_config* cfg, const gcs_assoc_meas* m, const gcs_assoc_view* v,
                 gcs_assoc_outputs* o, const int32_t* n_valid_dev = nullptr);
void assoc_collect(gcs_assoc_ctx* c, gcs_assoc_outputs* o);
int assoc_bind_stream(gcs_assoc_ctx* c, void* s);
// gcs_visual_pose_evidence (visual_pose_evidence.py:260-412) split at its wait; collect takes the count
int vpe_launch(gcs_assoc_ctx* c, const gcs_assoc_meas* m, const gcs_assoc_view* v, const double* responsibilities,
               const int32_t* candidate_pool_indices, const double* row_masses, int32_t k_assoc,
               const double* z_lin_pose, double eps_lift, double eps_mass, const int32_t* n_valid_dev = nullptr);
void vpe_collect(gcs_assoc_ctx* c, int32_t n_valid, int32_t k_assoc, const double* z_lin_pose, double eps_lift,
                 gcs_vpe_outputs* o);

int pmap_bind_stream(gcs_pmap* p, void* s);
// create_empty_tile (primitive_map.py:148-174) without the wait
int pmap_clear_tile_launch(gcs_pmap* p, int32_t tile);
// primitive_map_recency_inflate (:1400-1484): partials in their own mapped region, read by collect
int pmap_recency_launch(gcs_pmap* p, const int32_t* tiles, int32_t n, int64_t scan_seq, double lam,
                        double min_scale);
void pmap_recency_collect(gcs_pmap* p, int32_t n, double* stats);
// extract_atlas_map_view (:356-450); the view's tile ids also land in p's device tile-id buffer
int pmap_view_launch(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, int32_t m_view,
                     double eps_lift, double eps_mass, gcs_pmap_view* o);
// copy of the last staged tile ids (pmap_view_launch) to dst (device, n)
int pmap_copy_staged_ids(gcs_pmap* p, int64_t* dst, int32_t n);
// step 12b (pipeline.py:1232-1492): everything up to the cull queued; collect waits, reads the
// statistics and runs the merge-reduce of the tiles that need it
int pmap_update_launch(gcs_pmap* p, const int32_t* tiles, const int64_t* tile_ids, int32_t n, const double* z_t6,
                       double timestamp, int64_t scan_seq, int64_t next_global_id, const gcs_pmap_update_config* cfg,
                       const gcs_pmap_update_inputs* in);
int pmap_update_collect(gcs_pmap* p, int64_t* next_global_id, gcs_pmap_update_stats* st, int32_t* counts);

}  // namespace live
}  // namespace gcs
