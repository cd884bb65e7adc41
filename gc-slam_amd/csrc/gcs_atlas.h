// Host construction of the bin atlas and the scale-mode lookup structures.
//
// Nearest-bin pools: for a cube-map cell with centre c, corner radius r_c and nearest-bin
// distance rho_c, any direction q in the cell has its nearest bin n(q) within
// d(q, n(q)) <= d(q, n(c)) <= r_c + rho_c of q, hence within 2 r_c + rho_c of c.  The pool of
// c holds every bin inside that radius (plus margin), so a scan of the pool with the exact
// canonical dot returns the same bin as a brute-force scan of all B bins.
#pragma once
#include <stdint.h>

#include <vector>

namespace gcs {
namespace atlas {

void fibonacci(int B, double* dirs /*B*3*/);
void knn(const double* dirs, int B, int K, int* out /*B*K*/);
void nearest(const double* dirs, int B, int nq, const double* q, int* out);
void reverse(const int* knn, int B, int K, std::vector<int>& off, std::vector<int>& idx);
int grid_for_bins(int B);
// Per cube-map cell the bins that can be nearest to a direction in the cell.  bounds == nullptr:
// ascending ids.  Otherwise nearest-first order (angle from the cell centre) and, per entry, a float
// upper bound of the dot of any in-cell direction with that entry and every later one (-2 padding).
void cell_pools(const double* dirs, int B, int G, std::vector<int>& pools, int& width,
                std::vector<float>* bounds = nullptr);

// Device bin order (declared layout, DESIGN.md "bin order"): bins sorted by cube face and the
// Hilbert index of their face coordinates, so consecutive device bins form compact patches and a
// tile of bins shares its reverse-kNN source buckets.  order[device id] = reference id.
void hilbert_order(const double* dirs, int B, std::vector<int>& order);

// Per tile of `tile` consecutive device bins: the ascending unique source buckets of the tile's
// reverse-kNN lists (src_off/src CSR) and, per reverse-kNN entry, its index in that list.
// Returns the largest per-tile source count.
int tile_sources(const std::vector<int>& rknn_off, const std::vector<int>& rknn, int B, int tile,
                 std::vector<int>& src_off, std::vector<int>& src, std::vector<uint16_t>& local);

}  // namespace atlas
}  // namespace gcs
