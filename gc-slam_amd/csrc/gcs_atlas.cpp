// Bin atlas construction on the host (once per context).
//   * Fibonacci directions: archive/bin_atlas.py:40-61.
//   * DECLARED scale-mode structures (DESIGN.md "candidate rule"):
//       knn[b]   = K nearest atlas bins of bin b by the canonical dot, ties -> lower id;
//       rknn     = reverse kNN lists (CSR, ascending source id) for the bin-centric gather;
//       pools[c] = for cube-map cell c, every bin that can be the nearest bin of a direction
//                  falling in c (radius 2 r_c + rho_c, see gcs_atlas.h), ascending ids.
#include "gcs_atlas.h"

#include <math.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "gcs_math.h"

namespace gcs {
namespace atlas {

void fibonacci(int B, double* dirs) {
  const double pi = 3.141592653589793;
  const double golden = pi * (1.0 + sqrt(5.0));
  for (int i = 0; i < B; ++i) {
    double idx = (double)i + 0.5;
    double phi = acos(1.0 - (2.0 * idx) / (double)B);
    double theta = golden * idx;
    double x = sin(phi) * cos(theta), y = sin(phi) * sin(theta), z = cos(phi);
    double n = sqrt(dot3_exact(x, y, z, x, y, z));
    double d = n + kEpsMass;
    dirs[3 * i] = x / d;
    dirs[3 * i + 1] = y / d;
    dirs[3 * i + 2] = z / d;
  }
}

namespace {

struct Grid {
  double h;
  int n;
  std::vector<int> start, idx;
  int coord(double x) const {
    int c = (int)floor((x + 1.0) / h);
    return c < 0 ? 0 : (c >= n ? n - 1 : c);
  }
  void build(const double* dirs, int B, double hh) {
    h = hh;
    n = std::max(1, (int)ceil(2.0 / h));
    size_t nc = (size_t)n * n * n;
    start.assign(nc + 1, 0);
    std::vector<int> cell(B);
    for (int b = 0; b < B; ++b) {
      cell[b] = (coord(dirs[3 * b]) * n + coord(dirs[3 * b + 1])) * n + coord(dirs[3 * b + 2]);
      start[cell[b] + 1]++;
    }
    for (size_t c = 0; c < nc; ++c) start[c + 1] += start[c];
    idx.assign(B, 0);
    std::vector<int> fill(start.begin(), start.end() - 1);
    for (int b = 0; b < B; ++b) idx[fill[cell[b]]++] = b;  // ascending ids inside each voxel
  }
  template <class F>
  void visit(const double* q, int rho, F&& f) const {
    int cx = coord(q[0]), cy = coord(q[1]), cz = coord(q[2]);
    for (int x = std::max(0, cx - rho); x <= std::min(n - 1, cx + rho); ++x)
      for (int y = std::max(0, cy - rho); y <= std::min(n - 1, cy + rho); ++y)
        for (int z = std::max(0, cz - rho); z <= std::min(n - 1, cz + rho); ++z) {
          size_t c = ((size_t)x * n + y) * n + z;
          for (int i = start[c]; i < start[c + 1]; ++i) f(idx[i]);
        }
  }
};

template <class F>
void parallel_for(int n, F&& f) {
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int i = (int)t; i < n; i += (int)nt) f(i);
    });
  for (auto& x : th) x.join();
}

struct Cand {
  double s;
  int id;
};
inline bool better(const Cand& a, const Cand& b) { return a.s > b.s || (a.s == b.s && a.id < b.id); }

// exact top-k (canonical dot, ties -> lower id) of query q; grid search with completeness check
void topk(const Grid& g, const double* dirs, int B, const double* q, int k, int* out) {
  std::vector<Cand> c;
  for (int rho = 1;; ++rho) {
    c.clear();
    g.visit(q, rho, [&](int b) {
      c.push_back({dot3_exact(q[0], q[1], q[2], dirs[3 * b], dirs[3 * b + 1], dirs[3 * b + 2]), b});
    });
    bool all = (2 * rho + 1) >= g.n;
    if ((int)c.size() >= k) {
      std::partial_sort(c.begin(), c.begin() + k, c.end(), better);
      double chord = sqrt(std::max(0.0, 2.0 - 2.0 * c[k - 1].s));
      if (all || chord <= rho * g.h * (1.0 - 1e-9)) break;
    } else if (all) {
      std::sort(c.begin(), c.end(), better);
      break;
    }
  }
  for (int i = 0; i < k; ++i) out[i] = i < (int)c.size() ? c[i].id : -1;
}

double grid_h(int B, int K) { return std::min(2.0, 1.2 * 2.0 * sqrt((double)std::max(K, 1) / (double)B)); }

}  // namespace

void knn(const double* dirs, int B, int K, int* out) {
  Grid g;
  g.build(dirs, B, grid_h(B, K));
  parallel_for(B, [&](int b) { topk(g, dirs, B, dirs + 3 * b, K, out + (size_t)b * K); });
}

void nearest(const double* dirs, int B, int nq, const double* q, int* out) {
  Grid g;
  g.build(dirs, B, grid_h(B, 1));
  parallel_for(nq, [&](int i) {
    const double* d = q + 3 * i;
    if (d[0] == 0.0 && d[1] == 0.0 && d[2] == 0.0) { out[i] = 0; return; }
    topk(g, dirs, B, d, 1, out + i);
  });
}

void reverse(const int* knn_tab, int B, int K, std::vector<int>& off, std::vector<int>& idx) {
  off.assign(B + 1, 0);
  for (size_t i = 0; i < (size_t)B * K; ++i) off[knn_tab[i] + 1]++;
  for (int b = 0; b < B; ++b) off[b + 1] += off[b];
  idx.assign((size_t)B * K, 0);
  std::vector<int> fill(off.begin(), off.end() - 1);
  for (int a = 0; a < B; ++a)
    for (int k = 0; k < K; ++k) idx[fill[knn_tab[(size_t)a * K + k]]++] = a;
}

static void cell_point(int face, double u, double v, double* p) {
  double x, y, z;
  switch (face) {
    case 0: x = 1.0; y = u; z = v; break;
    case 1: x = -1.0; y = u; z = v; break;
    case 2: x = u; y = 1.0; z = v; break;
    case 3: x = u; y = -1.0; z = v; break;
    case 4: x = u; y = v; z = 1.0; break;
    default: x = u; y = v; z = -1.0; break;
  }
  double n = sqrt(x * x + y * y + z * z);
  p[0] = x / n; p[1] = y / n; p[2] = z / n;
}

static double angle(const double* a, const double* b) {
  double c = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
  c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
  return acos(c);
}

int grid_for_bins(int B) {
  const double pi = 3.141592653589793;
  double s = sqrt(4.0 * pi / (double)B);
  return std::max(1, (int)ceil(2.0 / s));
}

void cell_pools(const double* dirs, int B, int G, std::vector<int>& pools, int& width, std::vector<float>* bounds) {
  int ncell = 6 * G * G;
  Grid g;
  g.build(dirs, B, grid_h(B, 4));
  std::vector<std::vector<int>> lists(ncell);
  std::vector<std::vector<float>> blists(bounds ? ncell : 0);
  parallel_for(ncell, [&](int c) {
    int face = c / (G * G), iu = (c / G) % G, iv = c % G;
    double du = 2.0 / G;
    double u = -1.0 + (iu + 0.5) * du, v = -1.0 + (iv + 0.5) * du;
    double ctr[3], cor[3];
    cell_point(face, u, v, ctr);
    double rc = 0.0;
    for (int k = 0; k < 4; ++k) {
      cell_point(face, u + ((k & 1) ? 0.5 : -0.5) * du, v + ((k & 2) ? 0.5 : -0.5) * du, cor);
      rc = std::max(rc, angle(ctr, cor));
    }
    int nb;
    topk(g, dirs, B, ctr, 1, &nb);
    double rho_c = angle(ctr, dirs + 3 * nb);
    double R = 2.0 * rc + rho_c + 1e-6;
    double chord = 2.0 * sin(std::min(R, 3.14159) * 0.5);
    int rho = std::max(1, (int)ceil(chord / g.h));
    double cosR = cos(std::min(R, 3.141592653589793)) - 1e-12;
    std::vector<int>& L = lists[c];
    g.visit(ctr, rho, [&](int b) {
      double s = ctr[0] * dirs[3 * b] + ctr[1] * dirs[3 * b + 1] + ctr[2] * dirs[3 * b + 2];
      if (s >= cosR) L.push_back(b);
    });
    if (!bounds) {
      std::sort(L.begin(), L.end());
      return;
    }
    // nearest-first order (angle from the cell centre, ties by id) with, per entry, an upper bound of
    // the dot of any direction in the cell with that bin and every later one: a direction within rc
    // of the centre is at least theta_b - rc from bin b, so dot <= cos(max(theta_b - rc, 0)); the
    // bound is rounded up to float with a 1e-6 margin, so a search may stop once the next entry's
    // bound is below its best dot (no later bin can reach or tie it)
    std::vector<std::pair<double, int>> th(L.size());
    for (size_t k = 0; k < L.size(); ++k) th[k] = {angle(ctr, dirs + 3 * L[k]), L[k]};
    std::sort(th.begin(), th.end());
    std::vector<float>& F = blists[c];
    F.resize(L.size());
    for (size_t k = 0; k < L.size(); ++k) {
      L[k] = th[k].second;
      const double bd = cos(std::max(th[k].first - rc, 0.0)) + 1e-6;
      F[k] = std::nextafter((float)bd, 2.0f);
    }
  });
  width = 1;
  for (auto& L : lists) width = std::max(width, (int)L.size() + 1);  // >= one -1 terminator
  width = (width + 3) & ~3;                                           // int4 loads
  pools.assign((size_t)ncell * width, -1);
  for (int c = 0; c < ncell; ++c)
    std::copy(lists[c].begin(), lists[c].end(), pools.begin() + (size_t)c * width);
  if (bounds) {
    bounds->assign((size_t)ncell * width, -2.0f);  // padding: below any dot, ends the search
    for (int c = 0; c < ncell; ++c)
      std::copy(blists[c].begin(), blists[c].end(), bounds->begin() + (size_t)c * width);
  }
}

namespace {
// Hilbert index of (x, y) on an n x n grid (n a power of two)
uint64_t hilbert_d(uint32_t n, uint32_t x, uint32_t y) {
  uint64_t d = 0;
  for (uint32_t s = n / 2; s > 0; s /= 2) {
    uint32_t rx = (x & s) > 0, ry = (y & s) > 0;
    d += (uint64_t)s * s * ((3 * rx) ^ ry);
    if (ry == 0) {
      if (rx == 1) { x = s - 1 - x; y = s - 1 - y; }
      std::swap(x, y);
    }
  }
  return d;
}
}  // namespace

void hilbert_order(const double* dirs, int B, std::vector<int>& order) {
  const uint32_t n = 1u << 15;
  std::vector<uint64_t> key(B);
  for (int b = 0; b < B; ++b) {
    const double* d = dirs + 3 * b;
    double ax = fabs(d[0]), ay = fabs(d[1]), az = fabs(d[2]);
    int f;
    double m, u, v;
    if (ax >= ay && ax >= az) { f = d[0] >= 0.0 ? 0 : 1; m = ax; u = d[1]; v = d[2]; }
    else if (ay >= az) { f = d[1] >= 0.0 ? 2 : 3; m = ay; u = d[0]; v = d[2]; }
    else { f = d[2] >= 0.0 ? 4 : 5; m = az; u = d[0]; v = d[1]; }
    if (!(m > 0.0)) { m = 1.0; u = v = 0.0; }
    auto q = [&](double x) {
      long c = (long)floor((x / m + 1.0) * 0.5 * n);
      return (uint32_t)std::min<long>(std::max<long>(c, 0), n - 1);
    };
    key[b] = ((uint64_t)f << 40) | hilbert_d(n, q(u), q(v));
  }
  order.resize(B);
  for (int b = 0; b < B; ++b) order[b] = b;
  std::stable_sort(order.begin(), order.end(), [&](int a, int c) { return key[a] < key[c]; });
}

int tile_sources(const std::vector<int>& off, const std::vector<int>& idx, int B, int tile, std::vector<int>& src_off,
                 std::vector<int>& src, std::vector<uint16_t>& local) {
  const int nt = (B + tile - 1) / tile;
  src_off.assign(nt + 1, 0);
  src.clear();
  local.assign(idx.size(), 0);
  int most = 0;
  std::vector<int> u;
  for (int t = 0; t < nt; ++t) {
    const int b0 = t * tile, b1 = std::min(B, b0 + tile);
    u.assign(idx.begin() + off[b0], idx.begin() + off[b1]);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    for (int q = off[b0]; q < off[b1]; ++q)
      local[q] = (uint16_t)(std::lower_bound(u.begin(), u.end(), idx[q]) - u.begin());
    src.insert(src.end(), u.begin(), u.end());
    src_off[t + 1] = (int)src.size();
    most = std::max(most, (int)u.size());
  }
  return most;
}

}  // namespace atlas
}  // namespace gcs
