// Micro-benchmark of the surfel key sort (k_sf_sort_lds) alone: event-timed launches over seeded keys at
// several sizes and key widths, checked against a host stable sort.  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -I../include -Icsrc ../tools/sf_sort_bench.hip -L/opt/rocm/lib -lrccl
#include "gcs_surfels.hip"

#include <cstdio>
#include <random>
#include <vector>

int main() {
  using namespace gcs;
  const int cases[][3] = {{8192, 8192, 0}, {8192, 8192, 1}, {4096, 8192, 0}, {1024, 8192, 0}, {8192, 100, 0}, {8192, 65536, 0}};
  uint32_t *d_keys, *d_vals;
  int32_t* d_run;
  hipMalloc(&d_keys, 8192 * 4);
  hipMalloc(&d_vals, 8192 * 4);
  hipMalloc(&d_run, 2 * 65536 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& cs : cases) {
    const int n = cs[0], n_cells = cs[1], clustered = cs[2];
    std::mt19937 g(5);
    std::vector<uint32_t> keys(n);
    for (int i = 0; i < n; ++i) keys[i] = clustered ? (uint32_t)(g() % 64) * 97 % n_cells : g() % (n_cells + 1);
    hipMemcpy(d_keys, keys.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(d_run, 0, 2 * n_cells * 4);
    SfParams a{};
    a.n_cells = n_cells;
    int end_bit = 1;
    while ((1UL << end_bit) <= (unsigned long)n_cells) ++end_bit;
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k_sf_sort_lds, dim3(1), dim3(kSortThreads), 0, 0, d_keys, n, a, end_bit, d_vals, d_run);
    const int reps = 50;
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_sf_sort_lds, dim3(1), dim3(kSortThreads), 0, 0, d_keys, n, a, end_bit, d_vals, d_run);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint32_t> vals(n);
    hipMemcpy(vals.data(), d_vals, n * 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> ref(n);
    for (int i = 0; i < n; ++i) ref[i] = i;
    std::stable_sort(ref.begin(), ref.end(), [&](uint32_t x, uint32_t y) { return keys[x] < keys[y]; });
    const bool ok = vals == ref;
    printf("n=%5d n_cells=%6d end_bit=%2d clustered=%d: %.2f us per launch (back to back), %s\n", n, n_cells, end_bit,
           clustered, 1000.f * ms / reps, ok ? "ok" : "MISMATCH");
  }
  return 0;
}
