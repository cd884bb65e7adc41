// Host check: the shared fixed-size PSD projection (gcs_small.h small::psd_project<N>, which the device
// IMU / odometry assembly and the host branch both run) against the host numerics' run-time-n form
// (gcs_host.cpp host::psd_project), bit for bit, on random 3x3 / 6x6 matrices -- PSD and indefinite,
// with exactly-zero rows and columns (the zero-row split) -- so the in-place masked split equals the
// compacted one.  Built and run by tests/test_small_numerics.py.
#include <cstdio>
#include <cstring>
#include <random>
#include "gcs_small.h"
#include "gcs_host.h"
using namespace gcs;
int main() {
  std::mt19937_64 g(7);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::uniform_int_distribution<int> ui(0, 3);
  long bad = 0, zero_path = 0, jac = 0;
  for (int it = 0; it < 200000; ++it) {
    const int n = (it & 1) ? 6 : 3;
    double M[36];
    for (int i = 0; i < n * n; ++i) M[i] = nd(g);
    if (ui(g) == 0) {  // PSD-ish
      double A[36];
      for (int i = 0; i < n * n; ++i) A[i] = M[i];
      for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) { double s = 0; for (int k = 0; k < n; ++k) s += A[i*n+k]*A[j*n+k]; M[i*n+j] = s; }
    }
    const int nz = ui(g);  // zero rows / cols
    bool hadz = false;
    for (int z = 0; z < nz; ++z) {
      const int r = ui(g) % n;
      for (int j = 0; j < n; ++j) M[r * n + j] = M[j * n + r] = 0.0;
      hadz = true;
    }
    double o1[36], o2[36];
    const double d1 = n == 3 ? small::psd_project<3>(M, 1e-12, o1) : small::psd_project<6>(M, 1e-12, o1);
    const double d2 = host::psd_project(n, M, 1e-12, o2);
    zero_path += hadz; jac += d1 > 0;
    if (memcmp(o1, o2, n * n * 8) != 0 || memcmp(&d1, &d2, 8) != 0) { if (bad < 5) printf("mismatch n=%d it=%d d %g %g\n", n, it, d1, d2); ++bad; }
  }
  printf("bad %ld zero-row cases %ld nonzero delta %ld\n", bad, zero_path, jac);
}
