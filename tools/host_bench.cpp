// CPU micro-benchmark of the host 22-D numerics of one gcs_scan (prologue, overlap window, tail,
// combine), on a belief after three scans (tools/host_bench_input.py writes the inputs).
// Build: make -C gc-slam_amd host_bench ; run: gc-slam_amd/build/host_bench tools/host_bench_in.bin
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "gcs_host.h"
#include "gcs_math.h"

using namespace gcs;
using namespace gcs::host;
using clk = std::chrono::steady_clock;

template <class F>
double time_us(F f, int reps = 2000) {
  // minimum over 20 batches (the container's CPU is shared: the mean is noise)
  for (int i = 0; i < 50; ++i) f();
  double best = 1e30;
  const int per = reps / 20 > 0 ? reps / 20 : 1;
  for (int b = 0; b < 20; ++b) {
    auto t0 = clk::now();
    for (int i = 0; i < per; ++i) f();
    best = std::min(best, std::chrono::duration<double, std::micro>(clk::now() - t0).count() / per);
  }
  return best;
}

int main(int argc, char** argv) {
  const int M = 512;
  std::vector<double> buf(22 * 22 + 22 + 22 * 22 + M * 7 + 16);
  FILE* f = fopen(argc > 1 ? argv[1] : "tools/host_bench_in.bin", "rb");
  if (!f || fread(buf.data(), sizeof(double), buf.size(), f) != buf.size()) { printf("input?\n"); return 1; }
  fclose(f);
  Belief b{};
  memcpy(b.L, buf.data(), sizeof(b.L));
  memcpy(b.h, buf.data() + 484, sizeof(b.h));
  const double* Q = buf.data() + 506;
  const double* st = buf.data() + 990;
  const double* gy = st + M;
  const double* ac = gy + 3 * M;
  const double* tt = ac + 3 * M;  // t0, t1, t_last, t_scan
  double g[3] = {0, 0, -9.81};
  volatile double sink = 0;
  Belief pred;
  double infl[3], mu_prev[DZ];
  printf("predict_diffusion      %7.2f us\n", time_us([&] { predict_diffusion(b, Q, 0.1, pred, infl, mu_prev); sink += pred.h[0]; }));
  SpdFactor fp;
  printf("spd_factor_lifted 22   %7.2f us\n", time_us([&] { spd_factor_lifted(DZ, pred.L, kEpsLift, fp); sink += fp.Lc[0]; }));
  double x[DZ];
  printf("spd_factor_solve 22    %7.2f us\n", time_us([&] { spd_factor_solve(fp, pred.h, x); sink += x[0]; }));
  double Li[DZ * DZ];
  printf("spd_factor_inverse 22  %7.2f us\n", time_us([&] { spd_factor_inverse(fp, Li); sink += Li[0]; }));
  std::vector<double> w(M);
  printf("smooth_window x512     %7.2f us\n", time_us([&] { for (int i = 0; i < M; ++i) w[i] = smooth_window(st[i], tt[0], tt[1], 0.01); sink += w[3]; }));
  PreintOut pre;
  double z3[3] = {0, 0, 0};
  printf("preintegrate_imu 512   %7.2f us\n", time_us([&] { preintegrate_imu(M, st, gy, ac, w.data(), z3, z3, z3, g, pre); sink += pre.ess; }));
  double dP[27], dn[3];
  printf("imu_meas_iw_suffstats  %7.2f us\n", time_us([&] { imu_meas_iw_suffstats(M, st, gy, ac, w.data(), z3, z3, z3, g, dP, dn); sink += dP[0]; }));
  // IMU/odometry branch
  ImuOdomInputs in{};
  double pose0[6] = {0.1, 0.02, 0, 0, 0, 0.03}, posep[6] = {0.2, 0.03, 0, 0, 0, 0.06}, om[3] = {0, 0, 0.3};
  double Sg[9] = {1e-7, 0, 0, 0, 1e-7, 0, 0, 0, 1e-7}, Sa[9] = {1e-5, 0, 0, 0, 1e-5, 0, 0, 0, 1e-5};
  double cov6[36] = {}, tw[6] = {1, 0, 0, 0, 0, 0.3};
  for (int i = 0; i < 6; ++i) cov6[7 * i] = 1e-4;
  double mu0[DZ] = {}, mu1[DZ] = {};
  in.m = M; in.stamps = st; in.gyro = gy; in.accel = ac; in.w_int = w.data();
  in.dt_imu = 0.005; in.dt_int = 0.2; in.dt_sec = 0.1; in.omega_avg = om;
  in.drot_int = pre.delta_pose + 3; in.dp_int = pre.delta_pose; in.dv_int = pre.delta_v;
  in.pose0 = pose0; in.pose_pred = posep; in.mu_prev = mu0; in.mu_inc = mu1; in.accel_bias = mu1 + 12;
  in.gravity = g; in.Sigma_g = Sg; in.Sigma_a = Sa; in.odom_pose = posep; in.odom_cov = cov6; in.odom_twist = tw;
  in.odom_twist_cov = cov6; in.planar_z_ref = 0; in.planar_z_sigma = 0.1; in.planar_vz_sigma = 0.01;
  static ImuOdomOut io;
  printf("imu_odom_branch        %7.2f us\n", time_us([&] { imu_odom_branch(in, io); sink += io.L[0]; }));
  double out22[DZ * DZ];
  printf("psd_project 22 (fast)  %7.2f us\n", time_us([&] { sink += psd_project(DZ, pred.L, kEpsPsd, out22); }));
  double c6[6];
  printf("psd_project 22 (eigh)  %7.2f us\n", time_us([&] { sink += psd_project(DZ, pred.L, kEpsPsd, out22, c6); }, 200));
  double Qo[DZ * DZ], nu[7], Psi[252], nu2[7], Psi2[252], c2[2], dPs[252] = {}, dnu[7] = {1, 1, 1, 1, 1, 1, 1};
  datasheet_iw_state(nu, Psi);
  printf("process_noise_Q        %7.2f us\n", time_us([&] { process_noise_Q(nu, Psi, Qo); sink += Qo[0]; }));
  printf("process_iw_apply       %7.2f us\n", time_us([&] { process_iw_apply(nu, Psi, dPs, dnu, nu2, Psi2, c2); sink += nu2[0]; }));
  double mnu[3], mPsi[27], mnu2[3], mPsi2[27];
  datasheet_meas_iw_state(mnu, mPsi);
  printf("meas_iw_apply          %7.2f us\n", time_us([&] { meas_iw_apply(mnu, mPsi, dP, dn, mnu2, mPsi2, c2); sink += mnu2[0]; }));
  double ev6[6], V6[36], P6[36];
  for (int i = 0; i < 36; ++i) P6[i] = pred.L[(i / 6) * DZ + i % 6];
  printf("jacobi_eigh 6          %7.2f us\n", time_us([&] { jacobi_eigh(6, P6, ev6, V6); sink += ev6[0]; }));
  double mu[DZ];
  printf("mean_increment         %7.2f us\n", time_us([&] { mean_increment(b, mu); sink += mu[0]; }));
  printf("(sink %g)\n", (double)sink);
  return 0;
}
