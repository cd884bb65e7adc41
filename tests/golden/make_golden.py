#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (committed; re-run only on a deliberate oracle
change).

What the fixtures are: seeded inputs and the numpy oracle's outputs (oracle/, a float64
restatement of the reference operators; each oracle function cites the reference file:line it
follows).  The reference itself is JAX 0.9.0 and cannot be imported here (ModuleNotFoundError: jax;
SURVEY.md 8(c)), and its own tests hold no golden vectors for these operators, so these fixtures are
ORACLE-GENERATED: they freeze the restatement (tests/test_golden.py re-derives them on CPU) and are
the committed vectors the GPU parity suite checks the HIP path against (tests/test_gpu_parity.py).
Parity with the JAX reference stays "unpinned" (DESIGN.md section 3).

Inputs are stored in the fixture (not regenerated), so a change to gcslam.synthetic cannot move them.

Usage: python tests/golden/make_golden.py
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd")]

from gcslam import synthetic  # noqa: E402  (input generator only)
from oracle import ops, pipeline as opipe  # noqa: E402

ORIGIN = np.array([0.0, 0.0, 0.5])
XI = np.array([0.1, 0.002, 0.0, 0.0, 0.001, 0.03])


def point_stage():
    """Rows 1 + 3 (point_budget.py:50-109, deskew_constant_twist.py:31-69): 3000 raw points, cap 1024
    (stride 3), fixed twist."""
    sc = synthetic.make_scan(3008, 11)
    n, cap = 3000, 1024
    bud = ops.point_budget_resample(sc["points"][:n], sc["timestamps"][:n], sc["weights"][:n], n_points_cap=cap)
    dk = ops.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], sc["scan_start_time"],
                                   sc["scan_end_time"], XI)
    return dict(xyz_record=sc["xyz_record"][:n], timestamps=sc["timestamps"][:n], weights=sc["weights"][:n],
                n_raw=n, cap=cap, t0=sc["scan_start_time"], t1=sc["scan_end_time"], xi=XI,
                budget_indices=bud["indices"].astype(np.int64), budget_weights=bud["weights"],
                total_mass_in=bud["total_mass_in"], deskew_points=dk["points"], deskew_weights=dk["weights"])


def soft_assign_scale():
    """Rows 4-6, scale mode (binning.py:56-209 restricted to K candidates; declared rule DESIGN.md 3):
    B=1024 Fibonacci atlas, K=16, 1024 points."""
    B, K, n = 1024, 16, 1024
    sc = synthetic.make_scan(n, 12)
    bins = ops.fibonacci_atlas(B)
    knn = ops.bin_knn_table(bins, K)
    dk = ops.deskew_constant_twist(sc["points"], sc["timestamps"], sc["weights"], sc["scan_start_time"],
                                   sc["scan_end_time"], XI)
    d = ops.point_directions(dk["points"], ORIGIN)
    tau = ops.tau_for_bins(B)
    sa = ops.bin_soft_assign_scale(d, bins, knn, tau)
    st = ops.scan_bin_moment_match_scale(dk["points"], dk["weights"], sa["indices"], sa["responsibilities"],
                                         ORIGIN, B)
    return dict(xyz_record=sc["xyz_record"], timestamps=sc["timestamps"], weights=sc["weights"],
                t0=sc["scan_start_time"], t1=sc["scan_end_time"], xi=XI, n_bins=B, k=K, tau=tau,
                bins=bins, knn=knn.astype(np.int32), nearest=ops.nearest_bin(d, bins).astype(np.int32),
                cand_ids=sa["indices"].astype(np.int32), resp=sa["responsibilities"], avg_entropy=sa["avg_entropy"],
                **{f"st_{k}": v for k, v in st.items() if isinstance(v, np.ndarray)},
                st_psd_projection_delta=st["psd_projection_delta"], st_ess=st["ess"],
                st_mass_epsilon_ratio=st["mass_epsilon_ratio"])


def soft_assign_dense():
    """Rows 4-6, the reference's dense N x B form at the legacy B=48 (binning.py:56-209)."""
    B, n = 48, 384
    sc = synthetic.make_scan(n, 13)
    bins = ops.fibonacci_atlas(B)
    dk = ops.deskew_constant_twist(sc["points"], sc["timestamps"], sc["weights"], sc["scan_start_time"],
                                   sc["scan_end_time"], XI)
    d = ops.point_directions(dk["points"], ORIGIN)
    sa = ops.bin_soft_assign_dense(d, bins, 0.1)
    st = ops.scan_bin_moment_match_dense(dk["points"], dk["weights"], sa["responsibilities"], ORIGIN)
    return dict(xyz_record=sc["xyz_record"], timestamps=sc["timestamps"], weights=sc["weights"],
                t0=sc["scan_start_time"], t1=sc["scan_end_time"], xi=XI, n_bins=B, tau=0.1, bins=bins,
                resp=sa["responsibilities"], avg_entropy=sa["avg_entropy"],
                **{f"st_{k}": v for k, v in st.items() if isinstance(v, np.ndarray)})


def scan_steps(mode, B, cap, n_raw, n_scans=3):
    """The 14-step per-scan pipeline (pipeline.py:316-1591, bin path) over n_scans consecutive scans
    from the identity prior and an empty map; per-scan outputs stacked."""
    bins = ops.fibonacci_atlas(B)
    knn = ops.bin_knn_table(bins, 16) if mode == "scale" else None
    cfg = opipe.BinPathConfig(n_points_cap=cap, n_bins=B, mode=mode, lidar_origin=tuple(ORIGIN),
                              tau=ops.tau_for_bins(B))
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(B)
    out = dict(mode=mode, n_bins=B, cap=cap, n_raw=n_raw, Q=Q, tau=cfg.tau)
    keys = ("xyz_record", "timestamps", "weights", "imu_stamps", "imu_gyro", "imu_accel", "odom_pose", "odom_cov_se3",
            "odom_twist", "odom_twist_cov")
    rec = {k: [] for k in ("z_t", "X_anchor", "L", "h", "z_lin", "beta", "T", "dPsi", "dnu", "meas_dPsi",
                           "meas_dnu", "L_ev", "h_ev", "scan_N", "map", "L_io", "h_io", "alpha")}
    times = ("scan_start_time", "scan_end_time", "dt_sec", "t_last_scan", "t_scan")
    for k in keys + times:
        out[f"in_{k}"] = []
    for s in range(n_scans):
        sc = synthetic.make_scan(n_raw, 20 + s)
        for k in keys + times:
            out[f"in_{k}"].append(np.asarray(sc[k]))
        r = opipe.process_scan_bin_path(b, sc, Q, cfg, bins, knn, ms)
        rec["z_t"].append(r["z_t"])
        rec["X_anchor"].append(r["belief"].X_anchor)
        rec["L"].append(r["belief"].L)
        rec["h"].append(r["belief"].h)
        rec["z_lin"].append(r["belief"].z_lin)
        rec["beta"].append(r["beta"])
        rec["T"].append(r["total_trigger"])
        rec["dPsi"].append(r["iw_process_dPsi"])
        rec["dnu"].append(r["iw_process_dnu"])
        rec["meas_dPsi"].append(r["iw_meas_dPsi"])
        rec["meas_dnu"].append(r["iw_meas_dnu"])
        rec["L_ev"].append(r["L_evidence"])
        rec["h_ev"].append(r["h_evidence"])
        rec["scan_N"].append(r["scan_bins"]["N"])
        rec["L_io"].append(r["imu_odom"]["L"])   # step 9 IMU/odometry evidence (pipeline.py:745-750)
        rec["h_io"].append(r["imu_odom"]["h"])
        rec["alpha"].append(r["alpha"])
        st = r["map"].stats
        rec["map"].append(np.concatenate([st.S_dir.T, st.S_dir_scatter.reshape(B, 9).T, st.N_dir[None],
                                          st.N_pos[None], st.sum_p.T, st.sum_ppT.reshape(B, 9).T], axis=0))
        b, ms = r["belief"], r["map"]
    for k in list(out):
        if k.startswith("in_"):
            out[k] = np.stack(out[k])
    out.update({f"out_{k}": np.stack([np.asarray(x) for x in v]) for k, v in rec.items()})
    return out


def combine():
    """Hypothesis combine + IW applies (hypothesis.py:51-117, inverse_wishart_jax.py:126-185,
    measurement_noise_iw_jax.py:59-100, backend_node.py:1999-2119) over 4 hypotheses with distinct
    beliefs; the measurement-noise statistics come from 4 synthetic IMU windows."""
    rng = np.random.default_rng(5)
    H = 4
    results = []
    for k in range(H):
        A = rng.normal(size=(22, 22))
        L = A @ A.T + 22.0 * np.eye(22)
        bel = ops.Belief(rng.normal(0, 0.05, 6), 1.0, rng.normal(0, 1e-3, 22), L, rng.normal(size=22))
        dPsi = np.stack([np.outer(v, v) for v in rng.normal(size=(7, 6))])
        results.append(dict(belief=bel, iw_process_dPsi=dPsi, iw_process_dnu=np.ones(7)))
    for k, res in enumerate(results):  # after the draws above, so those inputs are unchanged
        sc = synthetic.make_scan(16, 30 + k)
        w_int = ops.smooth_window_weights(sc["imu_stamps"], sc["t_last_scan"], sc["t_scan"], 0.01)
        res["iw_meas_dPsi"], res["iw_meas_dnu"] = ops.imu_meas_iw_suffstats(
            sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], w_int, 1e-3 * np.ones(3), np.array([0.0, 1e-2, 0.0]),
            np.array([0.01, -0.02, 0.3 * k]), np.array(ops.GRAVITY_W))
    w = np.array([0.5, 0.3, 0.199, 0.001])
    nu, Psi = ops.datasheet_process_noise_state()
    mnu, mPsi = ops.datasheet_measurement_noise_state()
    r = opipe.combine_and_update_noise(results, w, (nu, Psi), 3, (mnu, mPsi))
    return dict(weights=w, L=np.stack([x["belief"].L for x in results]), h=np.stack([x["belief"].h for x in results]),
                z_lin=np.stack([x["belief"].z_lin for x in results]),
                X_anchor=np.stack([x["belief"].X_anchor for x in results]),
                dPsi=np.stack([x["iw_process_dPsi"] for x in results]), nu0=nu, Psi0=Psi,
                out_L=r["combined"]["L"], out_h=r["combined"]["h"], out_z_lin=r["combined"]["z_lin"],
                out_nu=r["iw_state"][0], out_Psi=r["iw_state"][1], out_Q=r["Q"],
                meas_dPsi=np.stack([x["iw_meas_dPsi"] for x in results]),
                meas_dnu=np.stack([x["iw_meas_dnu"] for x in results]), meas_nu0=mnu, meas_Psi0=mPsi,
                out_meas_nu=r["meas_state"][0], out_meas_Psi=r["meas_state"][1], out_meas_cert=r["meas_cert"])


FIXTURES = {
    "point_stage": point_stage,
    "soft_assign_scale": soft_assign_scale,
    "soft_assign_dense": soft_assign_dense,
    "scan_dense_b48": lambda: scan_steps("dense", 48, 2048, 4096),
    "scan_scale_b1024": lambda: scan_steps("scale", 1024, 2048, 4096),
    "combine_h4": combine,
}


def main():
    for name, fn in FIXTURES.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **fn())
        print(f"{path}: {os.path.getsize(path) / 1024:.0f} KiB")


if __name__ == "__main__":
    main()
