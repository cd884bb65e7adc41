"""SURVEY.md 8(f) row 3 on the device: the step-9 IMU / odometry evidence family (FS/backend/pipeline.py:
442-566, 595-776 and the eleven factor files) as one workgroup (gcs_imu_odom.hip, through the C-ABI
gcs_imu_odom_evidence_device), against the numpy oracle (oracle/imu_odom.py) at the host branch's bars on
the reference's own raw Kimera IMU / odometry windows and on synthetic ones; then whole scans with the
device branch (GCS_DEBUG_DEVICE_IMU_ODOM) against the same scans with the host branch."""

import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from golden_util import load
from gcslam import synthetic
from oracle import se3
from test_imu_odom import TOL, _inputs, _oracle

pytestmark = pytest.mark.gpu

ORIGIN = (0.0, 0.0, 0.5)


def _ctx():
    from gcslam.context import HypothesisContext
    return HypothesisContext(n_bins=48, n_points_cap=2048, max_raw_points=4096, mode="dense", lidar_origin=ORIGIN)


def _device(ctx, d):
    from gcslam import _lib as L
    keep = {k: np.ascontiguousarray(v, np.float64) for k, v in d.items() if isinstance(v, np.ndarray)}
    s = L.GcsImuOdomInputs()
    s.m = keep["stamps"].shape[0]
    for k, v in keep.items():
        setattr(s, k, v.ctypes.data)
    s.t_last_scan, s.t_scan, s.dt_sec = d["t_last_scan"], d["t_scan"], d["dt_sec"]
    s.planar_z_ref, s.planar_z_sigma, s.planar_vz_sigma = 0.0, 0.1, 0.01
    Lm, h, cert = np.zeros(484), np.zeros(22), np.zeros(L.IMU_ODOM_CERT_LEN)
    rc = ctx.lib.gcs_imu_odom_evidence_device(ctx.h, C.byref(s), L.dptr(Lm), L.dptr(h), L.dptr(cert))
    assert rc == 0, ctx.lib.gcs_last_error(ctx.h)
    return Lm.reshape(22, 22), h, cert


def _check(ctx, d):
    L_o, h_o, named, info, dt_int, dt_imu, om = _oracle(d)
    L_d, h_d, cert = _device(ctx, d)
    sc = np.abs(L_o).max()
    np.testing.assert_allclose(L_d, L_o, rtol=1e-9, atol=1e-12 * sc)
    np.testing.assert_allclose(h_d, h_o, rtol=1e-9, atol=1e-12 * max(np.abs(h_o).max(), 1.0))
    np.testing.assert_allclose(cert[0], info["trigger"], rtol=1e-9)
    np.testing.assert_allclose(cert[1:7], [info["ess_weighted"], info["kappa"], info["transport_sigma"],
                                           info["imu_scale"], info["odom_scale"], info["mean_reliability"]], **TOL)
    np.testing.assert_allclose(cert[7:10], [named["odom"]["nll_per_ess"], named["imu"]["nll_per_ess"],
                                            named["gyro"]["nll_per_ess"]], rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(cert[10:15], [dt_int, dt_imu, *om], **TOL)
    assert np.all(np.isfinite(L_d)) and np.allclose(L_d, L_d.T, atol=1e-9 * sc)


def test_device_branch_kimera_windows_match_oracle():
    g = load("kimera_imu_odom_windows")
    rng = np.random.default_rng(3)
    ctx = _ctx()
    try:
        for k in range(1, g["t_scan"].shape[0]):
            pose0 = g["odom_pose"][k - 1]
            pose_pred = g["odom_pose"][k] + np.concatenate([rng.normal(0, 0.01, 3), rng.normal(0, 0.002, 3)])
            mu_prev = np.concatenate([rng.normal(0, 1e-3, 6), g["odom_twist"][k - 1][:3], rng.normal(0, 1e-4, 13)])
            mu_inc = np.concatenate([rng.normal(0, 1e-3, 6), g["odom_twist"][k][:3], rng.normal(0, 1e-3, 3),
                                     rng.normal(0, 1e-2, 3), rng.normal(0, 1e-4, 7)])
            d = _inputs(g["imu_stamps"][k], g["imu_gyro"][k], g["imu_accel"][k], float(g["t_last_scan"][k]),
                        float(g["t_scan"][k]), 0.1, pose0, pose_pred, mu_prev, mu_inc, g["odom_pose"][k],
                        g["odom_cov_se3"], g["odom_twist"][k], g["odom_twist_cov"])
            _check(ctx, d)
    finally:
        ctx.close()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_device_branch_synthetic_windows_match_oracle(seed):
    sc = synthetic.make_scan(16, 40 + seed)
    rng = np.random.default_rng(seed)
    pose0 = np.concatenate([rng.normal(0, 0.2, 3), rng.normal(0, 0.1, 3)])
    pose_pred = se3.se3_compose(pose0, np.array([0.1, 0.0, 0.0, 0.0, 0.0, 0.03]))
    d = _inputs(sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], sc["t_last_scan"], sc["t_scan"], 0.1, pose0,
                pose_pred, rng.normal(0, 1e-2, 22), rng.normal(0, 1e-2, 22), sc["odom_pose"], sc["odom_cov_se3"],
                sc["odom_twist"], sc["odom_twist_cov"], sigma_warp=0.02)
    ctx = _ctx()
    try:
        _check(ctx, d)
        # a window past the kernel's 1,024 samples fails loudly (no host fallback)
        rep = -(-2000 // d["stamps"].shape[0])
        d2 = dict(d, stamps=np.tile(d["stamps"], rep), gyro=np.tile(d["gyro"], (rep, 1)),
                  accel=np.tile(d["accel"], (rep, 1)), w_int=np.tile(d["w_int"], rep))
        with pytest.raises(AssertionError, match="1024"):
            _device(ctx, d2)
    finally:
        ctx.close()


@pytest.mark.parametrize("mode,B,cap,n", [("dense", 48, 2048, 4096), ("scale", 20000, 8192, 8192)])
def test_scans_with_device_branch_match_host_branch(mode, B, cap, n):
    """Three consecutive 14-step scans with the device IMU / odometry branch against the same scans with
    the host branch: z_t, the belief, the IMU / odometry evidence and its certificates."""
    from gcslam import _lib as L
    from gcslam.context import HypothesisContext
    from gcslam.synthetic import scan_kwargs
    runs = []
    for dev in (0, 1):
        ctx = HypothesisContext(n_bins=B, n_points_cap=cap, max_raw_points=n, mode=mode, lidar_origin=ORIGIN)
        ctx.set_debug(L.DEBUG_DEVICE_IMU_ODOM, dev)
        out = []
        try:
            for s in range(3):
                sc = synthetic.make_scan(n, 120 + s)
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                o = ctx.scan(rec, 16, t, w, n, **scan_kwargs(sc))
                X, _, z, Lm, h = ctx.get_belief()
                out.append(dict(z_t=np.array(o.z_t[:]), L=Lm, h=h, Lio=np.array(o.L_imu_odom[:]),
                                hio=np.array(o.h_imu_odom[:]), certs=np.array(o.imu_odom_certs[:]),
                                cert=np.array(o.cert[:])))
        finally:
            ctx.close()
        runs.append(out)
    # the evidence itself at the device-vs-host bars of the windows above, on every scan; the scan's
    # downstream outputs at the pipeline's multi-scan bar (tests/test_gpu_fullsize.py: rtol 1e-7) on the
    # first two scans, and the pose-6 conditioning (cert[49], an eigenvalue ratio of the summed evidence:
    # a scale-mode scan measured 1.1e-5 relative between the two branches' sum orders) at 1e-4.  The loop
    # feeds each branch's z_t back into its own deskew and map, and the reference's nearest-bin step is
    # discontinuous: a point within ~1e-9 of a Voronoi boundary between two bins changes its candidate
    # set under a 1e-9 m pose change.  By the third scale-mode scan (20,000 bins, 8,192 points) that had
    # moved z_t by 1.8e-7 m and single L entries by up to 1.2e-5 of max|L| (profiles/r06/imu_odom/), so
    # that scan's z_t / L take atol 1e-6 m / 1e-4 max|L|.
    bad = []
    for s in range(3):
        a, b = runs[0][s], runs[1][s]
        late = s >= 2
        checks = [("Lio", 1e-9, 1e-12 * np.abs(a["Lio"]).max()), ("hio", 1e-9, 1e-12 * max(np.abs(a["hio"]).max(), 1.0)),
                  ("certs", 1e-8, 1e-12), ("z_t", 1e-7, 1e-6 if late else 1e-9),
                  ("L", 1e-7, (1e-4 if late else 1e-7) * np.abs(a["L"]).max())]
        for k, rt, at in checks:
            if not np.allclose(b[k], a[k], rtol=rt, atol=at):
                i = int(np.argmax(np.abs(b[k] - a[k]) - rt * np.abs(a[k])))
                bad.append((s, k, dict(at=i, host=float(a[k].flat[i]), device=float(b[k].flat[i]),
                                       max_abs=float(np.abs(b[k] - a[k]).max()))))
        ca, cb = a["cert"][42:57], b["cert"][42:57]
        rt = np.full(15, 1e-7)
        rt[49 - 42] = 1e-4
        if not np.all(np.abs(cb - ca) <= rt * np.abs(ca) + 1e-12):
            bad.append((s, "cert[42:57]", [float(x) for x in (np.abs(cb - ca) / (np.abs(ca) + 1e-12))]))
    assert not bad, bad
