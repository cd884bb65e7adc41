"""Device IMU preintegration (k_preint): the window weights, the parallel-prefix
preintegration and the deskew twist against the oracle's sequential restatement
(imu_preintegration.py:20-147, pipeline.py:466-483), and whole scans with the device twist against
the host prologue's.

Tolerances: the device scan re-associates the rotation products and the velocity / position sums
(prefix scans instead of the sequential carry), so the twist differs from the sequential form at
rounding level -- 1e-12 absolute on radians / metres over the window.  A scan that deskews with it
agrees with the host-twist scan at the full-pipeline parity bars (test_full_pipeline_matches_oracle's):
the rounding-level twist change moves points by ~1e-16 m, and the scan's evidence chain (Matrix-Fisher
rotation, planar WLS over eps-weighted bins) amplifies that to ~2e-10 in z_t (measured)."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from gpu_util import device_scan
from oracle import ops, se3
from gcslam.synthetic import scan_kwargs

pytestmark = pytest.mark.gpu

G = np.array([0.0, 0.0, -9.81])


def _device_preint(stamps, gyro, accel, t0, t1, sigma, rotvec, gb, ab, rotation_only=False):
    import ctypes as C
    from gcslam import _lib as L
    lib = L.load()
    arr = [np.ascontiguousarray(x, np.float64) for x in (stamps, gyro, accel, rotvec, gb, ab, G)]
    out = np.zeros(16)
    rc = lib.gcs_debug_preintegrate(0, len(stamps), *(a.ctypes.data for a in arr[:3]), t0, t1, sigma,
                                    *(a.ctypes.data for a in arr[3:]), int(rotation_only), out.ctypes.data)
    assert rc == 0, rc
    return out


def _oracle(stamps, gyro, accel, t0, t1, sigma, rotvec, gb, ab, rotation_only=False):
    w = ops.smooth_window_weights(stamps, t0, t1, sigma)
    pre = ops.preintegrate_imu(stamps, gyro, accel, w, rotvec, gb, ab, G)
    xi = np.array(se3.se3_log(pre["delta_pose"]), np.float64)
    if rotation_only:
        xi[:3] = 0.0
    return xi, pre


def _window(kind, rng):
    if kind == "synthetic":  # the bench's window: 200 Hz over the scan +- margins, zero-padded to 512
        from gcslam import synthetic
        sc = synthetic.make_scan(64, 3)
        return (sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], sc["scan_start_time"], sc["scan_end_time"])
    n = {"short": 37, "single": 1, "long": 1300, "fast": 512}[kind]
    t0 = 100.0
    stamps = t0 - 0.05 + np.sort(rng.uniform(0.0, 0.2, n)) if kind != "long" else t0 - 1.0 + np.arange(n) * 1e-3
    if kind == "short":
        stamps[5] = stamps[4]  # a repeated stamp inside the window (dt = 0 step)
    scale = 6.0 if kind == "fast" else 0.5  # fast: ~1 rad per window
    gyro = rng.normal(0.0, scale, (n, 3))
    accel = rng.normal(0.0, 1.0, (n, 3)) + np.array([0.0, 0.0, 9.81])
    return stamps, gyro, accel, t0, t0 + 0.1


@pytest.mark.parametrize("kind,rotation_only", [("synthetic", False), ("short", False), ("single", False),
                                                ("long", False), ("fast", False), ("synthetic", True)])
def test_k_preint_matches_oracle(kind, rotation_only):
    rng = np.random.default_rng(7)
    stamps, gyro, accel, t0, t1 = _window(kind, rng)
    sigma = 0.013
    rotvec = np.array([0.05, -0.3, 1.1])
    gb = np.array([0.001, -0.002, 0.0005])
    ab = np.array([0.02, 0.01, -0.03])
    out = _device_preint(stamps, gyro, accel, t0, t1, sigma, rotvec, gb, ab, rotation_only)
    xi, pre = _oracle(stamps, gyro, accel, t0, t1, sigma, rotvec, gb, ab, rotation_only)
    np.testing.assert_allclose(out[:6], xi, rtol=0, atol=1e-12)
    assert out[6] == pytest.approx(pre["ess"], rel=1e-13)
    np.testing.assert_allclose(out[7:13], pre["delta_pose"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(out[13:16], pre["delta_v"], rtol=0, atol=1e-11)
    if kind == "single":  # one sample: dt = 0, an exact identity -- the zero twist, ess = w
        assert np.all(out[:6] == 0.0) and np.all(out[7:16] == 0.0)


def test_scan_device_preint_matches_host_prologue():
    """gcs_scan with GCS_DEBUG_DEVICE_PREINT = 1 (k_preint on the stream ahead of k_points, the twist
    through the device word) against the host prologue, three consecutive scans: the posterior, the
    scan statistics and the map agree at the full-pipeline bars, and the ess certificate (cert[10])
    to 1e-13."""
    from gcslam import _lib as L
    from gcslam import synthetic as syn
    from gcslam.context import HypothesisContext
    outs = []
    for dev in (1, 0):
        ctx = HypothesisContext(lidar_origin=(0.0, 0.0, 0.5), max_raw_points=1 << 20, n_bins=20000,
                                n_points_cap=8192, mode="scale")
        ctx.set_debug(L.DEBUG_DEVICE_PREINT, dev)
        res = []
        for k in range(3):
            sc = syn.make_scan(8192, 51 + k)
            rec, t, w = device_scan(sc)
            o = ctx.scan(rec, 16, t, w, 8192, **scan_kwargs(sc))
            res.append((ctx.get_scan_stats(), ctx.get_map()[0], np.array(o.belief.L[:]), np.array(o.z_t[:]),
                        np.array(o.cert[:])))
        outs.append(res)
        ctx.close()
    for k in range(3):
        (sa, ma, La, za, ca), (sb, mb, Lb, zb, cb) = outs[0][k], outs[1][k]
        assert ca[10] == pytest.approx(cb[10], rel=1e-13)
        np.testing.assert_allclose(za, zb, rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(La, Lb, rtol=1e-7, atol=1e-7 * np.abs(Lb).max())
        np.testing.assert_allclose(sa, sb, rtol=1e-7, atol=1e-9 * max(np.abs(sb).max(), 1.0))
        np.testing.assert_allclose(ma, mb, rtol=1e-7, atol=1e-9 * max(np.abs(mb).max(), 1.0))
