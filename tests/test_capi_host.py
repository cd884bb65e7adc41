"""CPU tests of the C-ABI library: it loads, exports every symbol declared in include/gcslam_hip.h,
and its host-side numerics / atlas tables match the oracle (no GPU compute calls here)."""

import ctypes as C
import os
import re

import numpy as np
import pytest

from gcslam import _lib as L
from oracle import ops, se3
from oracle.primitives import psd_project, spd_inverse_lifted, spd_solve_lifted

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol(lib):
    hdr = open(os.path.join(ROOT, "include", "gcslam_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(gcs_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(L.SYMBOLS), declared ^ set(L.SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.gcs_abi_version() == 4


@pytest.mark.parametrize("n", [3, 6, 22])
def test_psd_project_matches_oracle(lib, n):
    rng = np.random.default_rng(n)
    for shift in (-0.5, 0.0, 1.0):
        A = rng.standard_normal((n, n))
        M = np.ascontiguousarray(A @ A.T + shift * np.eye(n) + 1e-3 * rng.standard_normal((n, n)))
        out = np.zeros((n, n))
        cert = np.zeros(6)
        assert lib.gcs_psd_project(n, L.dptr(M), 1e-12, L.dptr(out), L.dptr(cert)) == 0
        ref, rc = psd_project(M)
        scale = np.abs(M).max()
        assert np.allclose(out, ref, atol=1e-13 * scale * n, rtol=0)
        assert cert[0] == pytest.approx(rc[0], abs=1e-13 * scale * n)
        assert cert[1] == pytest.approx(rc[1], rel=1e-12, abs=1e-300)


def _psd3_cases():
    """Symmetric 3x3 inputs of the bin finalize: full-rank scatter, one to three clamped
    eigenvalues (one, two or three points), near-double roots, negative noise, large norms."""
    rng = np.random.default_rng(3)
    out = []
    for scale in (1e-6, 1e-3, 1.0, 1e2):
        for rank in (0, 1, 2, 3):
            for _ in range(40):
                X = rng.standard_normal((rank, 3)) * scale ** 0.5
                M = X.T @ X
                M = M + 1e-17 * scale * rng.standard_normal((3, 3))        # rounding-level noise
                out.append(M)
    for lam in ([1e-3, 1e-3, 0.0], [1.0, 1e-13, -1e-13], [2e-12, 1e-12, 5e-13], [1e-3, 1e-3, 1e-3],
                [1e-3, 2e-12, 0.9e-12], [-1e-14, -1e-14, 1e-4], [6e-13, -4e-13, 3e-13], [9e-13, 0.0, 0.0],
                # (near) double top roots over a clamped bottom one (the closed form of gcs_math.h
                # psd3_deflate), near-triple clusters below eps, a negative triple
                [1e-3, 1e-3 * (1 + 1e-9), -1e-5], [2.0, 2.0, -3.0], [7e-4, 7e-4, 3e-13], [1e-3, 1e-3, -1e-3],
                [5e-13, 5e-13, 5e-13], [5e-13, 5e-13 * (1 + 1e-10), 5e-13], [-2e-13, -2e-13, -2e-13],
                [4e-13, 4e-13, 1e-3]):
        Q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
        out.append(Q @ np.diag(lam) @ Q.T)
    out.append(np.zeros((3, 3)))
    return out


def test_psd_project3_matches_oracle(lib):
    """The device 3x3 PSD projection (host build) against primitives.psd_project (numpy eigh)."""
    for M in _psd3_cases():
        M = np.ascontiguousarray(M)
        out = np.zeros((3, 3))
        d = np.zeros(1)
        assert lib.gcs_psd_project3(L.dptr(M), L.dptr(out), L.dptr(d)) == 0
        ref, rc = psd_project(M)
        s = np.abs(M).max() + 1e-12
        assert np.allclose(out, ref, atol=1e-14 * s + 1e-22, rtol=0), (M, out, ref)
        assert d[0] == pytest.approx(rc[0], abs=1e-14 * s + 1e-22), (M, d[0], rc[0])
        assert np.linalg.eigvalsh(0.5 * (out + out.T)).min() >= 1e-12 * (1 - 1e-6) - 1e-15 * s


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_imu_meas_iw_suffstats_match_oracle(lib, seed):
    """Gyro + accel measurement-noise IW statistics (measurement_noise_iw_jax.py:130-218 with the
    pipeline's dt_imu / valid mask / omega_avg, pipeline.py:522-566) on a padded IMU window."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))
    from gcslam import synthetic
    rng = np.random.default_rng(seed)
    sc = synthetic.make_scan(16, seed)
    w_int = ops.smooth_window_weights(sc["imu_stamps"], sc["t_last_scan"], sc["t_scan"], 0.01 + 0.02 * seed)
    w_int = np.where(sc["imu_stamps"] > 0.0, w_int, 0.0)
    gb, ab = 1e-3 * rng.standard_normal(3), 1e-2 * rng.standard_normal(3)
    rv = rng.standard_normal(3) * 0.3
    g = np.array(ops.GRAVITY_W)
    ref, ref_nu = ops.imu_meas_iw_suffstats(sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], w_int, gb, ab, rv, g)
    args = [np.ascontiguousarray(a, np.float64) for a in (sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], w_int,
                                                            gb, ab, rv, g)]
    dPsi, dnu = np.zeros(27), np.zeros(3)
    assert lib.gcs_imu_meas_iw_suffstats(len(w_int), *[L.dptr(a) for a in args], L.dptr(dPsi), L.dptr(dnu)) == 0
    assert np.allclose(dPsi.reshape(3, 3, 3), ref, rtol=1e-11, atol=1e-22)
    assert np.array_equal(dnu, ref_nu)
    assert np.all(dPsi.reshape(3, 3, 3)[2] == 0.0)                     # lidar block untouched here


def test_meas_iw_apply_matches_oracle(lib):
    """measurement_noise_apply_suffstats_jax (measurement_noise_iw_jax.py:59-100): forgetting, PSD,
    softplus projection of nu into [p + 1.5, 1000]."""
    rng = np.random.default_rng(4)
    nu, Psi = ops.datasheet_measurement_noise_state()
    for it in range(4):
        dP = np.stack([np.outer(v, v) * s for v, s in zip(rng.standard_normal((3, 3)), (1e-8, 1e-4, 1e-3))])
        if it == 3:
            dP[0] -= 1e-6 * np.eye(3)                                        # forces a PSD clamp
        dn = np.array([1.0, 1.0, float(it % 2)])
        ref = ops.measurement_noise_iw_apply(nu, Psi, dP, dn)
        nu_o, Psi_o, c = np.zeros(3), np.zeros(27), np.zeros(2)
        a = [np.ascontiguousarray(x, np.float64).reshape(-1) for x in (nu, Psi, dP, dn)]
        assert lib.gcs_meas_iw_apply(*[L.dptr(x) for x in a], L.dptr(nu_o), L.dptr(Psi_o), L.dptr(c)) == 0
        # unclamped blocks: the host PSD fast path returns sym(M) with delta 0, the oracle's eigh
        # rebuild differs by rounding (~1e-16 |M|), so absolute bars scale with the block norm
        s = np.abs(ref[1]).max()
        assert np.allclose(nu_o, ref[0], rtol=1e-14, atol=0)
        assert np.allclose(Psi_o.reshape(3, 3, 3), ref[1], rtol=1e-12, atol=1e-14 * s)
        assert c[0] == pytest.approx(ref[2][0], rel=1e-9, abs=1e-13 * s) and c[1] == pytest.approx(ref[2][1], rel=1e-12)
        nu, Psi = ref[0], ref[1]


def test_spd_solve_and_inverse_match_oracle(lib):
    rng = np.random.default_rng(11)
    A = rng.standard_normal((22, 22))
    Lm = np.ascontiguousarray(A @ A.T + 0.1 * np.eye(22))
    b = rng.standard_normal(22)
    x = np.zeros(22)
    inv = np.zeros((22, 22))
    lib.gcs_spd_solve_lifted(22, L.dptr(Lm), L.dptr(b), 1e-9, L.dptr(x))
    lib.gcs_spd_inverse_lifted(22, L.dptr(Lm), 1e-9, L.dptr(inv))
    assert np.allclose(x, spd_solve_lifted(Lm, b)[0], rtol=1e-10, atol=1e-12)
    assert np.allclose(inv, spd_inverse_lifted(Lm)[0], rtol=1e-10, atol=1e-12)


def test_svd3_reconstructs_and_matches_numpy_singular_values(lib):
    rng = np.random.default_rng(12)
    for k in range(20):
        H = rng.standard_normal((3, 3))
        if k % 5 == 0:
            H[:, 2] = H[:, 0] + H[:, 1]         # rank 2
        H = np.ascontiguousarray(H)
        U, s, V = np.zeros(9), np.zeros(3), np.zeros(9)
        lib.gcs_svd3(L.dptr(H), L.dptr(U), L.dptr(s), L.dptr(V))
        U, V = U.reshape(3, 3), V.reshape(3, 3)
        assert np.allclose(U @ np.diag(s) @ V.T, H, atol=1e-13)
        assert np.allclose(s, np.linalg.svd(H)[1], atol=1e-13)
        assert np.allclose(U.T @ U, np.eye(3), atol=1e-12) and np.allclose(V.T @ V, np.eye(3), atol=1e-12)


def _mf_rotation_numpy(H):
    """matrix_fisher_evidence.py:215-222: SVD, det fix of U's last column, R = U' Vt."""
    U, s, Vt = np.linalg.svd(H)
    U[:, 2] *= np.sign(np.linalg.det(U @ Vt))
    return U @ Vt


@pytest.mark.parametrize("kind", ["random", "near_rotation", "reflection", "rank2", "zero"])
def test_mf_rotation_matches_svd_rule(lib, kind):
    rng = np.random.default_rng(21)
    for k in range(25):
        if kind == "near_rotation":   # well aligned scans: H close to R diag(s)
            Q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
            Q *= np.sign(np.linalg.det(Q))
            H = Q @ np.diag(rng.uniform(0.5, 50.0, 3)) + 1e-3 * rng.standard_normal((3, 3))
        elif kind == "reflection":
            H = rng.standard_normal((3, 3))
            if np.linalg.det(H) > 0:
                H[:, 0] *= -1
        elif kind == "rank2":
            H = rng.standard_normal((3, 3))
            H[:, 2] = H[:, 0] - 2 * H[:, 1]
        elif kind == "zero":
            H = np.zeros((3, 3))
        else:
            H = rng.standard_normal((3, 3))
        H = np.ascontiguousarray(H)
        R = np.zeros(9)
        lib.gcs_mf_rotation(L.dptr(H), L.dptr(R))
        R = R.reshape(3, 3)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.linalg.det(R) == pytest.approx(1.0, abs=1e-12)
        if kind == "zero":
            assert np.allclose(R, np.eye(3))
        elif kind != "rank2":           # rank-deficient H: R is not unique; only the rule above holds
            assert np.allclose(R, _mf_rotation_numpy(H), atol=1e-11)


def test_predict_and_fusion_match_oracle(lib):
    rng = np.random.default_rng(13)
    b = ops.Belief.identity_prior()
    b.L = b.L + np.diag(rng.uniform(1, 10, 22))
    b.h = rng.standard_normal(22)
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    s = L.belief_to_struct(b.X_anchor, b.stamp_sec, b.z_lin, b.L, b.h)
    o = L.GcsBelief()
    cert = np.zeros(4)
    lib.gcs_predict_diffusion(C.byref(s), L.dptr(np.ascontiguousarray(Q)), 0.1, C.byref(o), L.dptr(cert))
    ref, infl = ops.predict_diffusion(b, Q, 0.1)
    X, st, z, Lm, h = L.struct_to_arrays(o)
    assert np.allclose(Lm, ref.L, rtol=1e-9, atol=1e-9 * np.abs(ref.L).max())
    assert np.allclose(h, ref.h, rtol=1e-9, atol=1e-12)
    Lev = np.ascontiguousarray(np.diag(rng.uniform(0, 5, 22)))
    hev = rng.standard_normal(22)
    p2 = L.GcsBelief()
    d = np.zeros(1)
    lib.gcs_info_fusion_additive(C.byref(o), L.dptr(Lev), L.dptr(hev), 1.0, C.byref(p2), L.dptr(d))
    r2, inf2 = ops.info_fusion_additive(ref, Lev, hev, 1.0)
    assert np.allclose(L.struct_to_arrays(p2)[3], r2.L, rtol=1e-9, atol=1e-9 * np.abs(r2.L).max())


def test_preintegration_matches_oracle(lib):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))
    from gcslam import synthetic
    sc = synthetic.make_scan(256, 0)
    w = ops.smooth_window_weights(sc["imu_stamps"], sc["scan_start_time"], sc["scan_end_time"], 0.01)
    rv, gb, ab = np.array([0.01, -0.02, 0.3]), np.array([1e-3, 0, 0]), np.array([0, 1e-2, 0])
    g = np.array(ops.GRAVITY_W)
    ref = ops.preintegrate_imu(sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], w, rv, gb, ab, g)
    dp = np.zeros(6)
    ess = np.zeros(1)
    args = [np.ascontiguousarray(a, np.float64) for a in (sc["imu_stamps"], sc["imu_gyro"], sc["imu_accel"], w, rv,
                                                            gb, ab, g)]
    lib.gcs_preintegrate_imu(len(w), *[L.dptr(a) for a in args], L.dptr(dp), L.dptr(ess))
    assert np.allclose(dp, ref["delta_pose"], rtol=1e-11, atol=1e-14)
    assert ess[0] == pytest.approx(ref["ess"], rel=1e-13)


@pytest.mark.parametrize("B", [48, 1000, 20000])
def test_atlas_knn_nearest_bit_exact(lib, B):
    d = np.zeros((B, 3))
    lib.gcs_fibonacci_atlas(B, L.dptr(d))
    assert np.allclose(d, ops.fibonacci_atlas(B), atol=2e-15, rtol=0)
    K = min(16, B)
    knn = np.zeros((B, K), np.int32)
    lib.gcs_knn_table(B, L.dptr(d), K, L.iptr(knn))
    assert np.array_equal(knn, ops.bin_knn_table(d, K))           # bit-exact indices
    rng = np.random.default_rng(B)
    q = np.ascontiguousarray(ops.point_directions(rng.standard_normal((3000, 3)), np.zeros(3)))
    q[0] = 0.0                                                     # degenerate zero direction -> bin 0
    nb = np.zeros(3000, np.int32)
    lib.gcs_nearest_bins(B, L.dptr(d), 3000, L.dptr(q), L.iptr(nb))
    assert np.array_equal(nb, ops.nearest_bin(q, d))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import importlib
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(RuntimeError):
        L.load()


def test_ma_hex_stencil_matches_tiling():
    """gcs_ma_hex_stencil (gcs_live_scan's tiles, host code) against ma_hex_stencil_tile_ids (tiling.py:167-209)."""
    from gcslam import _lib as L
    from gcslam.primitive_map import ma_hex_stencil_tile_ids
    lib = L.load()
    rng = np.random.default_rng(3)
    out = np.zeros(L.LIVE_MAX_TILES, np.int64)
    for _ in range(200):
        c = np.ascontiguousarray(rng.normal(0, 50, 3))
        h = float(rng.choice([0.5, 1.0, 2.0, 3.7]))
        rxy, rz = int(rng.integers(0, 3)), int(rng.integers(0, 2))
        n = lib.gcs_ma_hex_stencil(L.dptr(c), h, rxy, rz, out.ctypes.data_as(L.c_int64_p), len(out))
        assert n >= 0
        assert out[:n].tolist() == ma_hex_stencil_tile_ids(c, h, rxy, rz)
