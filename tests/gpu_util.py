"""Shared helpers for the GPU parity tests (test infrastructure; imports the oracle as checker)."""

import numpy as np

from oracle import ops

SCAN_FIELD_NAMES = ["N", "s_dir", "S_dir_scatter", "p_bar", "Sigma_p", "kappa_scan"]


def scan_fields(st):
    """Oracle ScanBinStats -> field-major (26, B) like the device layout (gcs_layout.h)."""
    B = st["N"].shape[0]
    return np.concatenate([st["N"][None], st["s_dir"].T, st["S_dir_scatter"].reshape(B, 9).T, st["p_bar"].T,
                           st["Sigma_p"].reshape(B, 9).T, st["kappa_scan"][None]], axis=0)


def map_fields(m: ops.MapBinStats):
    B = m.N_dir.shape[0]
    return np.concatenate([m.S_dir.T, m.S_dir_scatter.reshape(B, 9).T, m.N_dir[None], m.N_pos[None], m.sum_p.T,
                           m.sum_ppT.reshape(B, 9).T], axis=0)


def map_from_fields(f):
    B = f.shape[1]
    return ops.MapBinStats(S_dir=f[0:3].T.copy(), S_dir_scatter=f[3:12].T.reshape(B, 3, 3).copy(), N_dir=f[12].copy(),
                           N_pos=f[13].copy(), sum_p=f[14:17].T.copy(), sum_ppT=f[17:26].T.reshape(B, 3, 3).copy())


def derived_fields(mu, kappa, centroid, Sigma_c):
    B = kappa.shape[0]
    return np.concatenate([mu.T, kappa[None], centroid.T, Sigma_c.reshape(B, 9).T], axis=0)


def scan_from_fields(f):
    B = f.shape[1]
    return dict(N=f[0].copy(), s_dir=f[1:4].T.copy(), S_dir_scatter=f[4:13].T.reshape(B, 3, 3).copy(),
                p_bar=f[13:16].T.copy(), Sigma_p=f[16:25].T.reshape(B, 3, 3).copy(), kappa_scan=f[25].copy())


def assert_close(name, got, ref, rtol, atol):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    err = np.abs(got - ref)
    tol = atol + rtol * np.abs(ref)
    bad = err > tol
    if np.any(bad):
        i = np.unravel_index(np.argmax(err - tol), err.shape)
        raise AssertionError(f"{name}: {bad.sum()} / {bad.size} outside tol; worst at {i}: got {got[i]!r} "
                             f"ref {ref[i]!r} (rtol {rtol}, atol {atol})")


# the map's field groups (map_fields order): S_dir, S_dir_scatter, N_dir, N_pos, sum_p, sum_ppT
MAP_GROUPS = ((0, 3), (3, 12), (12, 13), (13, 14), (14, 17), (17, 26))


def assert_close_groupwise(name, got, ref, groups, rtol, atol):
    """Norm-wise per bin and field group: |got - ref| <= atol + rtol * max |ref| over the group's
    entries of that bin.  The pushforward rotates each bin's moments into the fused frame, so an
    off-diagonal entry can be a cancellation of terms a thousand times its size (C3 bin 497,640:
    sum_ppT yx = 0.039 beside yy = 1,138); its rounding scales with the group, not with itself."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    for g0, g1 in groups:
        scale = np.abs(ref[g0:g1]).max(axis=0, keepdims=True)
        assert_close(f"{name} fields {g0}:{g1}", got[g0:g1], ref[g0:g1], 0.0, atol + rtol * scale)


def device_scan(sc, device="cuda:0"):
    import torch
    rec = torch.from_numpy(np.ascontiguousarray(sc["xyz_record"])).to(device)
    t = torch.from_numpy(np.ascontiguousarray(sc["timestamps"])).to(device)
    w = torch.from_numpy(np.ascontiguousarray(sc["weights"])).to(device)
    return rec, t, w
