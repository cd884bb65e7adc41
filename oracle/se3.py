"""SO(3)/SE(3) maps -- numpy restatement of
``fl_ws/src/fl_slam_poc/fl_slam_poc/common/geometry/se3_jax.py`` (test oracle only).

Every jnp.where branch is reproduced as a numpy where/if on the same
predicates so small-angle and near-pi behaviour match the reference.
"""

from __future__ import annotations

import numpy as np

SMALL_ANGLE_THRESHOLD = 1e-7  # se3_jax.py:29
NEAR_PI_THRESHOLD = 1e-7      # se3_jax.py:33


def skew(v):
    """se3_jax.py:41-52"""
    v = np.asarray(v, dtype=np.float64)
    return np.array([[0.0, -v[2], v[1]],
                     [v[2], 0.0, -v[0]],
                     [-v[1], v[0], 0.0]], dtype=np.float64)


def _dot3(a, b):
    # jnp.dot on 3-vectors; evaluated left to right without fma.
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def so3_exp(omega):
    """Rodrigues. se3_jax.py:260-300"""
    omega = np.asarray(omega, dtype=np.float64).reshape(3)
    theta_sq = _dot3(omega, omega)
    theta = np.sqrt(theta_sq)
    K = skew(omega)
    K_sq = K @ K
    small = theta < SMALL_ANGLE_THRESHOLD
    safe_theta = 1.0 if small else theta
    safe_theta_sq = 1.0 if theta_sq < SMALL_ANGLE_THRESHOLD ** 2 else theta_sq
    sin_coeff = 1.0 if small else np.sin(safe_theta) / safe_theta
    cos_coeff = 0.5 if small else (1.0 - np.cos(safe_theta)) / safe_theta_sq
    return np.eye(3) + sin_coeff * K + cos_coeff * K_sq


def so3_log(R):
    """Inverse Rodrigues with softmax near-pi axis. se3_jax.py:303-365"""
    R = np.asarray(R, dtype=np.float64)
    cos_theta = 0.5 * (np.trace(R) - 1.0)
    cos_theta = min(max(cos_theta, -1.0), 1.0)
    theta = np.arccos(cos_theta)
    skew_part = 0.5 * (R - R.T)
    vex_skew = np.array([skew_part[2, 1], skew_part[0, 2], skew_part[1, 0]])
    omega_small = vex_skew
    sin_theta = np.sin(theta)
    safe_sin = 1.0 if abs(sin_theta) < SMALL_ANGLE_THRESHOLD else sin_theta
    omega_general = (theta / (2.0 * safe_sin)) * (2.0 * vex_skew)
    diag_plus_1 = np.diag(R) + 1.0
    z = 50.0 * diag_plus_1
    e = np.exp(z - z.max())
    w = e / e.sum()
    axis_cols = np.stack([R[:, 0] + np.array([1.0, 0, 0]),
                          R[:, 1] + np.array([0, 1.0, 0]),
                          R[:, 2] + np.array([0, 0, 1.0])], axis=0)
    axis_col = w[0] * axis_cols[0] + w[1] * axis_cols[1] + w[2] * axis_cols[2]
    axis_norm = np.linalg.norm(axis_col)
    safe_axis_norm = 1.0 if axis_norm < SMALL_ANGLE_THRESHOLD else axis_norm
    omega_pi = (axis_col / safe_axis_norm) * theta
    if theta < SMALL_ANGLE_THRESHOLD:
        return omega_small
    if abs(theta - np.pi) < NEAR_PI_THRESHOLD:
        return omega_pi
    return omega_general


def _BC(theta, theta_sq):
    small = theta < SMALL_ANGLE_THRESHOLD
    safe_theta = 1.0 if small else theta
    safe_theta_sq = 1.0 if theta_sq < SMALL_ANGLE_THRESHOLD ** 2 else theta_sq
    safe_theta_cu = safe_theta_sq * safe_theta
    B = 0.5 - theta_sq / 24.0 if small else (1.0 - np.cos(safe_theta)) / safe_theta_sq
    C = 1.0 / 6.0 - theta_sq / 120.0 if small else (safe_theta - np.sin(safe_theta)) / safe_theta_cu
    return B, C


def se3_exp(xi):
    """se3_jax.py:474-504 -> [t, phi]"""
    xi = np.asarray(xi, dtype=np.float64).reshape(6)
    rho, phi = xi[:3], xi[3:6]
    theta_sq = _dot3(phi, phi)
    theta = np.sqrt(theta_sq)
    K = skew(phi)
    K_sq = K @ K
    B, C = _BC(theta, theta_sq)
    V = np.eye(3) + B * K + C * K_sq
    return np.concatenate([V @ rho, phi])


def _se3_V_inv(phi):
    """se3_jax.py:169-207"""
    phi = np.asarray(phi, dtype=np.float64).reshape(3)
    theta_sq = _dot3(phi, phi)
    theta = np.sqrt(theta_sq)
    K = skew(phi)
    K_sq = K @ K
    eps = 1e-12
    small = theta < SMALL_ANGLE_THRESHOLD
    safe_theta = 1.0 if small else theta
    safe_theta_sq = 1.0 if theta_sq < SMALL_ANGLE_THRESHOLD ** 2 else theta_sq
    denom = 2.0 * safe_theta * np.sin(safe_theta) + eps
    D = (1.0 / 12.0 + theta_sq / 720.0) if small else (1.0 / safe_theta_sq) - (1.0 + np.cos(safe_theta)) / denom
    return np.eye(3) - 0.5 * K + D * K_sq


def se3_log(T):
    """se3_jax.py:210-245"""
    T = np.asarray(T, dtype=np.float64).reshape(6)
    R = so3_exp(T[3:6])
    phi = so3_log(R)
    rho = _se3_V_inv(phi) @ T[:3]
    return np.concatenate([rho, phi])


def se3_compose(a, b):
    """se3_jax.py:405-424"""
    a = np.asarray(a, dtype=np.float64).reshape(6)
    b = np.asarray(b, dtype=np.float64).reshape(6)
    Ra, Rb = so3_exp(a[3:6]), so3_exp(b[3:6])
    return np.concatenate([a[:3] + Ra @ b[:3], so3_log(Ra @ Rb)])


def se3_inverse(a):
    """se3_jax.py:427-438"""
    a = np.asarray(a, dtype=np.float64).reshape(6)
    R = so3_exp(a[3:6])
    Rinv = R.T
    return np.concatenate([-Rinv @ a[:3], so3_log(Rinv)])


# ----------------------------------------------------------------------------
# Batched per-point deskew transform (the vmapped body of
# deskew_constant_twist.py:51-58): T = se3_exp(alpha * xi); p0 = R^T (p - t).
# Vectorised restatement of se3_exp + so3_exp with the same branch predicates.
# ----------------------------------------------------------------------------

def deskew_points(points, alpha, xi):
    points = np.asarray(points, dtype=np.float64)
    alpha = np.asarray(alpha, dtype=np.float64)
    xi = np.asarray(xi, dtype=np.float64).reshape(6)
    rho = alpha[:, None] * xi[None, :3]
    phi = alpha[:, None] * xi[None, 3:6]
    theta_sq = phi[:, 0] * phi[:, 0] + phi[:, 1] * phi[:, 1] + phi[:, 2] * phi[:, 2]
    theta = np.sqrt(theta_sq)
    small = theta < SMALL_ANGLE_THRESHOLD
    safe_theta = np.where(small, 1.0, theta)
    safe_theta_sq = np.where(theta_sq < SMALL_ANGLE_THRESHOLD ** 2, 1.0, theta_sq)
    safe_theta_cu = safe_theta_sq * safe_theta
    cs, sn = np.cos(safe_theta), np.sin(safe_theta)
    B = np.where(small, 0.5 - theta_sq / 24.0, (1.0 - cs) / safe_theta_sq)
    C = np.where(small, 1.0 / 6.0 - theta_sq / 120.0, (safe_theta - sn) / safe_theta_cu)
    K = np.zeros((points.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -phi[:, 2], phi[:, 1]
    K[:, 1, 0], K[:, 1, 2] = phi[:, 2], -phi[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -phi[:, 1], phi[:, 0]
    K_sq = np.einsum("nij,njk->nik", K, K)
    I = np.eye(3)[None]
    V = I + B[:, None, None] * K + C[:, None, None] * K_sq
    t = np.einsum("nij,nj->ni", V, rho)
    # so3_exp(phi) of the se3_exp output (same phi)
    sin_coeff = np.where(small, 1.0, sn / safe_theta)
    cos_coeff = np.where(small, 0.5, (1.0 - cs) / safe_theta_sq)
    R = I + sin_coeff[:, None, None] * K + cos_coeff[:, None, None] * K_sq
    return np.einsum("nji,nj->ni", R, points - t)
