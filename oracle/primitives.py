"""Branch-free numeric primitives -- numpy restatement of
``fl_ws/src/fl_slam_poc/fl_slam_poc/common/primitives.py`` (test oracle only)."""

from __future__ import annotations

import numpy as np

F64_EPS = float(np.finfo(np.float64).eps)


def psd_project(M, eps_psd=1e-12):
    """domain_projection_psd_core, primitives.py:80-123.

    Returns (M_psd, cert_vec) with cert_vec =
    [projection_delta, sym_delta, eig_min, eig_max, cond, near_null_count].
    """
    M = np.asarray(M, dtype=np.float64)
    M_sym = 0.5 * (M + M.T)
    sym_delta = np.linalg.norm(M_sym - M, ord="fro")
    w, V = np.linalg.eigh(M_sym)
    vals = np.maximum(w, eps_psd)
    M_psd = V @ np.diag(vals) @ V.T
    delta = np.linalg.norm(M_psd - M_sym, ord="fro")
    near_null = float(np.sum(vals < 10.0 * eps_psd))
    eig_min, eig_max = vals.min(), vals.max()
    return M_psd, np.array([delta, sym_delta, eig_min, eig_max, eig_max / eig_min, near_null])


def psd_project_batch(M, eps_psd=1e-12):
    """vmap(domain_projection_psd_core) over (B,3,3) -- primitives.py:126-138."""
    M = np.asarray(M, dtype=np.float64)
    M_sym = 0.5 * (M + np.swapaxes(M, -1, -2))
    w, V = np.linalg.eigh(M_sym)
    vals = np.maximum(w, eps_psd)
    M_psd = np.einsum("bij,bj,bkj->bik", V, vals, V)
    delta = np.sqrt(np.sum((M_psd - M_sym) ** 2, axis=(-1, -2)))
    return M_psd, delta


def spd_solve_lifted(L, b, eps_lift=1e-9):
    """spd_cholesky_solve_lifted_core, primitives.py:141-166 -> (x, lift_strength)."""
    L = np.asarray(L, dtype=np.float64)
    d = L.shape[0]
    Lc = np.linalg.cholesky(L + eps_lift * np.eye(d))
    y = np.linalg.solve(Lc, b)      # triangular solves restated as dense solves
    x = np.linalg.solve(Lc.T, y)
    return x, eps_lift * d


def spd_inverse_lifted(L, eps_lift=1e-9):
    """spd_cholesky_inverse_lifted_core, primitives.py:169-192."""
    L = np.asarray(L, dtype=np.float64)
    d = L.shape[0]
    Lc = np.linalg.cholesky(L + eps_lift * np.eye(d))
    Linv_c = np.linalg.solve(Lc, np.eye(d))
    return Linv_c.T @ Linv_c, eps_lift * d


def inv_mass(m, eps_mass=1e-12):
    """inv_mass_core, primitives.py:195-212."""
    denom = np.asarray(m, dtype=np.float64) + eps_mass + F64_EPS
    return 1.0 / denom, eps_mass / denom


def sigmoid(x):
    x = np.asarray(x, dtype=np.float64)
    return np.where(x >= 0, 1.0 / (1.0 + np.exp(-np.abs(x))),
                    np.exp(-np.abs(x)) / (1.0 + np.exp(-np.abs(x))))


def softplus(x):
    x = np.asarray(x, dtype=np.float64)
    return np.logaddexp(0.0, x)
