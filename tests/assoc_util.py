"""Seeded association scenes (numpy): a primitive atlas of MA-hex tiles, its AtlasMapView (oracle
restatement of extract_atlas_map_view) and a MeasurementBatch whose valid rows sit near map
primitives.  Shared by tests/test_association.py (CPU, small) and tests/test_gpu_association.py."""

from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import association as OA  # noqa: E402

SQ3H = float(np.sqrt(np.float64(3.0)) * 0.5)


def _spd(rng, n, lo, hi):
    A = rng.normal(size=(n, 3, 3))
    Q, _ = np.linalg.qr(A)
    ev = rng.uniform(lo, hi, size=(n, 3))
    return np.einsum("nij,nj,nkj->nik", Q, ev, Q)


def _unit(rng, n):
    d = rng.normal(size=(n, 3))
    return d / np.linalg.norm(d, axis=1, keepdims=True)


def make_scene(seed=0, n_feat=512, n_surfel=1024, n_valid_cam=300, n_valid_lidar=900, m_tile=1024, m_tile_view=1024,
               tile_span=2, h=2.0, fill=(0, 700), n_lobes=3, scan_seq=10, missing_tiles=1, dup_tile=False):
    """Returns (batch dict, view dict, tiles dict)."""
    assert m_tile >= m_tile_view, "a tile view selects m_tile_view of the tile's m_tile slots"
    rng = np.random.default_rng(seed)
    coords = [(a, b, 0) for a in range(-tile_span, tile_span + 1) for b in range(-tile_span, tile_span + 1)]
    tiles = {}
    next_id = 0
    all_pos = []
    for (a, b, c) in coords:
        tid = int(OA.tile_ids_from_cells(a, b, c))
        n = min(int(rng.integers(fill[0], fill[1] + 1)), m_tile)
        t = OA.empty_tile(m_tile)
        slots = rng.permutation(m_tile)[:n]
        s1 = (a + rng.uniform(0, 1, n)) * h
        s2 = (b + rng.uniform(0, 1, n)) * h
        x = s1
        y = (s2 - 0.5 * x) / SQ3H
        z = (c + rng.uniform(0, 1, n)) * h
        mu = np.stack([x, y, z], axis=1)
        Sig = _spd(rng, n, 1e-3, 5e-2)
        Lam = np.linalg.inv(Sig)
        t["Lambdas"][slots] = Lam
        t["thetas"][slots] = np.einsum("nij,nj->ni", Lam, mu)
        kap = rng.uniform(0.1, 100.0, n)
        t["etas"][slots, 0] = kap[:, None] * _unit(rng, n)
        t["etas"][slots, 1] = 0.1 * rng.normal(size=(n, 3))
        t["weights"][slots] = rng.uniform(0.1, 10.0, n)
        t["primitive_ids"][slots] = np.arange(next_id, next_id + n)
        next_id += n
        t["valid_mask"][slots] = True
        t["last_supported_scan_seq"][slots] = rng.integers(0, scan_seq + 3, n)
        tiles[tid] = t
        all_pos.append(mu)
    tile_ids = list(tiles.keys())
    # missing tiles (in the view list but absent from the atlas: empty tiles, primitive_map.py:375-379)
    for q in range(missing_tiles):
        tid = int(OA.tile_ids_from_cells(50 + q, 50, 0))
        tiles[tid] = OA.empty_tile(m_tile)
        tile_ids.append(tid)
    if dup_tile:  # a second copy of the first tile under another id: equal costs, stable order decides
        tid = int(OA.tile_ids_from_cells(60, 60, 0))
        tiles[tid] = {k: v.copy() for k, v in tiles[tile_ids[0]].items()}
        tile_ids.append(tid)
    view = OA.extract_atlas_map_view(tiles, tile_ids, m_tile_view)
    P = np.concatenate(all_pos, axis=0)
    # measurement batch: camera rows [0, n_feat), LiDAR rows [n_feat, n_total); the first
    # n_valid_* rows of each slice valid (measurement_batch.py:137-157 padding elsewhere)
    N = n_feat + n_surfel
    Lam = np.zeros((N, 3, 3))
    th = np.zeros((N, 3))
    eta = np.zeros((N, n_lobes, 3))
    w = np.zeros(N)
    valid = np.zeros(N, dtype=bool)
    rows = list(range(n_valid_cam)) + list(range(n_feat, n_feat + n_valid_lidar))
    nv = len(rows)
    src = P[rng.integers(0, P.shape[0], nv)] if P.shape[0] else rng.uniform(-4, 4, (nv, 3))
    mu = src + 0.05 * rng.normal(size=(nv, 3))
    Sig = _spd(rng, nv, 1e-3, 5e-2)
    L = np.linalg.inv(Sig)
    Lam[rows] = L
    th[rows] = np.einsum("nij,nj->ni", L, mu)
    kap = rng.uniform(0.1, 100.0, nv)
    eta[rows, 0] = kap[:, None] * _unit(rng, nv)
    if n_lobes > 1:
        eta[rows, 1] = 0.1 * rng.normal(size=(nv, 3))
    w[rows] = rng.uniform(0.1, 5.0, nv)
    valid[rows] = True
    batch = dict(Lambdas=Lam, thetas=th, etas=eta, weights=w, valid_mask=valid, n_valid=nv, n_feat=n_feat,
                 n_surfel=n_surfel)
    return batch, view, tiles


def budget_scene():
    """test_budget_assertions.py:22-88: K_ASSOC camera rows at the origin (Lambda = I, eta (1,0,0)), one
    tile with id 0 holding K_ASSOC identical primitives, m_tile_view = K_ASSOC."""
    K = OA.GC_K_ASSOC
    N = K
    Lam = np.zeros((N, 3, 3))
    Lam[:] = np.eye(3)
    eta = np.zeros((N, 3, 3))
    eta[:, 0] = (1.0, 0.0, 0.0)
    batch = dict(Lambdas=Lam, thetas=np.zeros((N, 3)), etas=eta, weights=np.ones(N), valid_mask=np.ones(N, bool),
                 n_valid=N, n_feat=N, n_surfel=0)
    t = OA.empty_tile(K)
    t["Lambdas"][:] = np.eye(3)
    t["etas"][:, 0] = (1.0, 0.0, 0.0)
    t["weights"][:] = 1.0
    t["primitive_ids"][:] = np.arange(K)
    t["valid_mask"][:] = True
    view = OA.extract_atlas_map_view({0: t}, [0], K)
    return batch, view
