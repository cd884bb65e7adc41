"""The bin kernel's dispatch order (k_tile_order / k_tile_order_xcd; gcs_debug_tile_order): only which
block computes which tile changes, so the order must be a permutation of the tiles; the classes of
staged records against the active mean go heaviest first; the XCD form deals each of 8 contiguous
groups of the active tiles (tile order) to the blocks b = g (mod 8), n / 8 tiles per group."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _order(active, work, xcd):
    from gcslam import _lib as L
    lib = L.load()
    n = len(active)
    a = np.ascontiguousarray(active, np.uint8)
    w = np.ascontiguousarray(work, np.uint32)
    out = np.zeros(n, np.int32)
    assert lib.gcs_debug_tile_order(0, a.ctypes.data, w.ctypes.data, n, int(xcd), out.ctypes.data) == 0
    return out


def _classes(active, work):
    a = active.astype(bool)
    A, W = int(a.sum()), int(work[a].astype(np.int64).sum())
    wa = work.astype(np.int64) * A
    c = np.where(2 * wa >= 3 * W, 0, np.where(wa >= W, 1, np.where(2 * wa >= W, 2, 3)))
    return np.where(a, c, 4)


@pytest.mark.parametrize("n,frac,seed", [(8192, 0.57, 0), (8192, 0.0, 1), (8192, 1.0, 2), (4096, 0.003, 3),
                                         (2056, 0.3, 4), (8192, 0.001, 5)])
def test_tile_order_xcd_groups(n, frac, seed):
    rng = np.random.default_rng(seed)
    active = (rng.random(n) < frac).astype(np.uint8)
    # the scan's coverage is a band: make the active tiles clustered as well as random
    if 0 < frac < 1:
        active[n // 3:n // 3 + n // 10] = 1
    work = np.where(active > 0, rng.integers(1, 400, n), 0).astype(np.uint32)
    cls = _classes(active, work)
    base = _order(active, work, xcd=False)
    assert np.array_equal(np.sort(base), np.arange(n))
    # class order, tile order inside a class
    assert np.array_equal(base, np.lexsort((np.arange(n), cls)))
    got = _order(active, work, xcd=True)
    assert np.array_equal(np.sort(got), np.arange(n))                  # a permutation of the tiles
    act = np.flatnonzero(active)
    A, nq = len(act), n // 8
    grp = np.empty(n, int)
    bounds = [(g * A + 7) // 8 for g in range(9)]
    for g in range(8):
        grp[act[bounds[g]:bounds[g + 1]]] = g
    ina = np.flatnonzero(active == 0)
    ib = [g * nq - bounds[g] for g in range(9)]
    for g in range(8):
        grp[ina[ib[g]:ib[g + 1]]] = g
    for g in range(8):
        q = got[g::8]                                                   # the blocks of one XCD
        assert np.all(grp[q] == g)
        assert np.array_equal(q, np.array([j for j in base if grp[j] == g]))  # class order kept inside


def test_tile_order_not_multiple_of_8_falls_back():
    rng = np.random.default_rng(9)
    n = 8191
    active = (rng.random(n) < 0.5).astype(np.uint8)
    work = np.where(active > 0, rng.integers(1, 50, n), 0).astype(np.uint32)
    assert np.array_equal(_order(active, work, True), _order(active, work, False))
