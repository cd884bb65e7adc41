"""numpy restatement of the live primitive path's OT association -- TEST INFRASTRUCTURE ONLY.

FS = fl_ws/src/fl_slam_poc/fl_slam_poc.  Follows
  * associate_primitives_ot          FS/backend/operators/primitive_association.py:239-553
  * unbalanced Sinkhorn, fixed K     primitive_association.py:105-138
  * A_vmf and the sparse pool cost   primitive_association.py:141-197
  * measurement means / kappas       FS/backend/structures/measurement_batch.py:389-411
  * MA-hex tile stencil and packing  FS/common/tiling.py:72-86,148-186
  * AtlasMapView extraction          FS/backend/structures/primitive_map.py:303-322,356-450,475-498
The product path (gc-slam_amd/) never imports this; it is the checker of tests/test_association.py
and tests/test_gpu_association.py.

Sort semantics: the reference's candidate ordering is jax.lax.sort((cost, dt, prim_id, idx),
dimension=1) with lax.sort's default num_keys=1 -- cost is the only key and the sort is stable, so
ties fall to the pool position (dt and prim_id ride along as payload).  Here: np.argsort(kind=
"stable").  _select_topk_slots_fixed (primitive_map.py:319) likewise sorts by -score alone.

Pinning: the reference holds no golden vectors for this operator and JAX is absent here, so the
restatement is pinned by the reference's own budget test (test_budget_assertions.py:91-118,
restated in tests/test_association.py) and closed forms (A_vmf limits, identical primitives cost 0,
balanced Sinkhorn marginals); bit-level parity with JAX is parity unpinned.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GC_EPS_LIFT = 1e-9   # constants.py:71
GC_EPS_MASS = 1e-12  # constants.py
GC_K_ASSOC = 8       # constants.py:356
GC_K_SINKHORN = 50   # constants.py:357
GC_H_TILE = 2.0      # constants.py:408
GC_M_TILE_VIEW = 1024  # constants.py:436
BITS_PER_AXIS = 21   # tiling.py:80
BIAS = 1 << 20       # tiling.py:81
MASK = (1 << BITS_PER_AXIS) - 1
COST_INVALID = 1e12  # primitive_association.py:365


@dataclass
class AssociationConfig:
    """primitive_association.py:206-236 (same fields and defaults; policies as strings)."""
    k_assoc: int = GC_K_ASSOC
    k_sinkhorn: int = GC_K_SINKHORN
    beta: float = 0.5
    epsilon: float = 0.1
    tau_a: float = 0.5
    tau_b: float = 0.5
    cost_subtract_row_min: bool = True
    cost_scale_by_median: bool = False
    a_policy: str = "uniform"           # "uniform" | "weight_proportional"
    b_policy: str = "uniform"
    eps_mass: float = GC_EPS_MASS
    h_tile: float = GC_H_TILE
    r_stencil_tiles_xy: int = 1
    r_stencil_tiles_z: int = 0
    scan_seq: int = 0
    recency_decay_lambda: float = 0.02


def hex_disk_axial(radius):
    """tiling.py:171-186: axial (q, r) of a hex disk, sorted."""
    r = int(radius)
    out = []
    for q in range(-r, r + 1):
        for rr in range(max(-r, -q - r), min(r, -q + r) + 1):
            out.append((q, rr))
    out.sort()
    return out


def tile_ids_from_cells(c1, c2, cz):
    """tiling.py:148-163: pack (c1, c2, cz) into int64 tile ids."""
    c1, c2, cz = (np.asarray(c, dtype=np.int64) for c in (c1, c2, cz))
    u1, u2, uz = (c1 + BIAS) & MASK, (c2 + BIAS) & MASK, (cz + BIAS) & MASK
    return (u1 << (2 * BITS_PER_AXIS)) | (u2 << BITS_PER_AXIS) | uz


def solve3(L, b):
    """jax.vmap(jnp.linalg.solve) over (n, 3, 3) x (n, 3) (LAPACK gesv here as in JAX's CPU path)."""
    return np.linalg.solve(L, b[..., None])[..., 0]


def measurement_means(Lambdas, thetas, etas, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """measurement_batch.py:389-411: mu = (Lambda + eps I)^-1 theta, direction = eta_sum/(|eta_sum| +
    eps), kappa = |eta_sum| (eta_sum over the lobes)."""
    L = np.asarray(Lambdas, dtype=np.float64).reshape(-1, 3, 3) + eps_lift * np.eye(3)[None]
    pos = solve3(L, np.asarray(thetas, dtype=np.float64).reshape(-1, 3))
    e = np.asarray(etas, dtype=np.float64)
    es = e[:, 0, :].copy()
    for b in range(1, e.shape[1]):
        es = es + e[:, b, :]
    kap = np.sqrt((es[:, 0] * es[:, 0] + es[:, 1] * es[:, 1]) + es[:, 2] * es[:, 2])
    return pos, es / (kap[:, None] + eps_mass), kap


def A_vmf(k, eps=1e-12):
    """primitive_association.py:141-149: log(4 pi) + log sinh(k) - log k, stable log-sinh.  k**3 is
    lax.integer_pow (k k k)."""
    k = np.maximum(np.asarray(k, dtype=np.float64), eps)
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        ls = np.where(k > 20.0, k - np.log(2.0), np.where(k >= 1e-2, np.log(np.sinh(k)), np.log(k + (k * k * k) / 6.0)))
    return (np.log(4.0 * np.pi) + ls) - np.log(k)


def sparse_cost(mpos, mdir, mkap, vpos, vdir, vkap, cand, beta=0.5, eig_min=1e-12):
    """primitive_association.py:152-197: ||x_i - x_j||^2 + beta H^2_vMF over candidate pairs."""
    P, D, Kp = vpos[cand], vdir[cand], vkap[cand]
    diff = mpos[:, None, :] - P
    d_pos = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]
    s = mkap[:, None, None] * mdir[:, None, :] + Kp[:, :, None] * D
    km = 0.5 * np.sqrt((s[..., 0] * s[..., 0] + s[..., 1] * s[..., 1]) + s[..., 2] * s[..., 2])
    A_km = A_vmf(np.maximum(km, eig_min), eig_min)
    A_k1 = A_vmf(np.maximum(mkap[:, None], eig_min), eig_min)
    A_k2 = A_vmf(np.maximum(Kp, eig_min), eig_min)
    bc = np.exp(A_km - 0.5 * (A_k1 + A_k2))
    d_dir = np.maximum(0.0, 1.0 - bc)
    valid_dir = (mkap[:, None] > 0.0) & (Kp > 0.0)
    d_dir = np.where(valid_dir, d_dir, 0.0)
    return d_pos + float(beta) * d_dir


def sinkhorn_unbalanced(C, a, b, epsilon, tau_a, tau_b, K):
    """primitive_association.py:105-138 (fixed K iterations, no convergence check)."""
    C = np.asarray(C, dtype=np.float64)
    eps = max(float(epsilon), 1e-12)
    Km = np.exp(-C / eps)
    u = np.ones(C.shape[0])
    v = np.ones(C.shape[1])
    ua = 1.0 / (1.0 + float(tau_a) / eps)
    vb = 1.0 / (1.0 + float(tau_b) / eps)
    for _ in range(int(K)):
        u = (a / (Km @ v + 1e-12)) ** ua
        v = (b / (Km.T @ u + 1e-12)) ** vb
    return (u[:, None] * Km) * v[None, :]


def _p95(x):
    s = np.sort(np.asarray(x, dtype=np.float64).reshape(-1))
    return float(s[min(int(0.95 * s.shape[0]), s.shape[0] - 1)])


def extract_atlas_map_view(tiles, tile_ids, m_tile_view, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """primitive_map.py:356-450 over a dict tile_id -> tile arrays (Lambdas, thetas, etas, weights,
    primitive_ids, valid_mask, last_supported_scan_seq); missing tiles are empty.  Per tile the top
    m_tile_view slots by weight (invalid -> -1e30), stable (primitive_map.py:303-322)."""
    k = int(m_tile_view)
    if k <= 0:
        raise ValueError(f"extract_atlas_map_view: m_tile_view must be > 0, got {m_tile_view}")
    parts = {f: [] for f in ("Lambdas", "thetas", "etas", "weights", "primitive_ids", "valid_mask",
                             "last_supported_scan_seq", "candidate_slots", "candidate_tile_ids")}
    for tid in tile_ids:
        t = tiles[int(tid)]
        if t["weights"].shape[0] < k:
            raise ValueError("m_tile_view exceeds the tile size (the reference's view would be short)")
        score = np.where(t["valid_mask"], t["weights"], -1e30)
        slots = np.argsort(-score, kind="stable")[:k].astype(np.int32)
        for f in ("Lambdas", "thetas", "etas", "weights", "primitive_ids", "valid_mask", "last_supported_scan_seq"):
            parts[f].append(np.asarray(t[f])[slots])
        parts["candidate_slots"].append(slots)
        parts["candidate_tile_ids"].append(np.full((k,), int(tid), dtype=np.int64))
    v = {f: np.concatenate(x, axis=0) for f, x in parts.items()}
    v["valid_mask"] = v["valid_mask"].astype(bool)
    pos, dirs, kap = measurement_means(v["Lambdas"], v["thetas"], v["etas"], eps_lift, eps_mass)
    v.update(positions=pos, directions=dirs, kappas=kap, tile_ids=np.asarray(tile_ids, dtype=np.int64),
             m_tile_view=k)
    return v


def empty_tile(m_tile):
    """primitive_map.py:148-174 (the fields association reads)."""
    return dict(Lambdas=np.zeros((m_tile, 3, 3)), thetas=np.zeros((m_tile, 3)), etas=np.zeros((m_tile, 3, 3)),
                weights=np.zeros(m_tile), primitive_ids=np.zeros(m_tile, dtype=np.int64),
                valid_mask=np.zeros(m_tile, dtype=bool), last_supported_scan_seq=np.zeros(m_tile, dtype=np.int64))


def stencil(cfg):
    """The stencil offsets in the reference's order: z slab outer, axial disk inner (:309-336)."""
    disk = hex_disk_axial(int(cfg.r_stencil_tiles_xy))
    dzs = list(range(-int(cfg.r_stencil_tiles_z), int(cfg.r_stencil_tiles_z) + 1))
    return [(q, r, z) for z in dzs for (q, r) in disk]


def associate_primitives_ot(batch, view, cfg=None, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """primitive_association.py:239-553.  batch: dict Lambdas (N,3,3), thetas, etas (N,L,3), weights,
    valid_mask, n_valid; view: extract_atlas_map_view's dict.  Returns (result dict, cert dict)."""
    cfg = cfg or AssociationConfig()
    K = int(cfg.k_assoc)
    valid = np.asarray(batch["valid_mask"]).astype(np.float64)
    N = valid.shape[0]
    M_valid = int(np.sum(view["valid_mask"]))
    if int(batch["n_valid"]) == 0 or M_valid == 0:
        z = np.zeros((N, K))
        res = dict(responsibilities=z, candidate_pool_indices=np.zeros((N, K), np.int32),
                   candidate_tile_ids=np.zeros((N, K), np.int64), candidate_slots=np.zeros((N, K), np.int64),
                   row_masses=np.zeros(N), cost_matrix=z.copy())
        return res, dict(exact=True, total_cost=0.0)
    mpos, mdir, mkap = measurement_means(batch["Lambdas"], batch["thetas"], batch["etas"], eps_lift, eps_mass)
    vpos, vdir, vkap = view["positions"], view["directions"], view["kappas"]
    # stencil tiles and the pool (:309-348)
    h = max(float(cfg.h_tile), 1e-12)
    s1 = mpos[:, 0]
    s2 = mpos[:, 0] * 0.5 + mpos[:, 1] * (np.sqrt(np.float64(3.0)) * 0.5)
    c1 = np.floor(s1 / h).astype(np.int64)
    c2 = np.floor(s2 / h).astype(np.int64)
    cz = np.floor(mpos[:, 2] / h).astype(np.int64)
    st = stencil(cfg)
    sid = np.stack([tile_ids_from_cells(c1 + q, c2 + r, cz + z) for (q, r, z) in st], axis=1)  # (N, S)
    tids = np.asarray(view["tile_ids"], dtype=np.int64)
    eq = sid[:, :, None] == tids[None, None, :]
    has = eq.any(axis=2)
    tix = np.where(has, np.argmax(eq, axis=2), 0)
    m = int(view["m_tile_view"])
    pool_idx = ((tix.astype(np.int64) * m)[:, :, None] + np.arange(m)[None, None, :]).reshape(N, -1)
    cost_pool = sparse_cost(mpos, mdir, mkap, vpos, vdir, vkap, pool_idx, cfg.beta)
    pool_valid = np.asarray(view["valid_mask"])[pool_idx] & np.repeat(has[:, :, None], m, axis=2).reshape(N, -1)
    cost_pool = np.where(pool_valid, cost_pool, COST_INVALID)
    order = np.argsort(cost_pool, axis=1, kind="stable")  # lax.sort, num_keys=1, stable (:376)
    cand = np.take_along_axis(pool_idx, order, axis=1)[:, :K].astype(np.int32)
    cand = np.where(valid[:, None] > 0.0, cand, 0).astype(np.int32)
    slots = np.asarray(view["candidate_slots"])[cand].astype(np.int64)
    ctid = np.asarray(view["candidate_tile_ids"])[cand].astype(np.int64)
    C = sparse_cost(mpos, mdir, mkap, vpos, vdir, vkap, cand, cfg.beta)
    last = np.asarray(view["last_supported_scan_seq"], dtype=np.int64)[cand]
    dt = np.maximum(0, int(cfg.scan_seq) - last).astype(np.float64)
    C = C + (float(cfg.epsilon) * float(cfg.recency_decay_lambda)) * dt
    if cfg.cost_subtract_row_min:
        C = C - np.min(C, axis=1, keepdims=True)
    if cfg.cost_scale_by_median:
        C = C / (np.median(C) + 1e-12)
    if cfg.a_policy == "uniform":
        sum_a = max(float(np.sum(valid)), cfg.eps_mass)
        a = valid / sum_a
    elif cfg.a_policy == "weight_proportional":
        w = valid * np.asarray(batch["weights"], dtype=np.float64)
        sum_a = max(float(np.sum(w)), cfg.eps_mass)
        a = w / sum_a
    else:
        raise ValueError(f"Unsupported measurement mass policy: {cfg.a_policy}")
    if cfg.b_policy != "uniform":
        raise ValueError(f"Unsupported map mass policy: {cfg.b_policy}. Only UNIFORM is implemented.")
    b = np.ones(K) / float(K)
    sum_b = float(np.sum(b))
    dec = np.exp(-float(cfg.recency_decay_lambda) * dt)
    dec = np.where(dec > 0.0, dec, 0.0)
    b_row = dec / np.maximum(np.sum(dec, axis=1, keepdims=True), cfg.eps_mass)
    pi = sinkhorn_unbalanced(C, a, b, cfg.epsilon, cfg.tau_a, cfg.tau_b, cfg.k_sinkhorn)
    rm = np.sum(pi, axis=1)
    res = dict(responsibilities=pi * (valid[:, None] > 0.0), candidate_pool_indices=cand, candidate_tile_ids=ctid,
               candidate_slots=slots, row_masses=rm, cost_matrix=C)
    cm = np.sum(pi, axis=0)
    tm = float(np.sum(pi))
    cert = dict(exact=False,
                marginal_defect_a=float(np.linalg.norm(rm - a)), marginal_defect_b=float(np.linalg.norm(cm - b)),
                transport_mass_total=tm, sum_a=float(sum_a), sum_b=sum_b, sum_m=float(np.sum(rm)),
                sum_novel=float(np.sum(np.maximum(a - rm, 0.0))), p95_a=_p95(a), p95_b=_p95(b),
                nonzero_a=int(np.sum(a > cfg.eps_mass)), nonzero_b=int(np.sum(b > cfg.eps_mass)),
                b_recency_p95=_p95(b_row), ess_total=float(np.sum(rm) ** 2 / (np.sum(rm ** 2) + cfg.eps_mass)),
                mass_epsilon_ratio=float(cfg.eps_mass) / (tm + float(cfg.eps_mass)),
                total_cost=float(np.sum(pi * C)), alloc_bytes_est=int(N * K * 8 * 4), largest_tensor_shape=(N, K),
                segment_sum_k=K)
    cert["support_frac"] = float(cert["nonzero_a"]) / float(max(N, 1))
    return res, cert


def candidate_stats(meas_valid, view_valid, candidate_pool_indices, candidate_tile_ids, eps_mass=GC_EPS_MASS):
    """The MapUpdateCert's candidate statistics of the map branch (FS/backend/pipeline.py:879-905):
    per measurement row the candidates whose view entry is valid, their distinct tile ids (-1
    excluded), the means of both over the valid rows (denominator max(valid rows, eps_mass)) and the
    p95 of the valid rows' counts with the invalid rows at -1 (sorted, index min(int(0.95 n), n - 1)).
    Returns (tiles_mean, prims_mean, prims_p95); zeros without a valid row."""
    valid = np.asarray(meas_valid).astype(bool)
    if int(valid.sum()) == 0:
        return 0.0, 0.0, 0.0
    cp = np.asarray(candidate_pool_indices)
    cand_valid = np.asarray(view_valid).astype(bool)[cp]
    cand_tiles = np.where(cand_valid, np.asarray(candidate_tile_ids), -1)
    cand_counts = cand_valid.astype(np.float64).sum(1)
    ts = np.sort(cand_tiles, axis=1)
    is_new = np.concatenate([np.ones((ts.shape[0], 1), bool), ts[:, 1:] != ts[:, :-1]], axis=1)
    distinct = (is_new & (ts != -1)).astype(np.float64).sum(1)
    vr = valid.astype(np.float64)
    denom = max(float(vr.sum()), eps_mass)
    cs = np.sort(np.where(valid, cand_counts, -1.0))
    i95 = min(int(0.95 * float(cs.shape[0])), int(cs.shape[0]) - 1)
    return float((distinct * vr).sum() / denom), float((cand_counts * vr).sum() / denom), float(cs[i95])
