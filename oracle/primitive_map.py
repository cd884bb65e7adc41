"""numpy restatement of the live primitive path's map maintenance -- TEST INFRASTRUCTURE ONLY.

FS = fl_ws/src/fl_slam_poc/fl_slam_poc.  Follows FS/backend/structures/primitive_map.py:
  * PrimitiveMapTile / create_empty_tile      :98-174
  * _select_topk_slots_fixed                  :303-322   (view: top weights, stable on -score)
  * _select_lowest_mass_slots_fixed           :325-353   (insert: eviction targets, stable on mass)
  * extract_atlas_map_view + view core        :356-450, :474-498
  * primitive_map_insert_masked               :807-981
  * primitive_map_fuse                        :992-1163
  * primitive_map_cull                        :1175-1304 (weight threshold; max_primitives unsupported)
  * primitive_map_forget                      :1314-1384
  * primitive_map_recency_inflate             :1400-1484
  * primitive_map_merge_reduce                :1501-2031
The product path (gc-slam_amd/) never imports this; it is the checker of tests/test_primitive_map.py
and tests/test_gpu_primitive_map.py.

A tile is a dict of numpy arrays with the reference's field names (Lambdas (M,3,3), thetas (M,3),
etas (M,B,3), weights, timestamps, created_timestamps, last_supported_scan_seq,
last_update_scan_seq, primitive_ids, valid_mask, colors, cam_mass, lidar_mass, rgb_cam_accum,
rgb_cam_denom, rgb); the operators update it in place and return the reference's scalars.

Sort semantics: jax.lax.sort with the default num_keys=1 sorts on the first operand only and is
stable, and its float comparator treats -0.0 and 0.0 as equal; jnp.argsort is stable.  Here:
np.argsort(kind="stable") on the same keys (numpy also orders -0.0 == 0.0).  Scatter-adds
(.at[].add) accumulate in input order (XLA's CPU scatter); 3x3 solves / inverses / determinants
are LAPACK LU (np.linalg), as in JAX's CPU path.

Pinning: the reference's own tests for these operators (test_primitive_map_merge_reduce.py,
test_map_color_provenance.py) are restated in tests/test_primitive_map.py together with closed
forms; JAX is absent, so bit-level parity with the reference is parity unpinned.
"""

from __future__ import annotations

import numpy as np

GC_EPS_LIFT = 1e-9        # constants.py:71
GC_EPS_MASS = 1e-12
GC_EPS_PSD = 1e-12
GC_VMF_N_LOBES = 3        # constants.py:463
GC_RECENCY_DECAY_LAMBDA = 0.02   # constants.py:419
GC_RECENCY_MIN_SCALE = 0.05      # constants.py:420
GC_PRIMITIVE_FORGETTING_FACTOR = 0.995       # constants.py:442
GC_PRIMITIVE_MERGE_THRESHOLD = 0.1           # constants.py:445
GC_K_MERGE_PAIRS_PER_TILE = 4                # constants.py:448
GC_PRIMITIVE_MERGE_MAX_TILE_SIZE = 2048      # constants.py:450
GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD = 1e-4    # constants.py:453
GRAY = np.array([0.5, 0.5, 0.5])

FIELDS_F64 = ("Lambdas", "thetas", "etas", "weights", "timestamps", "created_timestamps", "colors", "cam_mass",
              "lidar_mass", "rgb_cam_accum", "rgb_cam_denom", "rgb")
FIELDS_I64 = ("last_supported_scan_seq", "last_update_scan_seq", "primitive_ids")


def create_empty_tile(m_tile, n_lobes=GC_VMF_N_LOBES):
    """primitive_map.py:148-174."""
    return dict(Lambdas=np.zeros((m_tile, 3, 3)), thetas=np.zeros((m_tile, 3)), etas=np.zeros((m_tile, n_lobes, 3)),
                weights=np.zeros(m_tile), timestamps=np.zeros(m_tile), created_timestamps=np.zeros(m_tile),
                last_supported_scan_seq=np.zeros(m_tile, np.int64), last_update_scan_seq=np.zeros(m_tile, np.int64),
                primitive_ids=np.zeros(m_tile, np.int64), valid_mask=np.zeros(m_tile, bool),
                colors=np.zeros((m_tile, 3)), cam_mass=np.zeros(m_tile), lidar_mass=np.zeros(m_tile),
                rgb_cam_accum=np.zeros((m_tile, 3)), rgb_cam_denom=np.zeros(m_tile),
                rgb=np.broadcast_to(GRAY, (m_tile, 3)).copy())


def copy_tile(t):
    return {k: np.array(v, copy=True) for k, v in t.items()}


def select_topk_slots(weights, valid, k):
    """:303-322: top k by weight (invalid -> -1e30), stable on -score."""
    score = np.where(valid, weights, -1e30)
    return np.argsort(-score, kind="stable")[:k].astype(np.int32)


def select_lowest_mass_slots(weights, valid, last_supported, scan_seq, lam, k):
    """:325-353: lowest retention w exp(-lam max(0, seq - last)) (empty slots -inf first), stable."""
    dt = np.maximum(0, int(scan_seq) - np.asarray(last_supported, np.int64))
    decay = np.exp(-float(lam) * dt.astype(np.float64))
    key = np.where(valid, weights * decay, -np.inf)
    return np.argsort(key, kind="stable")[:k].astype(np.int32)


def _solve(L, b):
    return np.linalg.solve(L, b[..., None])[..., 0]


def extract_atlas_map_view(tiles, tile_ids, m_tile_view, m_tile, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """:356-450 + _extract_primitive_map_view_core (:474-498); a tile missing from `tiles` is empty."""
    k = int(m_tile_view)
    if k <= 0:
        raise ValueError(f"extract_atlas_map_view: m_tile_view must be > 0, got {m_tile_view}")
    parts = {f: [] for f in ("Lambdas", "thetas", "etas", "weights", "primitive_ids", "valid_mask",
                             "last_supported_scan_seq", "rgb", "candidate_slots", "candidate_tile_ids")}
    for tid in tile_ids:
        t = tiles.get(int(tid)) or create_empty_tile(m_tile)
        slots = select_topk_slots(t["weights"], t["valid_mask"], k)
        for f in ("Lambdas", "thetas", "etas", "weights", "primitive_ids", "valid_mask", "last_supported_scan_seq",
                  "rgb"):
            parts[f].append(np.asarray(t[f])[slots])
        parts["candidate_slots"].append(slots)
        parts["candidate_tile_ids"].append(np.full(slots.shape, int(tid), np.int64))
    v = {f: np.concatenate(x, axis=0) for f, x in parts.items()}
    L = v["Lambdas"] + eps_lift * np.eye(3)[None]
    es = np.sum(v["etas"], axis=1)
    kap = np.linalg.norm(es, axis=1)
    v.update(positions=_solve(L, v["thetas"]), covariances=np.linalg.inv(L), directions=es / (kap[:, None] + eps_mass),
             kappas=kap, colors=v.pop("rgb"), tile_ids=np.asarray(tile_ids, np.int64), m_tile_view=k)
    return v


def insert_masked(tile, next_global_id, Lambdas_new, thetas_new, etas_new, weights_new, timestamp, valid_new_mask,
                  scan_seq=0, recency_decay_lambda=GC_RECENCY_DECAY_LAMBDA, colors_new=None, sources_new=None):
    """:807-981.  Returns (n_inserted, new_ids_full, dropped, next_global_id)."""
    weights_new = np.asarray(weights_new, np.float64).reshape(-1)
    do = np.asarray(valid_new_mask, bool).reshape(-1)
    K = weights_new.shape[0]
    tgt = select_lowest_mass_slots(tile["weights"], tile["valid_mask"], tile["last_supported_scan_seq"], scan_seq,
                                   recency_decay_lambda, K)
    n_ins = int(do.sum())
    prefix = np.cumsum(do.astype(np.int64)) - 1
    ids = np.where(do, int(next_global_id) + prefix, -1).astype(np.int64)
    colors_new = np.zeros((K, 3)) if colors_new is None else np.asarray(colors_new, np.float64)
    if sources_new is not None:
        s = np.asarray(sources_new, np.int32).reshape(-1)
        is_cam, is_lidar = (s == 0).astype(np.float64), (s == 1).astype(np.float64)
    else:
        is_cam, is_lidar = np.zeros(K), np.ones(K)
    cam = weights_new * is_cam
    lid = weights_new * is_lidar
    acc = colors_new * cam[:, None]
    rgb_new = np.where((cam > 0.0)[:, None], np.clip(colors_new, 0.0, 1.0), GRAY)
    sel = lambda new, f: np.where(do.reshape((-1,) + (1,) * (new.ndim - 1)), new, tile[f][tgt])  # noqa: E731
    upd = dict(Lambdas=sel(np.asarray(Lambdas_new, np.float64), "Lambdas"),
               thetas=sel(np.asarray(thetas_new, np.float64), "thetas"),
               etas=sel(np.asarray(etas_new, np.float64), "etas"), weights=sel(weights_new, "weights"),
               primitive_ids=sel(ids, "primitive_ids"), colors=sel(rgb_new, "colors"), cam_mass=sel(cam, "cam_mass"),
               lidar_mass=sel(lid, "lidar_mass"), rgb_cam_accum=sel(acc, "rgb_cam_accum"),
               rgb_cam_denom=sel(cam, "rgb_cam_denom"), rgb=sel(rgb_new, "rgb"),
               timestamps=sel(np.full(K, float(timestamp)), "timestamps"),
               created_timestamps=sel(np.full(K, float(timestamp)), "created_timestamps"),
               last_supported_scan_seq=sel(np.full(K, int(scan_seq), np.int64), "last_supported_scan_seq"),
               last_update_scan_seq=sel(np.full(K, int(scan_seq), np.int64), "last_update_scan_seq"))
    upd["valid_mask"] = tile["valid_mask"][tgt] | do
    for f, v in upd.items():
        tile[f][tgt] = v
    return n_ins, ids, int((~do).sum()), int(next_global_id) + n_ins


def fuse(tile, target_slots, Lambdas_meas, thetas_meas, etas_meas, weights_meas, responsibilities, timestamp,
         scan_seq=0, valid_mask=None, colors_meas=None, sources_meas=None, eps_mass=GC_EPS_MASS):
    """:992-1163 (the chunked scatter-adds accumulate in input order).  Returns n_fused."""
    tgt = np.asarray(target_slots).reshape(-1).astype(np.int64)
    K = tgt.shape[0]
    if K == 0:
        return 0
    M = tile["weights"].shape[0]
    resp = np.asarray(responsibilities, np.float64).reshape(-1)
    if valid_mask is not None:
        resp = resp * np.asarray(valid_mask).reshape(-1).astype(np.float64)
    w = np.asarray(weights_meas, np.float64).reshape(-1)
    Lm = np.asarray(Lambdas_meas, np.float64)
    th = np.asarray(thetas_meas, np.float64)
    et = np.asarray(etas_meas, np.float64)
    dL, dth, det_ = np.zeros((M, 3, 3)), np.zeros((M, 3)), np.zeros((M,) + et.shape[1:])
    dw, drs, dcam, dlid, dacc, dden = (np.zeros(M), np.zeros(M), np.zeros(M), np.zeros(M), np.zeros((M, 3)),
                                       np.zeros(M))
    cols = None if colors_meas is None else np.clip(np.asarray(colors_meas, np.float64), 0.0, 1.0)
    src = None if sources_meas is None else np.asarray(sources_meas, np.int32).reshape(-1)
    for n in range(K):   # .at[idx].add in input order
        s, r = tgt[n], resp[n]
        dL[s] += r * Lm[n]
        dth[s] += r * th[n]
        det_[s] += r * et[n]
        dw[s] += r * w[n]
        drs[s] += r
        if src is not None:
            wc = r * w[n] * float(src[n] == 0)
            dcam[s] += wc
            dlid[s] += r * w[n] * float(src[n] == 1)
            if cols is not None:
                dacc[s] += cols[n] * wc
                dden[s] += wc
    tile["cam_mass"] = tile["cam_mass"] + dcam
    tile["lidar_mass"] = tile["lidar_mass"] + dlid
    tile["rgb_cam_accum"] = tile["rgb_cam_accum"] + dacc
    tile["rgb_cam_denom"] = tile["rgb_cam_denom"] + dden
    est = np.clip(tile["rgb_cam_accum"] / np.maximum(tile["rgb_cam_denom"][:, None], eps_mass), 0.0, 1.0)
    tile["rgb"] = np.where((tile["cam_mass"] > 0.0)[:, None], est, GRAY)
    tile["colors"] = tile["rgb"].copy()
    tile["Lambdas"] = tile["Lambdas"] + dL
    tile["thetas"] = tile["thetas"] + dth
    tile["etas"] = tile["etas"] + det_
    tile["weights"] = tile["weights"] + dw
    tile["timestamps"][np.unique(tgt)] = float(timestamp)
    upd = drs > 0.0
    tile["last_supported_scan_seq"] = np.where(upd, int(scan_seq), tile["last_supported_scan_seq"]).astype(np.int64)
    tile["last_update_scan_seq"] = np.where(upd, int(scan_seq), tile["last_update_scan_seq"]).astype(np.int64)
    return int(np.unique(tgt).shape[0])


def cull(tile, weight_threshold=GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD, eps_mass=GC_EPS_MASS):
    """:1175-1304 (weight threshold).  Returns (n_culled, mass_dropped, mass_epsilon_ratio)."""
    if int(tile["valid_mask"].sum()) == 0:
        return 0, 0.0, 0.0
    below = tile["valid_mask"] & (tile["weights"] < weight_threshold)
    n = int(below.sum())
    if n == 0:
        return 0, 0.0, 0.0
    dropped = float(np.sum(tile["weights"] * below.astype(np.float64)))
    ratio = dropped / (float(np.sum(tile["weights"])) + eps_mass)
    tile["valid_mask"] = tile["valid_mask"] & ~below
    return n, dropped, ratio


def forget(tile, forgetting_factor=GC_PRIMITIVE_FORGETTING_FACTOR):
    """:1314-1384."""
    tile["weights"] = float(forgetting_factor) * tile["weights"]


def recency_inflate(tiles, tile_ids, scan_seq, recency_decay_lambda=GC_RECENCY_DECAY_LAMBDA,
                    min_scale=GC_RECENCY_MIN_SCALE):
    """:1400-1484.  Returns (strength, cov_inflation_trace, downscale_total, n_valid_total)."""
    down = infl = nv = 0.0
    for tid in tile_ids:
        t = tiles.get(int(tid))
        if t is None:
            continue
        valid = t["valid_mask"].astype(np.float64)
        dt = np.maximum(0, int(scan_seq) - t["last_supported_scan_seq"])
        decay = np.clip(np.exp(-float(recency_decay_lambda) * dt.astype(np.float64)), float(min_scale), 1.0)
        decay = np.where(t["valid_mask"], decay, 1.0)
        t["Lambdas"] = t["Lambdas"] * decay[:, None, None]
        t["thetas"] = t["thetas"] * decay[:, None]
        nv += float(np.sum(valid))
        down += float(np.sum((1.0 - decay) * valid))
        infl += float(np.sum(((1.0 / decay) - 1.0) * valid))
    return down / max(nv, 1.0), infl, down, nv


def merge_pair_distances(tile, eps_lift=GC_EPS_LIFT):
    """:1907-1930: Bhattacharyya distance over triu pairs (row-major), inf where a slot is invalid."""
    M = tile["weights"].shape[0]
    L = tile["Lambdas"] + eps_lift * np.eye(3)[None]
    mu = _solve(L, tile["thetas"])
    Sig = np.linalg.inv(L)
    dS = np.linalg.det(Sig)
    i, j = np.triu_indices(M, k=1)
    S = 0.5 * (Sig[i] + Sig[j])
    Si = np.linalg.inv(S + eps_lift * np.eye(3)[None])
    dmu = mu[i] - mu[j]
    quad = 0.125 * np.einsum("ni,nij,nj->n", dmu, Si, dmu)
    with np.errstate(divide="ignore", invalid="ignore"):
        logt = 0.5 * np.log(np.linalg.det(S) / np.sqrt(dS[i] * dS[j] + 1e-24))
    dist = quad + logt
    v = tile["valid_mask"]
    return np.where(v[i] & v[j], dist, np.inf), i, j, mu, Sig


def merge_reduce(tile, merge_threshold=GC_PRIMITIVE_MERGE_THRESHOLD, max_pairs=GC_K_MERGE_PAIRS_PER_TILE,
                 max_tile_size=GC_PRIMITIVE_MERGE_MAX_TILE_SIZE, eps_psd=GC_EPS_PSD, eps_lift=GC_EPS_LIFT):
    """:1809-2031 with _merge_reduce_jax (:1501-1807).  Returns (n_merged, status, pairs):
    status 'noop' (fewer than 2 valid / max_pairs <= 0 / nothing merged), 'cap' (M > max_tile_size:
    the budget-cap certificate, mass_epsilon_ratio (M - cap) / M), 'merged'."""
    M = tile["weights"].shape[0]
    if M < 2 or int(tile["valid_mask"].sum()) < 2 or int(max_pairs) <= 0:
        return 0, "noop", []
    if int(max_tile_size) > 0 and M > int(max_tile_size):
        return 0, "cap", []
    dist, ii, jj, mu, Sig = merge_pair_distances(tile, eps_lift)
    used = np.zeros(M, bool)
    pairs = []
    for idx in np.argsort(dist, kind="stable"):
        i, j, d = int(ii[idx]), int(jj[idx]), dist[idx]
        if len(pairs) < int(max_pairs) and np.isfinite(d) and d < merge_threshold and not used[i] and not used[j]:
            used[i] = used[j] = True
            pairs.append((i, j))
    for i, j in pairs:
        w1, w2 = tile["weights"][i], tile["weights"][j]
        ws = w1 + w2
        if not ws > 0.0:
            continue
        mu_m = (w1 * mu[i] + w2 * mu[j]) / ws
        d1, d2 = (mu[i] - mu_m)[:, None], (mu[j] - mu_m)[:, None]
        Sm = (w1 * (Sig[i] + d1 @ d1.T) + w2 * (Sig[j] + d2 @ d2.T)) / ws + eps_psd * np.eye(3)
        Lm = np.linalg.inv(Sm)
        tile["Lambdas"][i] = Lm
        tile["thetas"][i] = Lm @ mu_m
        tile["etas"][i] = (w1 * tile["etas"][i] + w2 * tile["etas"][j]) / ws
        cam = tile["cam_mass"][i] + tile["cam_mass"][j]
        tile["lidar_mass"][i] = tile["lidar_mass"][i] + tile["lidar_mass"][j]
        acc = tile["rgb_cam_accum"][i] + tile["rgb_cam_accum"][j]
        den = tile["rgb_cam_denom"][i] + tile["rgb_cam_denom"][j]
        rgb = np.where(cam > 0.0, np.clip(acc / np.maximum(den, eps_psd), 0.0, 1.0), GRAY)
        tile["cam_mass"][i], tile["rgb_cam_accum"][i], tile["rgb_cam_denom"][i] = cam, acc, den
        tile["weights"][i] = ws
        tile["colors"][i] = rgb
        tile["rgb"][i] = rgb
        tile["timestamps"][i] = max(tile["timestamps"][i], tile["timestamps"][j])
        tile["created_timestamps"][i] = min(tile["created_timestamps"][i], tile["created_timestamps"][j])
        for f in ("last_supported_scan_seq", "last_update_scan_seq"):
            tile[f][i] = max(tile[f][i], tile[f][j])
        tile["weights"][j] = 0.0
        tile["valid_mask"][j] = False
    n = len(pairs)
    return n, ("merged" if n > 0 else "noop"), pairs


GC_K_INSERT_TILE = 64        # constants.py:476-477
GC_ASSOC_BLOCK_SIZE = 256    # constants.py:473
BITS_PER_AXIS, BIAS = 21, 1 << 20   # tiling.py:80-81
MASK = (1 << BITS_PER_AXIS) - 1


def tile_ids_from_xyz(X, h_tile):
    """tiling.py:126-145 (packed MA-hex tile ids of world points)."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    h = max(float(h_tile), 1e-12)
    s2 = X[:, 0] * 0.5 + X[:, 1] * (np.sqrt(3.0) * 0.5)
    c1, c2, cz = (np.floor(X[:, 0] / h).astype(np.int64), np.floor(s2 / h).astype(np.int64),
                  np.floor(X[:, 2] / h).astype(np.int64))
    return (((c1 + BIAS) & MASK) << (2 * BITS_PER_AXIS)) | (((c2 + BIAS) & MASK) << BITS_PER_AXIS) | ((cz + BIAS) & MASK)


def to_world(R, t, Lambdas, thetas, etas, eps_lift=GC_EPS_LIFT):
    """pipeline.py:1248-1256 transform_gaussian_to_world, vmapped: (R Lambda) R^T, R mu + t, Lambda_w mu_w,
    each lobe R eta."""
    Lw = (R[None] @ np.asarray(Lambdas, np.float64)) @ R.T[None]
    mu_b = _solve(np.asarray(Lambdas, np.float64) + eps_lift * np.eye(3)[None], np.asarray(thetas, np.float64))
    mu_w = (R[None] @ mu_b[..., None])[..., 0] + t[None]
    return Lw, (Lw @ mu_w[..., None])[..., 0], (R[None, None] @ np.asarray(etas, np.float64)[..., None])[..., 0]


def map_update_step(tiles, next_global_id, batch, assoc, R, t, active_tile_ids, m_tile, timestamp, scan_seq,
                    k_insert_tile=GC_K_INSERT_TILE, h_tile=2.0, block_size=GC_ASSOC_BLOCK_SIZE,
                    recency_decay_lambda=GC_RECENCY_DECAY_LAMBDA, cull_threshold=GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD,
                    forgetting_factor=GC_PRIMITIVE_FORGETTING_FACTOR, merge_threshold=GC_PRIMITIVE_MERGE_THRESHOLD,
                    k_merge_pairs=GC_K_MERGE_PAIRS_PER_TILE, merge_max_tile_size=GC_PRIMITIVE_MERGE_MAX_TILE_SIZE,
                    eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS, eps_psd=GC_EPS_PSD):
    """pipeline.py:1244-1447 (step 12b): fuse per association block and active tile, novelty
    insertion per active tile, then cull / forget / merge-reduce per active tile.  batch: dict
    Lambdas, thetas, etas, weights, valid_mask, colors, sources; assoc: dict responsibilities,
    candidate_tile_ids, candidate_slots, row_masses.  tiles: dict id -> tile (missing active tiles are
    created).  Returns (next_global_id, MapUpdateCert counters dict)."""
    for tid in active_tile_ids:
        tiles.setdefault(int(tid), create_empty_tile(m_tile, np.asarray(batch["etas"]).shape[1]))
    valid = np.asarray(batch["valid_mask"], bool)
    N, K = np.asarray(assoc["responsibilities"]).shape
    st = dict(fused_count=0, fused_mass_total=0.0, insert_count_total=0, insert_mass_total=0.0, insert_mass_p95=0.0,
              evicted_count=0, evicted_mass_total=0.0, merged_count=0)
    nb = (N + block_size - 1) // block_size
    for b in range(nb):   # block_associations_for_fuse (primitive_association.py:561-588)
        idx = np.arange(b * block_size, (b + 1) * block_size)
        mi = np.minimum(idx, N - 1)
        vr = (idx < N) & valid[mi]
        tile_flat = np.asarray(assoc["candidate_tile_ids"])[mi].reshape(-1).astype(np.int64)
        slot_flat = np.asarray(assoc["candidate_slots"])[mi].reshape(-1).astype(np.int32)
        resp = (np.asarray(assoc["responsibilities"])[mi] * vr[:, None]).reshape(-1)
        vflat = np.repeat(vr, K)
        rep = lambda x: np.repeat(np.asarray(x)[mi], K, axis=0)  # noqa: E731
        Lw, thw, ew = to_world(R, t, rep(batch["Lambdas"]), rep(batch["thetas"]), rep(batch["etas"]), eps_lift)
        wm = rep(batch["weights"])
        for tid in active_tile_ids:
            vt = vflat & (tile_flat == int(tid))
            st["fused_mass_total"] += float(np.sum(wm * resp * vt.astype(np.float64)))
            st["fused_count"] += fuse(tiles[int(tid)], slot_flat, Lw, thw, ew, wm, resp, timestamp, scan_seq,
                                      valid_mask=vt, colors_meas=rep(batch["colors"]),
                                      sources_meas=rep(batch["sources"]), eps_mass=eps_mass)
    a = valid.astype(np.float64)
    a = a / max(np.sum(a), eps_mass)
    novelty = np.maximum(a - np.asarray(assoc["row_masses"], np.float64), 0.0)
    w = np.asarray(batch["weights"], np.float64)
    score = novelty * w - (1.0 - valid.astype(np.float64)) * 1e6
    mu_b = _solve(np.asarray(batch["Lambdas"]) + eps_lift * np.eye(3)[None], np.asarray(batch["thetas"]))
    mtid = tile_ids_from_xyz((R[None] @ mu_b[..., None])[..., 0] + t[None], h_tile)
    for tid in active_tile_ids:
        it = mtid == int(tid)
        sc = np.where(it, score, -1e30)
        ins = np.argsort(-sc, kind="stable")[:k_insert_tile]
        vn = it[ins] & (sc[ins] > -1e20)
        if not vn.any():
            vn = np.ones_like(vn)
        wi = np.where(it[ins], novelty[ins] * w[ins], 0.0)
        st["insert_mass_total"] += float(np.sum(wi))
        ws = np.sort(wi)
        if ws.shape[0] > 0:
            st["insert_mass_p95"] = max(st["insert_mass_p95"], float(ws[min(int(0.95 * ws.shape[0]), ws.shape[0] - 1)]))
        Lw, thw, ew = to_world(R, t, np.asarray(batch["Lambdas"])[ins], np.asarray(batch["thetas"])[ins],
                               np.asarray(batch["etas"])[ins], eps_lift)
        n, _, _, next_global_id = insert_masked(tiles[int(tid)], next_global_id, Lw, thw, ew, wi, timestamp, vn,
                                                scan_seq, recency_decay_lambda, np.asarray(batch["colors"])[ins],
                                                np.asarray(batch["sources"])[ins])
        st["insert_count_total"] += n
    for tid in active_tile_ids:
        n, dropped, _ = cull(tiles[int(tid)], cull_threshold, eps_mass)
        st["evicted_count"] += n
        st["evicted_mass_total"] += dropped
        forget(tiles[int(tid)], forgetting_factor)
        st["merged_count"] += merge_reduce(tiles[int(tid)], merge_threshold, k_merge_pairs, merge_max_tile_size,
                                           eps_psd, eps_lift)[0]
    return next_global_id, st


def ma_hex_stencil_tile_ids(center_xyz, h_tile, radius_xy, radius_z):
    """tiling.py:167-209: packed tile ids of the hex disk (sorted axial (q, r)) x z slab around the
    centre's MA-hex cell, z outer."""
    x, y, z = (float(v) for v in np.asarray(center_xyz, np.float64).ravel()[:3])
    h = max(float(h_tile), 1e-12)
    c1, c2, cz = int(np.floor(x / h)), int(np.floor((x * 0.5 + y * (np.sqrt(3.0) * 0.5)) / h)), int(np.floor(z / h))
    r = int(radius_xy)
    disk = sorted((q, rr) for q in range(-r, r + 1) for rr in range(max(-r, -q - r), min(r, -q + r) + 1))
    pack = lambda a, b, c: (((a + BIAS) & MASK) << (2 * BITS_PER_AXIS)) | (((b + BIAS) & MASK) << BITS_PER_AXIS) | (  # noqa: E731
        (c + BIAS) & MASK)
    return [int(pack(c1 + dq, c2 + dr, cz + dz)) for dz in range(-int(radius_z), int(radius_z) + 1) for dq, dr in disk]
