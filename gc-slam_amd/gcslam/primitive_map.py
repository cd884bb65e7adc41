"""The live primitive path's map on the MI355X: the AtlasMap's tiles resident
in HBM and the maintenance operators with the reference's calling conventions
(FS/backend/structures/primitive_map.py), running gcs_pmap_* (libgcslam_hip.so):

  extract_atlas_map_view         :356-450   -> gcslam.association.AtlasMapView (device tensors)
  primitive_map_insert_masked    :807-981   (+ primitive_map_insert_masked_tiles: several tiles, one call)
  primitive_map_fuse             :992-1163  (+ primitive_map_fuse_tiles: the pipeline's active-tile loop,
                                             pipeline.py:1301-1327, in one call)
  primitive_map_cull             :1175-1304
  primitive_map_forget           :1314-1384
  primitive_map_recency_inflate  :1400-1484
  primitive_map_merge_reduce     :1809-2031
  primitive_map_update           pipeline.py:1232-1492 (step 12b: fuse per association block, novelty
                                 insertion, cull / forget / merge per active tile) in one library call

Each operator returns the reference's (result, CertBundle, ExpectedEffect).  The reference's
AtlasMap is immutable (every operator returns a new one); this one is updated in place on the GPU
and result.atlas_map is the same object.  Inputs may be numpy arrays or device tensors.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib as L
from .association import AtlasMapView
from .certificates import CertBundle, ExpectedEffect, InfluenceCert

CHART_ID = "GC-RIGHT-01"
GC_EPS_LIFT = 1e-9
GC_EPS_MASS = 1e-12
GC_EPS_PSD = 1e-12
GC_VMF_N_LOBES = 3                          # constants.py:463
GC_PRIMITIVE_MAP_MAX_SIZE = 50000           # constants.py:392 (= GC_M_TILE)
GC_RECENCY_DECAY_LAMBDA = 0.02              # constants.py:419
GC_RECENCY_MIN_SCALE = 0.05                 # constants.py:420
GC_PRIMITIVE_FORGETTING_FACTOR = 0.995      # constants.py:442
GC_PRIMITIVE_MERGE_THRESHOLD = 0.1          # constants.py:445
GC_K_MERGE_PAIRS_PER_TILE = 4               # constants.py:448
GC_PRIMITIVE_MERGE_MAX_TILE_SIZE = 2048     # constants.py:450
GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD = 1e-4   # constants.py:453
GC_FUSE_CHUNK_SIZE = 1024                   # constants.py:470

_DT = {"f": np.float64, "i": np.int64, "u": np.uint8}
_KIND = ["f"] * 12 + ["i"] * 3 + ["u"]


def _torch():
    import torch
    return torch


class AtlasMap:
    """primitive_map.py:182-211: tile_id -> tile; here the tiles live in one gcs_pmap context on
    `device` (max_tiles storage slots of m_tile primitives) and `tiles` maps tile ids to storage
    indices.  next_global_id / total_count follow the reference's bookkeeping."""

    def __init__(self, m_tile: int = GC_PRIMITIVE_MAP_MAX_SIZE, max_tiles: int = 64, n_lobes: int = GC_VMF_N_LOBES,
                 max_merge: int = GC_PRIMITIVE_MERGE_MAX_TILE_SIZE, device: int = 0):
        self.lib = L.load()
        h = C.c_void_p()
        rc = self.lib.gcs_pmap_create(int(m_tile), int(max_tiles), int(n_lobes), int(max_merge), int(device),
                                      C.byref(h))
        if rc != 0:
            raise (ValueError if rc == -1 else RuntimeError)(f"gcs_pmap_create failed ({rc})")
        self.h = h
        self.m_tile, self.max_tiles, self.n_lobes, self.device = int(m_tile), int(max_tiles), int(n_lobes), int(device)
        self.max_merge = int(max_merge)
        self.tiles = {}
        self.counts = {}
        self.next_global_id = 0
        self.total_count = 0
        self._free = list(range(self.max_tiles))
        # storage slots that may hold data; every other slot is as gcs_pmap_create cleared it, so a tile
        # created there needs no clear (a kernel and a stream sync per new tile on the live path)
        self._written = set()
        self._dir_ver, self._dir = 0, None  # directory arrays for gcs_live_scan, rebuilt on change

    # ------------------------------------------------------------------ plumbing
    def close(self):
        if getattr(self, "h", None):
            self.lib.gcs_pmap_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.gcs_pmap_last_error(self.h).decode(errors="replace")
            raise (ValueError if rc in (-1, -3) else RuntimeError)(f"{what} failed ({rc}): {msg}")

    def _stream(self):
        torch = _torch()
        dev = f"cuda:{self.device}"
        self._chk(self.lib.gcs_pmap_set_stream(self.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                  "gcs_pmap_set_stream")

    @property
    def n_tiles(self) -> int:
        return len(self.tiles)

    @property
    def tile_ids(self) -> List[int]:
        return list(self.tiles.keys())

    def index(self, tile_id: int, create: bool = True) -> int:
        """Storage index of tile_id (create_empty_tile on first use, :148-174); -1 if absent."""
        tid = int(tile_id)
        if tid in self.tiles:
            return self.tiles[tid]
        if not create:
            return -1
        if not self._free:
            raise RuntimeError(f"primitive map holds max_tiles={self.max_tiles} tiles")
        idx = self._free.pop(0)
        if idx in self._written:
            self._chk(self.lib.gcs_pmap_clear_tile(self.h, idx), "gcs_pmap_clear_tile")
        self._written.add(idx)
        self.tiles[tid] = idx
        self.counts[tid] = 0
        self._dir_ver += 1
        return idx

    def directory(self):
        """The tile directory as gcs_live_args takes it: (ids int64, slots int32, free slots int32 in the
        order index() takes them, written uint8 per slot); cached until the directory changes."""
        if self._dir is None or self._dir[0] != self._dir_ver:
            n = len(self.tiles)
            ids = np.fromiter(self.tiles.keys(), np.int64, n)
            slots = np.fromiter(self.tiles.values(), np.int32, n)
            free = np.array(self._free, np.int32)
            written = np.zeros(max(self.max_tiles, 1), np.uint8)
            if self._written:
                written[np.fromiter(self._written, np.int64, len(self._written))] = 1
            self._dir = (self._dir_ver, ids, slots, free, written)
        return self._dir[1:]

    def adopt_created(self, ids, slots):
        """Record tiles gcs_live_scan created (index(create=True) of each, in order: the slots are the
        first free ones, cleared on the device where written)."""
        for tid, idx in zip(ids, slots):
            tid, idx = int(tid), int(idx)
            if self._free[0] != idx:
                raise RuntimeError(f"live scan created tile {tid} in slot {idx}, expected {self._free[0]}")
            self._free.pop(0)
            self._written.add(idx)
            self.tiles[tid] = idx
            self.counts[tid] = 0
        if len(ids):
            self._dir_ver += 1

    def _width(self, f):
        return {"Lambdas": (3, 3), "thetas": (3,), "etas": (self.n_lobes, 3), "colors": (3,), "rgb_cam_accum": (3,),
                "rgb": (3,)}.get(f, ())

    def read_tile(self, tile_id: int) -> dict:
        """The tile's arrays (reference field names and shapes) as numpy."""
        idx = self.index(tile_id, create=False)
        if idx < 0:
            raise KeyError(tile_id)
        out = {}
        for k, f in enumerate(L.PM_FIELDS):
            a = np.empty((self.m_tile,) + self._width(f), dtype=_DT[_KIND[k]])
            self._chk(self.lib.gcs_pmap_read(self.h, idx, k, a.ctypes.data), "gcs_pmap_read")
            out[f] = a.astype(bool) if f == "valid_mask" else a
        return out

    def write_tile(self, tile_id: int, arrays: dict):
        """Upload a tile (reference field names; missing fields keep their values)."""
        idx = self.index(tile_id, create=True)
        for k, f in enumerate(L.PM_FIELDS):
            if f in arrays:
                a = np.ascontiguousarray(np.asarray(arrays[f]).astype(_DT[_KIND[k]]).reshape(
                    (self.m_tile,) + self._width(f)))
                self._chk(self.lib.gcs_pmap_write(self.h, idx, k, a.ctypes.data), "gcs_pmap_write")
        if "valid_mask" in arrays:
            n = int(np.asarray(arrays["valid_mask"]).sum())
            self.total_count += n - self.counts.get(int(tile_id), 0)
            self.counts[int(tile_id)] = n


    def working_copy(self, tile_ids, into: "AtlasMap" = None) -> "AtlasMap":
        """A map holding device copies of the tiles of `tile_ids` this map has, with this map's
        bookkeeping (ids, counts): what a hypothesis that reads the node's map but must not update it
        works on -- the reference's maps are immutable and the node stores hypothesis 0's result only
        (backend_node.py:2062,2079-2083).  `into`: a scratch map to reuse (its tiles are dropped)."""
        ids = [int(t) for t in dict.fromkeys(int(x) for x in tile_ids)]
        if into is None or into.m_tile != self.m_tile or into.n_lobes != self.n_lobes or into.max_tiles < len(ids):
            into = AtlasMap(self.m_tile, max_tiles=max(len(ids), 1), n_lobes=self.n_lobes, max_merge=self.max_merge,
                            device=self.device)
        into.tiles, into.counts, into._free = {}, {}, list(range(into.max_tiles))
        into._dir_ver += 1
        present = [t for t in ids if t in self.tiles]
        dst = np.array([into._free.pop(0) for _ in present], dtype=np.int32)
        src = np.array([self.tiles[t] for t in present], dtype=np.int32)
        for t, d in zip(present, dst):
            into.tiles[t] = int(d)
            into.counts[t] = self.counts.get(t, 0)
        if present:
            into._chk(self.lib.gcs_pmap_copy_tiles(into.h, dst.ctypes.data, self.h, src.ctypes.data, len(present)),
                      "gcs_pmap_copy_tiles")
            into._written.update(int(d) for d in dst)
        into.next_global_id, into.total_count = self.next_global_id, self.total_count
        return into


def create_empty_atlas_map(m_tile: int = GC_PRIMITIVE_MAP_MAX_SIZE, max_tiles: int = 64, device: int = 0) -> AtlasMap:
    """primitive_map.py:214-227 (tiles are created on demand)."""
    return AtlasMap(m_tile=m_tile, max_tiles=max_tiles, device=device)


# ---------------------------------------------------------------------- results (reference dataclasses)
@dataclass
class PrimitiveMapInsertResult:      # :642-648
    atlas_map: AtlasMap
    tile_id: int
    n_inserted: int
    new_ids: object


@dataclass
class PrimitiveMapFuseResult:        # :984-989
    atlas_map: AtlasMap
    tile_id: int
    n_fused: int


@dataclass
class PrimitiveMapCullResult:        # :1166-1172
    atlas_map: AtlasMap
    tile_id: int
    n_culled: int
    mass_dropped: float


@dataclass
class PrimitiveMapForgetResult:      # :1307-1311
    atlas_map: AtlasMap
    tile_id: int


@dataclass
class PrimitiveMapRecencyInflateStats:   # :1392-1397
    staleness_inflation_strength: float
    staleness_cov_inflation_trace: float
    stale_precision_downscale_total: float


@dataclass
class PrimitiveMapMergeReduceResult:     # :1492-1498
    atlas_map: AtlasMap
    tile_id: int
    n_merged: int
    frobenius_correction: float


def _exact(chart_id, anchor_id, name, predicted=0.0, realized=0.0):
    return CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id), ExpectedEffect(name, predicted, realized)


class _Rows:
    """Device staging of proposal / contribution rows (kept alive for the call)."""

    def __init__(self, atlas: AtlasMap, n: int, Lambdas, thetas, etas, weights, valid=None, responsibilities=None,
                 colors=None, sources=None, tile_pos=None, slots=None):
        torch = _torch()
        dev = f"cuda:{atlas.device}"
        f64 = lambda x: torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x,  # noqa: E731
                                        device=dev).to(torch.float64).contiguous()
        i32 = lambda x: torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x,  # noqa: E731
                                        device=dev).to(torch.int32).contiguous()
        self.keep = []
        r = L.GcsPmapRows()
        r.n = int(n)

        def put(name, t):
            self.keep.append(t)
            setattr(r, name, t.data_ptr() if t.numel() else None)

        put("Lambdas", f64(Lambdas).reshape(n, 9))
        put("thetas", f64(thetas).reshape(n, 3))
        put("etas", f64(etas).reshape(n, -1) if n else f64(etas))
        put("weights", f64(weights).reshape(n))
        if valid is not None:
            put("valid", torch.as_tensor(np.asarray(valid) if not torch.is_tensor(valid) else valid,
                                         device=dev).to(torch.uint8).reshape(n).contiguous())
        if responsibilities is not None:
            put("responsibilities", f64(responsibilities).reshape(n))
        if colors is not None:
            put("colors", f64(colors).reshape(n, 3))
        if sources is not None:
            put("sources", i32(sources).reshape(n))
        if tile_pos is not None:
            put("tile_pos", i32(tile_pos).reshape(n))
        if slots is not None:
            put("slots", i32(slots).reshape(n))
        self.rows = r


def _tiles_arg(idx):
    a = np.ascontiguousarray(np.asarray(idx, dtype=np.int32))
    return a, L.iptr(a)


# ---------------------------------------------------------------------- operators
def view_buffers(n_lobes: int, n: int, k: int, dev: str):
    """Fresh AtlasMapView arrays of n tiles x k entries (one device allocation carved into the twelve
    outputs, 8-byte aligned segments; valid_mask written as 0/1 bytes straight into a bool view) and
    the gcs_pmap_view struct naming them."""
    torch = _torch()
    R = n * k
    spec = (("positions", torch.float64, (R, 3)), ("covariances", torch.float64, (R, 3, 3)),
            ("directions", torch.float64, (R, 3)), ("kappas", torch.float64, (R,)), ("weights", torch.float64, (R,)),
            ("primitive_ids", torch.int64, (R,)), ("last_supported_scan_seq", torch.int64, (R,)),
            ("etas", torch.float64, (R, n_lobes, 3)), ("colors", torch.float64, (R, 3)),
            ("candidate_tile_ids", torch.int64, (R,)), ("candidate_slots", torch.int32, (R,)),
            ("valid_mask", torch.bool, (R,)))
    sizes = [int(np.prod(shape)) * (8 if dt in (torch.float64, torch.int64) else 4 if dt == torch.int32 else 1)
             for _, dt, shape in spec]
    buf = torch.empty(sum((z + 7) // 8 * 8 for z in sizes), dtype=torch.uint8, device=dev)
    t, off = {}, 0
    for (name, dt, shape), z in zip(spec, sizes):
        t[name] = buf[off:off + z].view(dt).view(shape)
        off += (z + 7) // 8 * 8
    v = L.GcsPmapView()
    for name, x in t.items():
        setattr(v, name, x.data_ptr() if R else None)
    return t, v


def extract_atlas_map_view(atlas_map: AtlasMap, tile_ids: List[int], m_tile_view: int,
                           eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS) -> AtlasMapView:
    """:356-450: per listed tile the top m_tile_view slots by weight (stable on -score; a missing tile
    is viewed as empty), stitched in tile order, with means, covariances, resultant directions and
    kappas (:474-498)."""
    if int(m_tile_view) <= 0:
        raise ValueError(f"extract_atlas_map_view: m_tile_view must be > 0, got {m_tile_view}")
    torch = _torch()
    dev = f"cuda:{atlas_map.device}"
    n, k = len(tile_ids), int(m_tile_view)
    t, v = view_buffers(atlas_map.n_lobes, n, k, dev)
    idx, ip = _tiles_arg([atlas_map.index(tid, create=False) for tid in tile_ids])
    tids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int64))
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_extract_view(atlas_map.h, ip, tids.ctypes.data_as(L.c_int64_p), n, k,
                                                       float(eps_lift), float(eps_mass), C.byref(v)),
                   "gcs_pmap_extract_view")
    return AtlasMapView(tile_ids=torch.as_tensor(tids, device=dev), m_tile_view=k, **t)


def primitive_map_insert_masked_tiles(atlas_map: AtlasMap, tile_ids: List[int], Lambdas_new, thetas_new, etas_new,
                                      weights_new, timestamp: float, valid_new_mask, scan_seq: int = 0,
                                      recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA, colors_new=None,
                                      sources_new=None, chart_id: str = CHART_ID,
                                      anchor_id: str = "primitive_map_insert_masked"):
    """primitive_map_insert_masked on each listed tile in order with its K proposals (arrays
    (n_tiles, K, ...)); ids continue from next_global_id tile by tile, as the pipeline's loop
    (pipeline.py:1348-1392).  Returns one (result, cert, effect) per tile."""
    torch = _torch()
    n = len(tile_ids)
    wn = weights_new if torch.is_tensor(weights_new) else np.asarray(weights_new, np.float64)
    K = int(wn.shape[1]) if n else 0
    if K > atlas_map.m_tile:
        raise ValueError("K proposals exceed the tile size")
    idx, ip = _tiles_arg([atlas_map.index(tid, create=True) for tid in tile_ids])
    rows = _Rows(atlas_map, n * K, Lambdas_new, thetas_new, etas_new, weights_new, valid=valid_new_mask,
                 colors=colors_new, sources=sources_new)
    dev = f"cuda:{atlas_map.device}"
    new_ids = torch.empty((n, K), dtype=torch.int64, device=dev)
    n_ins = np.zeros(n, np.int32)
    cnt = np.zeros(n, np.int32)
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_insert_masked(
        atlas_map.h, ip, n, K, C.byref(rows.rows), float(timestamp), int(scan_seq), float(recency_decay_lambda),
        int(atlas_map.next_global_id), C.c_void_p(new_ids.data_ptr() if n * K else None), L.iptr(n_ins),
        L.iptr(cnt)), "gcs_pmap_insert_masked")
    vm = valid_new_mask.detach().cpu().numpy() if torch.is_tensor(valid_new_mask) else np.asarray(valid_new_mask)
    vm = vm.reshape(n, K).astype(bool) if n else vm
    out = []
    for t, tid in enumerate(tile_ids):
        ni = int(n_ins[t])
        atlas_map.next_global_id += ni
        atlas_map.total_count += ni
        atlas_map.counts[int(tid)] = int(cnt[t])
        dropped = int((~vm[t]).sum())
        cert = (CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["insert_unfilled_budget"],
                                         frobenius_applied=False) if dropped > 0
                else CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id))
        eff = ExpectedEffect("primitive_map_insert_masked", float(int(vm[t].sum())), float(ni))
        out.append((PrimitiveMapInsertResult(atlas_map, int(tid), ni, new_ids[t]), cert, eff))
    return out


def primitive_map_insert_masked(atlas_map: AtlasMap, tile_id: int, Lambdas_new, thetas_new, etas_new, weights_new,
                                timestamp: float, valid_new_mask, scan_seq: int = 0,
                                recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA, colors_new=None,
                                sources_new=None, chart_id: str = CHART_ID,
                                anchor_id: str = "primitive_map_insert_masked"):
    """:807-981: up to K masked proposals into the tile's K lowest-retention slots (empty first)."""
    add = lambda x: None if x is None else (x[None] if _torch().is_tensor(x) else np.asarray(x)[None])  # noqa: E731
    return primitive_map_insert_masked_tiles(atlas_map, [tile_id], add(Lambdas_new), add(thetas_new), add(etas_new),
                                             add(weights_new), timestamp, add(valid_new_mask), scan_seq,
                                             recency_decay_lambda, add(colors_new), add(sources_new), chart_id,
                                             anchor_id)[0]


def primitive_map_fuse_tiles(atlas_map: AtlasMap, active_tile_ids: List[int], tile_ids_flat, target_slots,
                             Lambdas_meas, thetas_meas, etas_meas, weights_meas, responsibilities, timestamp: float,
                             scan_seq: int = 0, valid_mask=None, colors_meas=None, sources_meas=None,
                             eps_mass: float = GC_EPS_MASS, chart_id: str = CHART_ID, anchor_id: str = "primitive_map"):
    """The pipeline's per-active-tile fuse loop (pipeline.py:1301-1327) in one call: tile t fuses the
    rows with tile_ids_flat == t (and valid); each (result, cert, effect) as primitive_map_fuse's."""
    torch = _torch()
    K = int((target_slots.shape if torch.is_tensor(target_slots) else np.asarray(target_slots).shape)[0])
    if K == 0 or not active_tile_ids:
        return [(PrimitiveMapFuseResult(atlas_map, int(t), 0),) + _exact(chart_id, anchor_id, "primitive_map_fuse")
                for t in active_tile_ids]
    idx, ip = _tiles_arg([atlas_map.index(tid, create=True) for tid in active_tile_ids])
    pos = {int(t): i for i, t in enumerate(active_tile_ids)}
    tf = tile_ids_flat.detach().cpu().numpy() if torch.is_tensor(tile_ids_flat) else np.asarray(tile_ids_flat)
    tpos = np.array([pos.get(int(t), -1) for t in tf.reshape(-1)], dtype=np.int32)
    rows = _Rows(atlas_map, K, Lambdas_meas, thetas_meas, etas_meas, weights_meas, valid=valid_mask,
                 responsibilities=responsibilities, colors=colors_meas, sources=sources_meas, tile_pos=tpos,
                 slots=target_slots)
    nf = np.zeros(1, np.int32)
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_fuse(atlas_map.h, ip, len(active_tile_ids), C.byref(rows.rows),
                                               float(timestamp), int(scan_seq), float(eps_mass), L.iptr(nf)),
                   "gcs_pmap_fuse")
    return [(PrimitiveMapFuseResult(atlas_map, int(t), int(nf[0])),
             CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
             ExpectedEffect("primitive_map_fuse", float(K), float(nf[0]))) for t in active_tile_ids]


def primitive_map_fuse(atlas_map: AtlasMap, tile_id: int, target_slots, Lambdas_meas, thetas_meas, etas_meas,
                       weights_meas, responsibilities, timestamp: float, scan_seq: int = 0, valid_mask=None,
                       colors_meas=None, sources_meas=None, eps_psd: float = GC_EPS_PSD, eps_mass: float = GC_EPS_MASS,
                       fuse_chunk_size: int = GC_FUSE_CHUNK_SIZE, chart_id: str = CHART_ID,
                       anchor_id: str = "primitive_map"):
    """:992-1163: PoE fuse of K rows into the tile's target slots (sums in row order; the chunking
    of the reference does not change that order)."""
    torch = _torch()
    K = int((target_slots.shape if torch.is_tensor(target_slots) else np.asarray(target_slots).shape)[0])
    return primitive_map_fuse_tiles(atlas_map, [tile_id], np.full(K, int(tile_id), np.int64), target_slots,
                                    Lambdas_meas, thetas_meas, etas_meas, weights_meas, responsibilities, timestamp,
                                    scan_seq, valid_mask, colors_meas, sources_meas, eps_mass, chart_id, anchor_id)[0]


def primitive_map_cull(atlas_map: AtlasMap, tile_id: int,
                       weight_threshold: float = GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD,
                       max_primitives: Optional[int] = None, chart_id: str = CHART_ID, anchor_id: str = "primitive_map"):
    """:1175-1304: valid primitives below the weight threshold are dropped (budgeting, mass logged)."""
    idx = atlas_map.index(tile_id, create=True)
    no_op = lambda: (PrimitiveMapCullResult(atlas_map, int(tile_id), 0, 0.0),) + _exact(  # noqa: E731
        chart_id, anchor_id, "primitive_map_cull")
    if atlas_map.counts.get(int(tile_id), 0) == 0:
        return no_op()
    thr = float(weight_threshold)
    if max_primitives is not None:   # :1220-1228: effective threshold from the sorted weights (host)
        t = atlas_map.read_tile(tile_id)
        below = t["valid_mask"] & (t["weights"] < thr)
        if atlas_map.counts[int(tile_id)] - int(below.sum()) > max_primitives:
            sw = np.sort(t["weights"] * t["valid_mask"].astype(np.float64))[::-1]
            if max_primitives < len(sw):
                thr = float(sw[max_primitives])
    ip = _tiles_arg([idx])
    nc, cnt = np.zeros(1, np.int32), np.zeros(1, np.int32)
    md, ws = np.zeros(1), np.zeros(1)
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_cull(atlas_map.h, ip[1], 1, thr, L.iptr(nc), L.dptr(md), L.dptr(ws),
                                               L.iptr(cnt)), "gcs_pmap_cull")
    n = int(nc[0])
    if n == 0:
        return no_op()
    atlas_map.counts[int(tile_id)] = int(cnt[0])
    atlas_map.total_count -= n
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["budgeting", "mass_drop"],
                                    influence=InfluenceCert.identity().with_overrides(
                                        mass_epsilon_ratio=float(md[0]) / (float(ws[0]) + GC_EPS_MASS)))
    return (PrimitiveMapCullResult(atlas_map, int(tile_id), n, float(md[0])), cert,
            ExpectedEffect("primitive_map_cull", float(n), float(n)))


def primitive_map_forget(atlas_map: AtlasMap, tile_id: int,
                         forgetting_factor: float = GC_PRIMITIVE_FORGETTING_FACTOR, chart_id: str = CHART_ID,
                         anchor_id: str = "primitive_map"):
    """:1314-1384: weights *= gamma (a missing tile: exact no-op)."""
    idx = atlas_map.index(tile_id, create=False)
    if idx < 0:
        return (PrimitiveMapForgetResult(atlas_map, int(tile_id)),) + _exact(chart_id, anchor_id,
                                                                             "primitive_map_forget")
    ip = _tiles_arg([idx])
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_forget(atlas_map.h, ip[1], 1, float(forgetting_factor)),
                   "gcs_pmap_forget")
    g = float(forgetting_factor)
    return (PrimitiveMapForgetResult(atlas_map, int(tile_id)), CertBundle.create_exact(chart_id, anchor_id),
            ExpectedEffect("primitive_map_forget", 1.0 - g, 1.0 - g))


def primitive_map_recency_inflate(atlas_map: AtlasMap, tile_ids: List[int], scan_seq: int,
                                  recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA,
                                  min_scale: float = GC_RECENCY_MIN_SCALE, chart_id: str = CHART_ID,
                                  anchor_id: str = "primitive_map_recency_inflate"):
    """:1400-1484: precision (Lambda, theta) of stale primitives scaled by clip(exp(-lambda dt))."""
    present = [atlas_map.tiles[int(t)] for t in tile_ids if int(t) in atlas_map.tiles]
    st = np.zeros(3)
    if present:
        ip = _tiles_arg(present)
        atlas_map._stream()
        atlas_map._chk(atlas_map.lib.gcs_pmap_recency_inflate(atlas_map.h, ip[1], len(present), int(scan_seq),
                                                              float(recency_decay_lambda), float(min_scale),
                                                              L.dptr(st)), "gcs_pmap_recency_inflate")
    down, infl, nv = float(st[0]), float(st[1]), float(st[2])
    stats = PrimitiveMapRecencyInflateStats(down / max(nv, 1.0), infl, down)
    return (atlas_map, CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect("primitive_map_recency_inflate", nv, nv), stats)


def primitive_map_merge_reduce(atlas_map: AtlasMap, tile_id: int,
                               merge_threshold: float = GC_PRIMITIVE_MERGE_THRESHOLD,
                               max_pairs: int = GC_K_MERGE_PAIRS_PER_TILE,
                               max_tile_size: int = GC_PRIMITIVE_MERGE_MAX_TILE_SIZE, eps_psd: float = GC_EPS_PSD,
                               eps_lift: float = GC_EPS_LIFT, chart_id: str = CHART_ID,
                               anchor_id: str = "primitive_map"):
    """:1809-2031: greedy disjoint pairs by Bhattacharyya distance below the threshold, moment-matched
    (Frobenius-corrected approximation).  A tile over max_tile_size returns the budget-cap cert."""
    def no_op(predicted, triggers=None, influence=None):
        res = PrimitiveMapMergeReduceResult(atlas_map, int(tile_id), 0, 0.0)
        cert = (CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=triggers,
                                         frobenius_applied=True, influence=influence or InfluenceCert.identity())
                if triggers else CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id))
        return res, cert, ExpectedEffect("primitive_map_merge_reduce", predicted, 0.0)

    idx = atlas_map.index(tile_id, create=False)
    if idx < 0:
        return no_op(0.0)
    M = atlas_map.m_tile
    if M < 2 or atlas_map.counts.get(int(tile_id), 0) < 2 or int(max_pairs) <= 0:
        return no_op(float(max_pairs))
    if int(max_tile_size) > 0 and M > int(max_tile_size):
        over = float(M - int(max_tile_size)) / float(max(M, 1))
        return no_op(float(max_pairs), ["merge_reduce_budget_cap"],
                     InfluenceCert.identity().with_overrides(mass_epsilon_ratio=over))
    nm, cnt = np.zeros(1, np.int32), np.zeros(1, np.int32)
    pairs = np.zeros(2 * int(max_pairs), np.int32)
    atlas_map._stream()
    atlas_map._chk(atlas_map.lib.gcs_pmap_merge_reduce(atlas_map.h, idx, float(merge_threshold), int(max_pairs),
                                                       float(eps_psd), float(eps_lift), L.iptr(nm), L.iptr(pairs),
                                                       L.iptr(cnt)), "gcs_pmap_merge_reduce")
    n = int(nm[0])
    atlas_map.last_merge_pairs = [(int(pairs[2 * k]), int(pairs[2 * k + 1])) for k in range(n)]
    if n <= 0:
        return no_op(float(max_pairs))
    atlas_map.counts[int(tile_id)] = int(cnt[0])
    atlas_map.total_count -= n
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["primitive_map_merge_reduce"],
                                    frobenius_applied=True, influence=InfluenceCert.identity().with_overrides(
                                        mass_epsilon_ratio=float(n) / float(max(M, 1))))
    return (PrimitiveMapMergeReduceResult(atlas_map, int(tile_id), n, float(n)), cert,
            ExpectedEffect("primitive_map_merge_reduce", float(max_pairs), float(n)))


def ma_hex_stencil_tile_ids(center_xyz, h_tile: float, radius_xy: int, radius_z: int) -> List[int]:
    """tiling.py:167-209: the packed MA-hex tile ids of the hex disk (radius_xy, sorted axial order) x
    z slab (radius_z, outer) around the cell of center_xyz -- the active / stencil tiles of a scan."""
    x, y, z = (float(v) for v in np.asarray(center_xyz, dtype=np.float64).ravel()[:3])
    h = max(float(h_tile), 1e-12)
    c1 = int(np.floor(x / h))
    c2 = int(np.floor((x * 0.5 + y * (np.sqrt(3.0) * 0.5)) / h))
    cz = int(np.floor(z / h))
    r = int(radius_xy)
    disk = sorted((q, rr) for q in range(-r, r + 1) for rr in range(max(-r, -q - r), min(r, -q + r) + 1))
    bits, bias = 21, 1 << 20
    mask = (1 << bits) - 1

    def pack(a, b, c):
        return (((a + bias) & mask) << (2 * bits)) | (((b + bias) & mask) << bits) | ((c + bias) & mask)

    return [int(pack(c1 + dq, c2 + dr, cz + dz)) for dz in range(-int(radius_z), int(radius_z) + 1)
            for dq, dr in disk]


@dataclass
class PrimitiveMapUpdateConfig:
    """The PipelineConfig fields step 12b reads (pipeline.py:187-206)."""
    k_insert_tile: int = 64                  # GC_K_INSERT_TILE
    block_size: int = 256                    # GC_ASSOC_BLOCK_SIZE
    k_merge_pairs_tile: int = GC_K_MERGE_PAIRS_PER_TILE
    primitive_merge_max_tile_size: int = GC_PRIMITIVE_MERGE_MAX_TILE_SIZE
    H_TILE: float = 2.0
    RECENCY_DECAY_LAMBDA: float = GC_RECENCY_DECAY_LAMBDA
    primitive_cull_weight_threshold: float = GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD
    primitive_forgetting_factor: float = GC_PRIMITIVE_FORGETTING_FACTOR
    primitive_merge_threshold: float = GC_PRIMITIVE_MERGE_THRESHOLD
    eps_lift: float = GC_EPS_LIFT
    eps_mass: float = GC_EPS_MASS
    eps_psd: float = GC_EPS_PSD


def update_config_struct(cfg: PrimitiveMapUpdateConfig):
    """gcs_pmap_update_config of a PrimitiveMapUpdateConfig."""
    return L.GcsPmapUpdateConfig(int(cfg.k_insert_tile), int(cfg.block_size), int(cfg.k_merge_pairs_tile),
                                 int(cfg.primitive_merge_max_tile_size), float(cfg.H_TILE),
                                 float(cfg.RECENCY_DECAY_LAMBDA), float(cfg.primitive_cull_weight_threshold),
                                 float(cfg.primitive_forgetting_factor), float(cfg.primitive_merge_threshold),
                                 float(cfg.eps_lift), float(cfg.eps_mass), float(cfg.eps_psd))


def primitive_map_update(atlas_map: AtlasMap, measurement_batch, assoc_result, z_t, active_tile_ids: List[int],
                         timestamp: float, scan_seq: int, config: Optional[PrimitiveMapUpdateConfig] = None) -> dict:
    """pipeline.py:1244-1447 (step 12b) on the GPU: the scan's MeasurementBatch (body frame) fused into
    the active tiles at z_t = [t, rotvec] through the association result, novelty insertion, then
    cull / forget / merge-reduce per tile.  Returns the MapUpdateCert counters (:1457-1486)."""
    return primitive_map_update_call(atlas_map, measurement_batch, assoc_result, z_t, active_tile_ids, timestamp,
                                     config)(scan_seq)


def primitive_map_update_call(atlas_map: AtlasMap, measurement_batch, assoc_result, z_t, active_tile_ids: List[int],
                              timestamp: float, config: Optional[PrimitiveMapUpdateConfig] = None):
    """`primitive_map_update` with its C-ABI arguments built once: call(scan_seq) runs
    gcs_pmap_map_update on them (the boundary call a C caller makes; tools/pmap_bench.py times it
    beside the Python call) and returns the MapUpdateCert counters."""
    torch = _torch()
    cfg = config or PrimitiveMapUpdateConfig()
    dev = f"cuda:{atlas_map.device}"
    f64 = lambda x: torch.as_tensor(x, device=dev).to(torch.float64).contiguous()  # noqa: E731
    i64 = lambda x: torch.as_tensor(x, device=dev).to(torch.int64).contiguous()  # noqa: E731
    b, a = measurement_batch, assoc_result
    keep = [f64(b.Lambdas), f64(b.thetas), f64(b.etas), f64(b.weights),
            torch.as_tensor(b.valid_mask, device=dev).to(torch.uint8).contiguous(),
            f64(b.colors) if getattr(b, "colors", None) is not None else None,
            torch.as_tensor(b.sources, device=dev).to(torch.int32).contiguous()
            if getattr(b, "sources", None) is not None else None,
            f64(a.responsibilities), i64(a.candidate_tile_ids), i64(a.candidate_slots), f64(a.row_masses)]
    N, K = int(keep[7].shape[0]), int(keep[7].shape[1])
    inp = L.GcsPmapUpdateInputs()
    for name, t in zip(("Lambdas", "thetas", "etas", "weights", "valid", "colors", "sources", "responsibilities",
                        "candidate_tile_ids", "candidate_slots", "row_masses"), keep):
        setattr(inp, name, t.data_ptr() if t is not None else None)
    inp.n_total, inp.n_lobes, inp.k_assoc = N, int(keep[2].reshape(N, -1, 3).shape[1]), K
    c = update_config_struct(cfg)
    idx, ip = _tiles_arg([atlas_map.index(t, create=True) for t in active_tile_ids])
    tids = np.ascontiguousarray(np.asarray(active_tile_ids, dtype=np.int64))
    z = np.ascontiguousarray(np.asarray(z_t, dtype=np.float64).reshape(6))
    nxt = np.array([atlas_map.next_global_id], dtype=np.int64)
    cnt = np.zeros(max(len(active_tile_ids), 1), np.int32)
    st = L.GcsPmapUpdateStats()
    atlas_map._stream()
    lib, h = atlas_map.lib, atlas_map.h
    args = (h, ip, tids.ctypes.data_as(L.c_int64_p), len(active_tile_ids), L.dptr(z), float(timestamp))
    tail = (nxt.ctypes.data_as(L.c_int64_p), C.byref(c), C.byref(inp), C.byref(st), L.iptr(cnt))

    def call(scan_seq: int) -> dict:
        nxt[0] = atlas_map.next_global_id
        atlas_map._chk(lib.gcs_pmap_map_update(*args, int(scan_seq), *tail), "gcs_pmap_map_update")
        atlas_map.total_count += int(st.insert_count_total) - int(st.evicted_count) - int(st.merged_count)
        atlas_map.next_global_id = int(nxt[0])
        for k, t in enumerate(active_tile_ids):
            atlas_map.counts[int(t)] = int(cnt[k])
        return dict(n_active_tiles=len(active_tile_ids), tile_ids_active=[int(t) for t in active_tile_ids],
                    insert_count_total=int(st.insert_count_total), insert_mass_total=float(st.insert_mass_total),
                    insert_mass_p95=float(st.insert_mass_p95), evicted_count=int(st.evicted_count),
                    evicted_mass_total=float(st.evicted_mass_total), fused_count=int(st.fused_count),
                    fused_mass_total=float(st.fused_mass_total), merged_count=int(st.merged_count))
    call.keep = (keep, inp, c, idx, ip, tids, z, nxt, cnt, st)
    return call
