#!/usr/bin/env python3
"""Timing of the primitive map on the GPU at the reference sizes: 7 active tiles of m_tile = 50,000
slots (GC_PRIMITIVE_MAP_MAX_SIZE), ~80 % valid, m_tile_view 1024, a MeasurementBatch of 1,536 rows
(GC_N_FEAT + GC_N_SURFEL) with an association result of k_assoc 8: wall time per call (each call
synchronises) of extract_atlas_map_view, step 12b (primitive_map_update: 6 fuse blocks, 7 x 64
proposals, cull, forget; merge-reduce is budget-capped at this tile size, as in the reference) and
recency_inflate.  With "cpu" as the second argument the numpy oracle runs the same view and step 12b
once (the CPU baseline of this path).  Run under rocprofv3 --kernel-trace --stats for the split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), ROOT]


def scene(rng, M, n_tiles, N, K, NL=3):
    import numpy as np
    from oracle import primitive_map as opm
    tiles = {}
    base = 1 << 40
    tids = [base + 17 * k for k in range(n_tiles)]
    for tid in tids:
        t = opm.create_empty_tile(M, NL)
        t["valid_mask"][:] = rng.random(M) < 0.8
        t["weights"][:] = rng.random(M)
        A = rng.normal(size=(M, 3, 3)) * 0.2
        t["Lambdas"][:] = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * 2.0
        t["thetas"][:] = rng.normal(size=(M, 3))
        t["etas"][:] = rng.normal(size=(M, NL, 3))
        t["last_supported_scan_seq"][:] = rng.integers(0, 50, M)
        t["primitive_ids"][:] = np.arange(M)
        tiles[tid] = t
    p = rng.uniform(-5, 5, size=(N, 3))
    A = rng.normal(size=(N, 3, 3)) * 0.2
    Lam = np.einsum("nij,nkj->nik", A, A) + np.eye(3)[None] * 3.0
    batch = dict(Lambdas=Lam, thetas=np.einsum("nij,nj->ni", Lam, p), etas=rng.normal(size=(N, NL, 3)),
                 weights=rng.random(N), valid_mask=rng.random(N) < 0.9, colors=rng.random((N, 3)),
                 sources=rng.integers(0, 2, N).astype(np.int32))
    assoc = dict(responsibilities=rng.random((N, K)) / K, candidate_tile_ids=rng.choice(np.array(tids), size=(N, K)),
                 candidate_slots=rng.integers(0, M, size=(N, K)), row_masses=rng.random(N) / N)
    return tiles, tids, batch, assoc


def main():
    import numpy as np
    import torch
    from types import SimpleNamespace
    from gcslam import primitive_map as gpm
    M, T, N, K = 50000, 7, 1536, 8
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rng = np.random.default_rng(0)
    tiles, tids, batch, assoc = scene(rng, M, T, N, K)
    z = np.array([0.3, -0.2, 0.1, 0.01, 0.02, 0.3])
    if len(sys.argv) > 2 and sys.argv[2] == "cpu":
        from oracle import primitive_map as opm, se3
        t0 = time.perf_counter()
        opm.extract_atlas_map_view(tiles, tids, 1024, M)
        t1 = time.perf_counter()
        opm.map_update_step(tiles, 0, batch, assoc, se3.so3_exp(z[3:]), z[:3], tids, M, 1.0, 60)
        t2 = time.perf_counter()
        print(f"oracle (numpy, 1 core): extract_atlas_map_view {1e3 * (t1 - t0):.1f} ms, "
              f"step 12b {1e3 * (t2 - t1):.1f} ms")
        return
    am = gpm.AtlasMap(m_tile=M, max_tiles=16, max_merge=0)
    for tid, t in tiles.items():
        am.write_tile(tid, t)
    dev = "cuda:0"
    b = SimpleNamespace(**{k: torch.as_tensor(v, device=dev) for k, v in batch.items()})
    a = SimpleNamespace(**{k: torch.as_tensor(v, device=dev) for k, v in assoc.items()})

    def timed(fn, n):
        for _ in range(2):
            fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return np.median(ts) * 1e3, np.percentile(ts, 90) * 1e3

    seq = [60]

    def upd():
        seq[0] += 1
        gpm.primitive_map_update(am, b, a, z, tids, 1.0, seq[0])

    # the C-ABI call alone (outputs allocated once, tile list prepared once): what a C caller pays
    import ctypes as C
    from gcslam import _lib as L
    out = gpm.extract_atlas_map_view(am, tids, 1024)
    vs = L.GcsPmapView()
    for name, _ in vs._fields_:
        setattr(vs, name, getattr(out, name).data_ptr())
    idx = np.ascontiguousarray(np.asarray([am.index(t, create=False) for t in tids], np.int32))
    tid_arr = np.ascontiguousarray(np.asarray(tids, np.int64))
    ip, tp = L.iptr(idx), tid_arr.ctypes.data_as(L.c_int64_p)

    def view_c():
        am._chk(am.lib.gcs_pmap_extract_view(am.h, ip, tp, len(tids), 1024, 1e-9, 1e-12, C.byref(vs)), "view")

    upd_call = gpm.primitive_map_update_call(am, b, a, z, tids, 1.0)

    def upd_c():
        seq[0] += 1
        upd_call(seq[0])

    for name, fn in (("extract_atlas_map_view 7 x 50,000 -> 7 x 1024", lambda: gpm.extract_atlas_map_view(am, tids, 1024)),
                     ("gcs_pmap_extract_view (C-ABI call alone) 7 x 50,000 -> 7 x 1024", view_c),
                     ("primitive_map_update (step 12b) N=1536 K=8, 7 tiles", upd),
                     ("gcs_pmap_map_update (step 12b, C-ABI call alone) N=1536 K=8, 7 tiles", upd_c),
                     ("primitive_map_recency_inflate 7 tiles", lambda: gpm.primitive_map_recency_inflate(am, tids, 70))):
        med, p90 = timed(fn, iters)
        print(f"{name}: median {med:.3f} ms, p90 {p90:.3f} ms over {iters} calls")
    am.close()


if __name__ == "__main__":
    main()
