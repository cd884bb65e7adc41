"""Bitwise snapshot of the bin path's device results, for A/B across a kernel change.

  python tools/bitwise_snapshot.py save OUT.npz     (on the GPU box, with the library under test)
  python tools/bitwise_snapshot.py compare A.npz B.npz

`save` runs fixed seeded scans through gcs_scan at C2 (65,536 x 100,000) and C3 (262,144 x 1,048,576),
a budget-stride case (131,072 raw points into a 32,768 cap), the sorted bucketing, and the per-operator
point stage + soft assign (responsibilities), and stores every result array.  `compare` reports, per
array, whether the two snapshots are bitwise equal and otherwise the largest relative difference.
"""

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gc-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

ORIGIN = (0.0, 0.0, 0.5)
XI = np.array([0.1, 0.002, 0.0, 0.0, 0.001, 0.03])


def _run(tag, out, n_raw, cap, B, scans, seed0, sorted_buckets=False, per_op=False):
    import torch
    from gcslam import _lib as L, synthetic
    from gcslam.context import HypothesisContext
    from gcslam.synthetic import scan_kwargs

    t0 = time.time()
    ctx = HypothesisContext(n_bins=B, n_points_cap=cap, mode="scale", k_cand=16, lidar_origin=ORIGIN,
                            max_raw_points=max(n_raw, 1 << 16))
    if sorted_buckets:
        ctx.set_debug(L.DEBUG_SORTED_BUCKETS, 1)
    for k in range(scans):
        sc = synthetic.make_scan(n_raw, seed0 + k)
        rec = torch.from_numpy(np.ascontiguousarray(sc["xyz_record"])).cuda()
        t = torch.from_numpy(np.ascontiguousarray(sc["timestamps"])).cuda()
        w = torch.from_numpy(np.ascontiguousarray(sc["weights"])).cuda()
        o = ctx.scan(rec, 16, t, w, n_raw, **scan_kwargs(sc))
        X, _, z, Lm, h = ctx.get_belief()
        out[f"{tag}/s{k}/z_t"] = np.array(o.z_t[:])
        out[f"{tag}/s{k}/cert"] = np.array(o.cert[:])
        out[f"{tag}/s{k}/X"] = np.asarray(X)
        out[f"{tag}/s{k}/L"] = np.asarray(Lm)
        out[f"{tag}/s{k}/h"] = np.asarray(h)
        out[f"{tag}/s{k}/scan_stats"] = np.asarray(ctx.get_scan_stats())
        m, d = ctx.get_map()
        out[f"{tag}/s{k}/map"] = np.asarray(m)
    if per_op:
        sc = synthetic.make_scan(n_raw, seed0 + 100)
        rec = torch.from_numpy(np.ascontiguousarray(sc["xyz_record"])).cuda()
        t = torch.from_numpy(np.ascontiguousarray(sc["timestamps"])).cuda()
        w = torch.from_numpy(np.ascontiguousarray(sc["weights"])).cuda()
        ps = ctx.point_stage(rec, 16, t, w, n_raw, sc["scan_start_time"], sc["scan_end_time"], XI)
        ids, r = ctx.bin_soft_assign()
        out[f"{tag}/op/ids"] = ids.cpu().numpy()
        out[f"{tag}/op/r"] = r.cpu().numpy()
        out[f"{tag}/op/points"] = ps["points"].cpu().numpy()
        cert = ctx.scan_bin_moment_match()
        out[f"{tag}/op/mm_cert"] = np.asarray(cert)
        out[f"{tag}/op/scan_stats"] = np.asarray(ctx.get_scan_stats())
    ctx.close()
    print(f"{tag}: {time.time() - t0:.1f} s", flush=True)


def _shrink(out):
    """Large arrays (C3: 218 MB of ScanBinStats per scan) become a SHA-1 of their bytes plus a strided
    sample (every 61st element) for the relative difference; the rest is kept whole."""
    import hashlib
    res = {}
    for k, v in out.items():
        v = np.ascontiguousarray(v)
        if v.size > (1 << 16):
            res[k + "#sha1"] = np.array(hashlib.sha1(v.view(np.uint8)).hexdigest())
            res[k + "#sample"] = v.reshape(-1)[::61].copy()
            if v.ndim == 2 and v.shape[0] <= 32:  # field-major (F, B): a hash per field row
                for f in range(v.shape[0]):
                    res[f"{k}#f{f:02d}"] = np.array(hashlib.sha1(np.ascontiguousarray(v[f]).view(np.uint8)).hexdigest())
        else:
            res[k] = v
    return res


def save(path):
    out = {}
    _run("c2", out, 65536, 65536, 100000, 3, 60, per_op=True)
    _run("c2sorted", out, 65536, 65536, 100000, 2, 60, sorted_buckets=True)
    _run("stride", out, 131072, 32768, 100000, 2, 90, per_op=True)
    _run("c3", out, 262144, 262144, 1048576, 2, 80, per_op=True)
    out = _shrink(out)
    np.savez_compressed(path, **out)
    print("saved", path, len(out), "arrays")


def compare(pa, pb):
    a, b = np.load(pa), np.load(pb)
    keys = sorted(set(a.files) | set(b.files))
    n_eq = 0
    for k in keys:
        if k not in a.files or k not in b.files:
            print(f"{k}: missing in {'A' if k not in a.files else 'B'}")
            continue
        x, y = a[k], b[k]
        if x.shape != y.shape:
            print(f"{k}: shape {x.shape} vs {y.shape}")
            continue
        if x.dtype.kind == "U":
            if x == y:
                n_eq += 1
            else:
                print(f"{k}: hash differs")
            continue
        if np.array_equal(x.view(np.uint8), y.view(np.uint8)):
            n_eq += 1
            continue
        xf, yf = x.astype(np.float64), y.astype(np.float64)
        den = np.maximum(np.abs(xf), np.abs(yf))
        rel = np.where(den > 0, np.abs(xf - yf) / np.where(den > 0, den, 1.0), 0.0)
        print(f"{k}: differs in {np.count_nonzero(x != y)} / {x.size}; max rel {np.nanmax(rel):.3e}, "
              f"max abs {np.nanmax(np.abs(xf - yf)):.3e}")
    print(f"{n_eq} / {len(keys)} arrays bitwise equal")


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
