#!/usr/bin/env python3
"""Per-block phase clocks of k_bins_scale (instrumented build: make -C gc-slam_amd prof).

Runs a few synthetic scans at C2 or C3 with GCSLAM_LIB pointing at libgcslam_hip_prof.so and
summarises the per-block stamps (wall_clock64, 100 MHz): phase durations for active and inactive
tiles, block lifetimes, start-time percentiles, staged records and per-bin work.
Usage: python tools/phase_prof.py [c2|c3]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))
os.environ.setdefault("GCSLAM_LIB", os.path.join(ROOT, "gc-slam_amd", "gcslam", "libgcslam_hip_prof.so"))


def main():
    import torch
    from gcslam import synthetic
    from gcslam.synthetic import scan_kwargs
    from gcslam.context import HypothesisContext
    cfg = {"c2": (65536, 100000), "c3": (262144, 1048576)}[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    N, B = cfg
    ctx = HypothesisContext(n_bins=B, n_points_cap=N, max_raw_points=N, mode="scale", k_cand=16,
                            lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
    for k in range(3):
        sc = synthetic.make_scan(N, k)
        rec = torch.from_numpy(sc["xyz_record"]).cuda()
        t = torch.from_numpy(sc["timestamps"]).cuda()
        w = torch.from_numpy(sc["weights"]).cuda()
        ctx.scan(rec, 16, t, w, N, **scan_kwargs(sc))
    ctx.synchronize()
    pc = (C.c_ulonglong * 4)()
    ctx.lib.gcs_debug_psd_count.argtypes = [C.c_void_p, C.c_int]
    assert ctx.lib.gcs_debug_psd_count(pc, 1) == 0
    print(f"3x3 PSD over 3 scans: non-zero inputs {pc[0]}, deflation path {pc[1]}, non-finite {pc[2]}")
    import re
    tb = int(re.search(r"(\d+)-bin tiles", ctx.describe()["backends"]["moment_match"]).group(1))
    nblk = (B + tb - 1) // tb
    print(f"tile: {tb} bins")
    buf = (C.c_ulonglong * (nblk * 16))()
    fn = ctx.lib.gcs_debug_prof
    fn.argtypes = [C.c_void_p, C.c_int]
    assert fn(buf, nblk * 16) == 0
    g = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 16).astype(np.int64)
    act = g[:, 7] == 1  # slot 7: 1 active, 0 inactive (zero rows written), 2 inactive and clean
    us = lambda x: x / 100.0  # noqa: E731  (100 MHz)
    t0 = g[:, 0].min()
    print(f"tiles {nblk}, active {act.sum()} ({act.mean():.1%})")
    print(f"kernel span {us(g[:, 6].max() - t0):.1f} us")
    life = us(g[:, 6] - g[:, 0])
    for name, m in (("active", act), ("inactive", g[:, 7] == 0), ("clean inactive", g[:, 7] == 2)):
        if not m.any():
            continue
        print(f"{name}: block life mean {life[m].mean():.2f} p90 {np.percentile(life[m], 90):.2f} max {life[m].max():.2f}")
        if name == "active":
            d = us(np.diff(g[m][:, 0:7], axis=1))
            print("  phases (A loads, rank+scan, stage, gather, finalize, reduce+store) mean",
                  np.round(d.mean(0), 2), "p90", np.round(np.percentile(d, 90, axis=0), 2))
            print(f"  staged records mean {g[m, 8].mean():.0f} p90 {np.percentile(g[m, 8], 90):.0f} max {g[m, 8].max()}"
                  f"; bin work max mean {g[m, 9].mean():.0f} max {g[m, 9].max()}; tile work mean {g[m, 10].mean():.0f}"
                  f" p90 {np.percentile(g[m, 10], 90):.0f} p99 {np.percentile(g[m, 10], 99):.0f} max {g[m, 10].max()}")
            if tb <= 64:  # phase D on wave 0 (wider tiles finalize on every wave: no hand-off stamps)
                ge = us(g[m][:, 11:14].max(1) - g[m][:, 4])
                print(f"  gather end, slowest of waves 1-3 minus wave 0: mean {ge.mean():.2f} p90 {np.percentile(ge, 90):.2f}")
                dd = us(np.diff(g[m][:, [4, 14, 15, 5]], axis=1))
                print("  phase D split (barriers, finalize_bin, MF term) mean", np.round(dd.mean(0), 2),
                      "p90", np.round(np.percentile(dd, 90, axis=0), 2))
            big = life[m] > np.percentile(life[m], 90)
            print(f"  slowest 10%: staged mean {g[m][big, 8].mean():.0f}, max-bin work mean {g[m][big, 9].mean():.0f}, "
                  f"tile work mean {g[m][big, 10].mean():.0f}")
        else:
            print(f"  count {m.sum()}")
    st = us(g[:, 0] - t0)
    print("block start percentiles (us) 0/10/25/50/75/90/100:", np.round(np.percentile(st, [0, 10, 25, 50, 75, 90, 100]), 2))
    ctx.close()


if __name__ == "__main__":
    main()
