"""Timing of gcs_extract_lidar_surfels on synthetic scans (8,192 = the reference budget, and 65,536
points), inputs resident in HBM: mean wall time per call over 200 calls (includes the final stream
sync and the n_valid read-back)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd")]


def main():
    import torch
    from gcslam import synthetic
    from gcslam.surfels import SurfelExtractor
    for n in (8192, 65536):
        sc = synthetic.make_scan(n, 1)
        p = torch.from_numpy(sc["points"]).cuda()
        t = torch.from_numpy(sc["timestamps"]).cuda()
        w = torch.from_numpy(sc["weights"]).cuda()
        ex = SurfelExtractor(max_points=n)
        for _ in range(10):
            r = ex.extract(p, t, w)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            r = ex.extract(p, t, w)
        dt = (time.perf_counter() - t0) / 200
        print(f"N={n}: {dt * 1e6:.1f} us per extract_lidar_surfels, n_valid {r['n_valid']}", flush=True)
        ex.close()


if __name__ == "__main__":
    main()
