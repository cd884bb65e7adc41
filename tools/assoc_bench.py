#!/usr/bin/env python3
"""Timing of gcs_associate_primitives_ot at the reference sizes (N_total = 512 + 1024 rows, k_assoc 8,
7 stencil tiles x m_tile_view 1024, 50 Sinkhorn iterations) on a seeded scene (tests/assoc_util.py):
wall time per call (the call synchronises).  python tools/assoc_bench.py [reps=30] [iters=50,0,10].
Run under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), os.path.join(ROOT, "tests"), ROOT]


def main():
    import numpy as np
    import torch
    from assoc_util import make_scene
    from test_gpu_association import _batch, _view
    from gcslam import association as GA
    batch, view, _ = make_scene(seed=0)
    b, v = _batch(batch), _view(view)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    # the reference's 50 Sinkhorn iterations, then 0 and 10 (the slope is one iteration's cost)
    its = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (50, 0, 10)
    for iters in its:
        cfg = GA.AssociationConfig(scan_seq=10, k_sinkhorn=iters)
        for _ in range(3):
            GA.associate_primitives_ot(b, v, cfg)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            GA.associate_primitives_ot(b, v, cfg)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        print(f"associate_primitives_ot N=1536 K=8 pool=7x1024 k_sinkhorn={iters}: median {np.median(ts):.3f} ms, "
              f"p90 {np.percentile(ts, 90):.3f} ms over {len(ts)} calls", flush=True)
        # the C-ABI call alone (gcs_associate_primitives_ot on prepared device inputs; it synchronises)
        call = GA._associator_for(1536, 7 * 1024, 8, 0).prepare(b, v, cfg)
        for _ in range(3):
            call()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        print(f"  C-ABI gcs_associate_primitives_ot k_sinkhorn={iters}: median {np.median(ts):.3f} ms, "
              f"p90 {np.percentile(ts, 90):.3f} ms over {len(ts)} calls", flush=True)
    del torch


if __name__ == "__main__":
    main()
