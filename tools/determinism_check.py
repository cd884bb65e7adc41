#!/usr/bin/env python3
"""Run-to-run determinism of the scale-mode scan sequence (the trajectory test's: 12 scans, B = 5,000,
N = 4,096, the hypothesis combine after each): REPS fresh contexts in one process, each sequence's
per-scan z_t compared bitwise with the first's.  Prints the number of distinct sequences and the
largest z_t difference.

  python tools/determinism_check.py [reps=20]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), os.path.join(ROOT, "tests"), ROOT]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch
    from golden_util import ORIGIN
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    from gcslam.synthetic import scan_kwargs
    scans = [synthetic.make_scan(4096, s) for s in range(12)]
    runs = []
    for r in range(reps):
        ctx = HypothesisContext(n_bins=5000, n_points_cap=4096, max_raw_points=4096, mode="scale",
                                lidar_origin=tuple(ORIGIN))
        zs = []
        try:
            for s, sc in enumerate(scans):
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                out = ctx.scan(rec, 16, t, w, 4096, **scan_kwargs(sc))
                zs.append(np.array(out.z_t[:], np.float64))
                combine_allreduce(ctx, 0, 1, s, want_belief=False)
        finally:
            ctx.close()
        runs.append(np.stack(zs))
        # other GPU work between the sequences (fresh allocations land on reused memory)
        junk = torch.randn(1 << 22, device="cuda") * (r + 1)
        del junk
    base = runs[0]
    diffs = [float(np.abs(z - base).max()) for z in runs]
    distinct = len({z.tobytes() for z in runs})
    print(f"{reps} sequences: {distinct} distinct; max |z - z_first| per run: "
          + " ".join(f"{d:.1e}" for d in diffs), flush=True)


if __name__ == "__main__":
    main()
