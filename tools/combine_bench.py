#!/usr/bin/env python3
"""Latency of the per-scan hypothesis exchange (gcs_combine_allreduce) at world size 1: the host-only
combine (no communicator) against the RCCL path (world-1 communicator: stage in, ncclAllReduce, stage
out with sequence + checksum, host poll), one JSON line per run.  The environment picks the variant
(GCSLAM_COMBINE_GRAPH=0: direct calls instead of the captured graph; GCSLAM_COMBINE_PROBE=noccl: the
staging without the collective, a timing probe).

  python tools/combine_bench.py [calls=2000]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), ROOT]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import torch
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import HypothesisComm
    from gcslam.synthetic import scan_kwargs
    ctx = HypothesisContext(n_bins=5000, n_points_cap=4096, max_raw_points=4096, mode="scale",
                            lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
    sc = synthetic.make_scan(4096, 0)
    rec = torch.from_numpy(sc["xyz_record"]).cuda()
    t = torch.from_numpy(sc["timestamps"]).cuda()
    w = torch.from_numpy(sc["weights"]).cuda()
    ctx.scan(rec, 16, t, w, 4096, **scan_kwargs(sc))
    comm = HypothesisComm(0, 1, 0)
    out = {}
    for name, h in (("host", None), ("rccl", comm.h)):
        fn = ctx.combine_call(h, 1.0, 1.0)
        for i in range(50):
            fn(i)
        ts = np.empty(calls)
        for i in range(calls):
            t0 = time.perf_counter()
            fn(i)
            ts[i] = time.perf_counter() - t0
        out[name] = dict(median_us=float(np.median(ts) * 1e6), p90_us=float(np.percentile(ts, 90) * 1e6),
                         mean_us=float(ts.mean() * 1e6))
    out["mirror_stats"] = list(ctx.mirror_stats())
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("GCSLAM_COMBINE")}
    ctx.close()
    comm.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
