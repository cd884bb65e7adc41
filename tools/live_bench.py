#!/usr/bin/env python3
"""bench.py's live_path measurement alone (one JSON line): the one-call live primitive path
(gcs_live_scan) and the per-operator path on the following scans, at the reference's sizes.

  python tools/live_bench.py [steps=30]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), ROOT]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    import bench
    r = bench.live_path_bench(0, steps=steps)
    from gcslam import pipeline as P
    if P.LIVE_STAMPS:  # GCSLAM_LIVE_STAMPS=1: mean us between consecutive phase stamps (calls of the chain path)
        seq, acc, cnt = P.LIVE_STAMPS, {}, {}
        for (a, ta), (b, tb) in zip(seq, seq[1:]):
            k = f"{a}->{b}"
            acc[k] = acc.get(k, 0.0) + (tb - ta) * 1e6
            cnt[k] = cnt.get(k, 0) + 1
        r["host_phases_us"] = {k: round(acc[k] / cnt[k], 1) for k in acc if cnt[k] >= 5}
        import numpy as np
        ph = np.array(P.LIVE_PHASES)
        r["live_scan_phases_us"] = dict(zip(("begin", "surfels_read", "pose_evidence_read", "finish", "12b_queued",
                                             "collect_wait"), np.round(ph.mean(0), 1).tolist()))
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
