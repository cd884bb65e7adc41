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
    if P.LIVE_STAMPS:  # GCSLAM_LIVE_STAMPS=1: mean us between the phase stamps of the timed chain calls
        import numpy as np
        calls, cur = [], None
        for name, t in P.LIVE_STAMPS:
            if name == "enter":
                cur = []
                calls.append(cur)
            cur.append((name, t))
        timed = calls[10:10 + steps]  # live_path_bench: 10 warm-up calls, then `steps` timed chain calls
        acc = {}
        for c in timed:
            for (a, ta), (b, tb) in zip(c, c[1:]):
                acc.setdefault(f"{a}->{b}", []).append((tb - ta) * 1e6)
        r["host_phases_us"] = {k: round(float(np.mean(v)), 1) for k, v in acc.items()}
        ph = np.array(P.LIVE_PHASES[10:10 + steps])
        names = ("begin", "surfels_queued", "surfels_read", "assoc_queued", "pose_evidence_read", "finish",
                 "12b_queued", "collect_wait")
        r["live_scan_phases_us"] = dict(zip(names, np.round(ph.mean(0)[:8], 1).tolist()))
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
