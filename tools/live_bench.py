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
    print(json.dumps(bench.live_path_bench(0, steps=steps)), flush=True)


if __name__ == "__main__":
    main()
