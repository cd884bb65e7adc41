#!/usr/bin/env python3
"""Device idle gaps of the per-scan kernel sequence, from a rocprofv3 --kernel-trace CSV.

  python tools/trace_gaps.py <run_kernel_trace.csv> [--skip 200] [--json out.json]

For every dispatch after the first --skip: the gap between its start and the latest end of any
earlier dispatch (the device was idle in between when the gap is positive -- across all queues, so
the pushforward on its own stream counts as busy time), grouped by kernel name: count, mean
duration, mean gap before it.  Also the device busy fraction over the window, which bounds what
hipGraph capture or fewer launches can recover (only the idle time)."""

import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name.replace("gcs::", "").replace("(anonymous namespace)::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=200)
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    rows = rows[a.skip:]
    if not rows:
        raise SystemExit("no dispatches after --skip")
    stats = defaultdict(lambda: [0, 0.0, 0.0, 0])  # count, dur, gap, gapped
    busy_end = rows[0][0]
    idle = 0.0
    for s, e, n in rows:
        gap = (s - busy_end) / 1e3
        st = stats[n]
        st[0] += 1
        st[1] += (e - s) / 1e3
        if gap > 0:
            st[2] += gap
            st[3] += 1
            idle += gap
        busy_end = max(busy_end, e)
    span = (busy_end - rows[0][0]) / 1e3
    out = dict(window_us=span, idle_us=idle, busy_frac=1.0 - idle / span if span else 0.0, dispatches=len(rows),
               kernels={n: dict(count=c, mean_us=d / c, mean_gap_before_us=g / c, gapped=k)
                        for n, (c, d, g, k) in sorted(stats.items(), key=lambda kv: -kv[1][1])})
    print(f"window {span:.1f} us, {len(rows)} dispatches, device idle {idle:.1f} us ({100 * idle / span:.1f} %)")
    print(f"{'kernel':60s} {'n':>6s} {'mean us':>8s} {'gap before':>10s}")
    for n, k in out["kernels"].items():
        print(f"{n[:60]:60s} {k['count']:6d} {k['mean_us']:8.2f} {k['mean_gap_before_us']:10.2f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
