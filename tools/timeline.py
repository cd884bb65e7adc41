#!/usr/bin/env python3
"""Per-scan kernel timeline from a rocprofv3 kernel trace (run_kernel_trace.csv): for scan k (counted by a
marker kernel's launches) every kernel's start offset, the gap before it and its duration.

  python tools/timeline.py <kernel_trace.csv> [scan=15] [marker=k_budget]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    si = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_budget"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = starts[si], starts[si + 1]
    t0 = prev = int(rows[a]["Start_Timestamp"])
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f} {r['Kernel_Name'][:80]}")
        prev, busy = e, busy + e - s
    print(f"busy {busy / 1e3:.1f} us, span {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
