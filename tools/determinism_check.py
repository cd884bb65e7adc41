#!/usr/bin/env python3
"""Run-to-run determinism of the scale-mode scan sequence (the trajectory test's: 12 scans, B = 5,000,
N = 4,096, the hypothesis combine after each): REPS fresh contexts in one process, each sequence's
per-scan z_t compared bitwise with the first's.  Prints the number of distinct sequences, the
largest z_t difference and any scan mirror that was re-read or taken after a stream synchronize.

  python tools/determinism_check.py [reps=20]      (DET_STAGES=1: also the first differing scan of each
                                                   device state checksum, gcs_debug_state_checksums;
                                                   DET_N / DET_B / DET_SCANS: the size, e.g. C3)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGES = os.environ.get("DET_STAGES", "0") == "1"  # also compare the device state checksums per scan (syncs)
PARTS = ["ScanBinStats", "map", "derived", "touched", "flags", "bin partial rows", "device scalars", "host mirror"]
sys.path[:0] = [os.path.join(ROOT, "gc-slam_amd"), os.path.join(ROOT, "tests"), ROOT]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch
    from golden_util import ORIGIN
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    from gcslam.synthetic import scan_kwargs
    N = int(os.environ.get("DET_N", "4096"))
    B = int(os.environ.get("DET_B", "5000"))
    n_scans = int(os.environ.get("DET_SCANS", "12"))
    scans = [synthetic.make_scan(N, s) for s in range(n_scans)]
    runs, st_runs = [], []
    DUMP = os.environ.get("DET_DUMP", "0") == "1"
    ref_ss = [None]
    for r in range(reps):
        stats = []
        ctx = HypothesisContext(n_bins=B, n_points_cap=N, max_raw_points=N, mode="scale",
                                lidar_origin=tuple(ORIGIN))
        zs = []
        try:
            for s, sc in enumerate(scans):
                rec = torch.from_numpy(sc["xyz_record"]).cuda()
                t = torch.from_numpy(sc["timestamps"]).cuda()
                w = torch.from_numpy(sc["weights"]).cuda()
                out = ctx.scan(rec, 16, t, w, N, **scan_kwargs(sc))
                zs.append(np.array(out.z_t[:], np.float64))
                combine_allreduce(ctx, 0, 1, s, want_belief=False)
                if STAGES:  # the device state the next scan reads, after this scan's pushforward
                    stats.append(ctx.state_checksums())
                if DUMP and s == 0:  # scan 0's ScanBinStats against the first run's: which fields / bins differ
                    ss = ctx.get_scan_stats()
                    if r == 0:
                        ref_ss[0] = ss
                    else:
                        d = np.nonzero(ss != ref_ss[0])
                        if len(d[0]):
                            fields = sorted(set(d[0].tolist()))
                            bins = sorted(set(d[1].tolist()))
                            ex = [(int(f), int(b), float(ref_ss[0][f, b]), float(ss[f, b]), float(ref_ss[0][0, b]),
                                   float(ss[0, b])) for f, b in list(zip(d[0], d[1]))[:8]]
                            print(f"run {r} scan 0: {len(d[0])} values differ; fields {fields}; {len(bins)} bins "
                                  f"(first {bins[:6]}); (field, bin, first run, this run, N first, N this) {ex}",
                                  flush=True)
            mstats = ctx.mirror_stats()
        finally:
            ctx.close()
        if mstats[1] or mstats[2]:
            print(f"run {r}: mirror accepted {mstats[0]}, re-read {mstats[1]}, via stream sync {mstats[2]}", flush=True)
        runs.append(np.stack(zs))
        st_runs.append(stats)
        # other GPU work between the sequences (fresh allocations land on reused memory)
        junk = torch.randn(1 << 22, device="cuda") * (r + 1)
        del junk
    base = runs[0]
    diffs = [float(np.abs(z - base).max()) for z in runs]
    distinct = len({z.tobytes() for z in runs})
    print(f"{reps} sequences: {distinct} distinct; max |z - z_first| per run: "
          + " ".join(f"{d:.1e}" for d in diffs), flush=True)
    if STAGES:  # per differing run: the first scan whose z_t or any state checksum differs
        for r in range(1, reps):
            fz = next((i for i in range(len(scans)) if not np.array_equal(runs[r][i], base[i])), None)
            first = {}
            for k, name in enumerate(PARTS):
                i = next((i for i in range(len(scans)) if st_runs[r][i][k] != st_runs[0][i][k]), None)
                if i is not None:
                    first[name] = i
            if fz is not None or first:
                print(f"run {r}: first differing scan -- z_t {fz}, state {first}", flush=True)


if __name__ == "__main__":
    main()
