"""Long run of the bench's cycled synthetic scans (bench.py: 8 resident scans, one hypothesis, host-only
combine) recording each scan's diagnostics, to find where a long sequence first turns non-finite:

    python tools/long_run.py [c2|c3] [N_SCANS_TOTAL]

Prints one JSON line per scan around the end (the last 12 before a failure, or every 50th), each with
z_t, the belief's max |L|, trace L and max |h|, the fusion scale and the evidence certificates that
gate it (cert[33] alpha, [34] fusion PSD delta, [49] pose-6 conditioning, [52] quality), the scan's
L_evidence / h_evidence norms and the IMU / odometry evidence norms."""

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gc-slam_amd")]

import bench  # noqa: E402
from gcslam import _lib as L  # noqa: E402
from gcslam.synthetic import scan_kwargs  # noqa: E402


def main():
    import torch
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    total = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    cfg = bench.CONFIGS[cfg_name]
    N = cfg["N"]
    ctx = bench.make_ctx(cfg, 0)
    ctx.set_belief(np.zeros(6), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
    scans = bench.resident_scans(N, "cuda:0")
    prepared = [ctx.prepare_scan(rec, 16, t, w, N, **scan_kwargs(sc)) for sc, rec, t, w in scans]
    out = L.GcsScanOutputs()
    scan_fn = ctx.scan_call(out)
    combine = ctx.combine_call(None, 1.0, 1.0)
    restart = os.environ.get("LONG_RESTART", "1") == "1"  # bench.py's per-pass restart of the belief
    hist = []
    err = None
    for s in range(total):
        try:
            if restart and s and s % bench.N_SCANS == 0:
                ctx.set_belief(np.zeros(6), 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
            scan_fn(prepared[s % bench.N_SCANS])
            combine(s)
        except (RuntimeError, ValueError) as e:
            err = f"scan {s}: {e}"
            break
        b = out.belief
        Lb = np.array(b.L[:]).reshape(22, 22)
        Le = np.array(out.L_evidence[:]).reshape(22, 22)
        Lio = np.array(out.L_imu_odom[:]).reshape(22, 22)
        c = np.array(out.cert[:])
        hist.append(dict(scan=s, z_t=[round(x, 6) for x in out.z_t[:]], X=[round(x, 4) for x in b.X_anchor[:]],
                         L_max=float(np.abs(Lb).max()), L_tr=float(np.trace(Lb)), h_max=float(np.abs(np.array(b.h[:])).max()),
                         alpha=float(c[33]), fdelta=float(c[34]), c6cond=float(c[49]), quality=float(c[52]),
                         Lev_max=float(np.abs(Le).max()), hev_max=float(np.abs(np.array(out.h_evidence[:])).max()),
                         Lio_max=float(np.abs(Lio).max()), finite_ev=bool(np.all(np.isfinite(Le))),
                         finite_io=bool(np.all(np.isfinite(Lio)))))
    torch.cuda.synchronize()
    show = hist[-12:] if err else hist[::50] + hist[-2:]
    for r in show:
        print(json.dumps(r), flush=True)
    print(json.dumps(dict(config=cfg_name, scans_run=len(hist), error=err, restart=restart)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
