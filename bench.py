#!/usr/bin/env python3
"""Benchmark: scans/s of the 14-step bin-path pipeline (BASELINE.json metric) on MI355X.

One step = one hypothesis runs the full per-scan pipeline (budget, predict, IMU preintegration,
deskew, soft assign, moment match + kappa, Matrix-Fisher, planar translation, tempered evidence,
fusion, recompose, pushforward map update, anchor drift) on a synthetic 64k-point scan whose
inputs are already resident in HBM, followed by the per-scan hypothesis combine: a sum
all-reduce of the 840-f64 payload (RCCL over xGMI for N>1) and the IW/Q update on every rank.
Hypotheses are sharded one per GPU (weak scaling).  value = hypothesis-scans/s of the whole job.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3] [--no-cpu-baseline]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))

CONFIGS = {
    # BASELINE.json configs[1]: 1 hypothesis, 64k-pt synthetic scans vs 100k-surfel map
    "c2": dict(N=65536, B=100000, K=16),
    # BASELINE.json configs[2]: 256k-pt scans vs 1M-surfel map (roofline config)
    "c3": dict(N=262144, B=1048576, K=16),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
N_SCANS = 8             # distinct synthetic scans resident in HBM, cycled
TIMING_STRIDE = 8       # roofline kernel stamped on every 8th scan of the timed region


def bins_kernel_bytes(N, B):
    """Algorithmic bytes of one k_bins_scale launch (BinSoftAssign responsibilities + ScanBinMomentMatch
    + kappa + Matrix-Fisher terms): each point record (80 B: p0, ray direction, w, softmax shift,
    1/Z) read once, each bin direction (32 B, f64 padded) read once, ScanBinStats written once
    (26 f64 per bin).  DESIGN.md section 5 "Roofline of the dominant kernel"."""
    return N * 80 + B * (26 * 8 + 32)


def cpu_baseline(cfg, seconds_target=15.0):
    """The oracle (numpy restatement, `port`) on a bounded sample of the same workload: full
    14-step scans at the same N, B, K on one host core."""
    sys.path.insert(0, ROOT)
    from gcslam import synthetic
    from gcslam.synthetic import scan_kwargs
    from oracle import ops, pipeline as opipe
    N, B = cfg["N"], cfg["B"]
    bins = ops.fibonacci_atlas(B)
    knn = ops.bin_knn_table(bins, cfg["K"])
    pc = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", k_cand=cfg["K"],
                             lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(B)
    scans = [synthetic.make_scan(N, k) for k in range(2)]
    n, t_tot = 0, 0.0
    while n < 2 or (t_tot < seconds_target and n < 16):
        sc = scans[n % 2]
        t0 = time.perf_counter()
        r = opipe.process_scan_bin_path(b, sc, Q, pc, bins, knn, ms)
        t_tot += time.perf_counter() - t0
        b, ms = r["belief"], r["map"]
        n += 1
    return dict(value=n / t_tot, unit="scans/s", cores=1, kind="port",
                sample=f"{n} full 14-step scans (numpy oracle, scale mode) at N={N}, B={B}, K={cfg['K']} "
                       f"on 1 host core, {t_tot:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    device = f"cuda:{local_rank}"
    torch.cuda.set_device(local_rank)

    from gcslam import synthetic
    from gcslam.synthetic import scan_kwargs
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce

    cfg = CONFIGS[args.config]
    N, B, K = cfg["N"], cfg["B"], cfg["K"]
    ctx = HypothesisContext(n_bins=B, n_points_cap=N, max_raw_points=N, mode="scale", k_cand=K,
                            lidar_origin=tuple(synthetic.LIDAR_ORIGIN), device=local_rank)
    # hypothesis prior perturbed per rank (N(0, (0.05 m, 0.5 deg)))
    rng = np.random.default_rng(1000 + rank)
    X0 = np.concatenate([rng.normal(0, 0.05, 3) * (rank > 0), rng.normal(0, np.deg2rad(0.5), 3) * (rank > 0)])
    ctx.set_belief(X0, 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))

    scans = []
    for k in range(N_SCANS):
        sc = synthetic.make_scan(N, k)
        rec = torch.from_numpy(sc["xyz_record"]).to(device)
        t = torch.from_numpy(sc["timestamps"]).to(device)
        w = torch.from_numpy(sc["weights"]).to(device)
        scans.append((sc, rec, t, w))
    torch.cuda.synchronize()

    state = dict(count=0, sample=False)
    host_ms = np.zeros(5)  # pre-device host, device submit+wait, host tail, whole gcs_scan, combine

    def step():
        if state["sample"]:  # roofline-kernel event stamps on every TIMING_STRIDE-th scan
            phase = state["count"] % TIMING_STRIDE
            if phase == 0:
                ctx.enable_timing(True, stages=["bins"])
            elif phase == 1:
                ctx.enable_timing(False)
        sc, rec, t, w = scans[state["count"] % N_SCANS]
        out = ctx.scan(rec, 16, t, w, N, **scan_kwargs(sc))
        tc = time.perf_counter()
        combine_allreduce(ctx, rank, world, state["count"], device=device, want_belief=False)
        host_ms[4] += (time.perf_counter() - tc) * 1e3
        host_ms[:4] += np.asarray(out.stage_ms[:4])
        state["count"] += 1

    for _ in range(args.warmup):
        step()
    # timed region: only the roofline kernel carries event stamps, on a sample of the scans
    # (each stamped dispatch costs queue time)
    state["sample"] = True
    ctx.stage_times(reset=True)
    host_ms[:] = 0.0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    state["sample"] = False
    ms_sum, counts = ctx.stage_times(reset=True)
    bins_ms = float(ms_sum[2] / counts[2]) if counts[2] else None
    bins_samples = int(counts[2])
    host_avg = dict(zip(["pre_device", "device_wait", "tail", "gcs_scan", "combine"], (host_ms / args.steps).tolist()))
    # diagnostic pass after the timed region: every device stage stamped (not part of `value`)
    ctx.enable_timing(True)
    for _ in range(min(args.steps, 20)):
        step()
    ctx.synchronize()
    ms_sum, counts = ctx.stage_times(reset=True)
    stage_avg = {name: (float(ms_sum[i] / counts[i]) if counts[i] else None)
                 for i, name in enumerate(ctx.STAGES)}

    if rank == 0:
        value = world * args.steps / elapsed
        ach = bins_kernel_bytes(N, B) / (bins_ms * 1e-3) / 1e9 if bins_ms else None
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_bins_{args.config}.json")
        if os.path.exists(pmc_path):
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        line = {
            "metric": "scans/sec (14-step pipeline) at 64k pts/scan" if args.config == "c2"
                      else "scans/sec (14-step pipeline) at 256k pts/scan",
            "value": value, "unit": "scans/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (seeded VLP-16-like scans, box room, IMU 200 Hz)",
            "config": {"workload": f"{args.config}: {N}-pt scans vs {B}-bin map, K={K} candidates, "
                                   f"1 hypothesis per GPU ({world} hypotheses), RCCL payload all-reduce per scan",
                       "n_points": N, "n_bins": B, "k_cand": K, "hypotheses": world,
                       "parallelism": f"hyp{world}"},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (ach / HBM_PEAK_GBS) if ach else None, "traffic": traffic,
                         "kernel": "k_bins_scale (BinSoftAssign+ScanBinMomentMatch+kappa+MF terms)",
                         "algorithmic_bytes_per_launch": bins_kernel_bytes(N, B),
                         "kernel_us": bins_ms * 1e3 if bins_ms else None, "timed_launches": bins_samples},
            "stage_ms": stage_avg,
            "host_ms": host_avg,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
