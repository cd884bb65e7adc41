#!/usr/bin/env python3
"""Benchmark: scans/s of the 14-step bin-path pipeline (BASELINE.json metric) on MI355X.

One step = one hypothesis runs the full per-scan pipeline (budget, predict, IMU preintegration,
deskew, soft assign, moment match + kappa, Matrix-Fisher, planar translation, IMU/odometry
evidence, tempered fusion, recompose, pushforward map update, anchor drift) on a synthetic 64k-point
scan whose inputs are already resident in HBM, followed by the per-scan hypothesis combine: a sum
all-reduce of the 840-f64 payload (RCCL over xGMI for N>1) and the IW/Q update on every rank.
Hypotheses are sharded one per GPU (weak scaling): `value` counts hypothesis-scans of the whole
job; the multi-hypothesis node's scans/s is `scans_per_s_node` (= value / n_gpus).

Besides the headline line (C2 = BASELINE.json configs[1]) the same run measures, on rank 0 at N=1:
the roofline kernel at C3 (configs[2], `roofline_c3`), the pinned-host H2D of one raw scan
(`host_ms.h2d`), and the numpy oracle on the host cores (`cpu_baseline`: 1 core, all cores, and
the C1-equivalent N=8192 x B=48 dense case).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3] [--no-cpu-baseline] [--no-c3]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N, or plain
`python bench.py --gpus N`: without a launcher's WORLD_SIZE this process starts the N rank processes
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1) before touching any GPU, and exits
with their status.  `--cpu-rehearsal` runs the launcher + per-scan payload exchange on CPU over gloo
(library pack / apply on synthetic hypotheses; tests/test_bench_launcher.py), not a benchmark.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
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
METRIC = "scans/sec (14-step pipeline) at 64k pts/scan"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
N_SCANS = 8             # distinct synthetic scans resident in HBM, cycled
ROOFLINE_MIN = 16       # stamped launches of the roofline kernel inside the timed region (at least)


def timing_stride(steps):
    """Every TIMING_STRIDE-th scan of the timed region stamps the roofline kernel with HIP events on its
    stream: the largest stride (at most 8) that still stamps ROOFLINE_MIN launches inside the region
    (the driver's 20-step run: every scan).  GCSLAM_BENCH_STRIDE overrides (A/B of the stamping cost)."""
    e = os.environ.get("GCSLAM_BENCH_STRIDE")
    if e:
        return max(1, int(e))
    return max(1, min(8, steps // ROOFLINE_MIN))


def bins_kernel_bytes(N, B):
    """SURVEY.md 8(d) algorithmic bytes of the fused BinSoftAssign + ScanBinMomentMatch (+kappa)
    kernel with responsibilities not materialised: N (3 s_p + 8 + 8) [xyz f32, t, w] + B 3 s_d
    [bin directions, f64] read; B 26 s_o [ScanBinStats, f64] written.  Returns (read, write)."""
    return N * (3 * 4 + 8 + 8) + B * 3 * 8, B * 26 * 8


def pmc_chain_traffic(config):
    """HBM bytes per scan of the chain's kernels (k_budget, k_points*, k_bins_scale*, the bins fold's
    k_fold<16>/k_final<16>) from the committed PMC passes (profiles/pmc_bins_<cfg>.json)."""
    path = os.path.join(ROOT, "profiles", f"pmc_bins_{config}.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    per = {}
    for k, v in d.get("kernels", {}).items():
        for tag, pat in (("budget", "k_budget"), ("points", "k_points"), ("bins", "k_bins_scale"),
                         ("bins_fold", "k_fold<16"), ("bins_fold", "k_final<16")):
            if pat in k:
                per[tag] = per.get(tag, 0.0) + v["hbm_bytes"]
    if not {"points", "bins", "bins_fold"} <= set(per):
        return None, None
    return per, f"profiles/pmc_bins_{config}.json ({d.get('round', '?')})"


def roofline_chain(N, B, stage_avg, label, config=None):
    """The north star's "BinSoftAssign + ScanBinMomentMatch" as the kernel chain that implements it:
    k_budget (row 1) + k_points (rows 1, 3, 5: gather, deskew, direction, nearest bin, K-candidate
    softmax normaliser) + k_bins_scale (rows 4-6 + MF terms) + the bin kernel's partial-row fold,
    each timed by its own dispatch events, against the same SURVEY 8(d) bytes as `roofline`."""
    names = ("budget", "points", "bins", "bins_fold")
    if any(stage_avg.get(k) is None for k in names[1:]):
        return None
    # self-budget scans launch no k_budget (k_points sums the stride windows, the bin kernel folds the
    # rows): the chain is the three kernels that run
    names = names if stage_avg.get("budget") is not None else names[1:]
    ms = sum(stage_avg[k] for k in names)
    rd, wr = bins_kernel_bytes(N, B)
    s = ms * 1e-3
    ach = (rd + wr) / s / 1e9
    out = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "read_frac": rd / s / 1e9 / HBM_PEAK_GBS, "write_frac": wr / s / 1e9 / HBM_PEAK_GBS,
           "chain_us": ms * 1e3, "kernels_us": {k: stage_avg[k] * 1e3 for k in names},
           "budget": "k_budget" if "budget" in names else "in k_points (self-budget: no k_budget launch)",
           "algorithmic_bytes": rd + wr, "config": label}
    per, src = pmc_chain_traffic(config) if config else (None, None)
    if per:  # the counter-based traffic of the same kernels beside the algorithmic bytes
        per = {k: v for k, v in per.items() if k in names}
        t = sum(per.values())
        out.update(traffic=t, traffic_per_kernel=per, traffic_source=src, traffic_frac=t / s / 1e9 / HBM_PEAK_GBS)
    return out


def roofline(N, B, kernel_ms, traffic=None, traffic_source=None):
    rd, wr = bins_kernel_bytes(N, B)
    if not kernel_ms:
        return None
    s = kernel_ms * 1e-3
    ach = (rd + wr) / s / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "read_GBs": rd / s / 1e9, "read_frac": rd / s / 1e9 / HBM_PEAK_GBS,
            "write_GBs": wr / s / 1e9, "write_frac": wr / s / 1e9 / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": traffic_source,
            # the counter-based rate beside the algorithmic one: PMC HBM bytes per launch / the same duration
            "traffic_frac": (traffic / s / 1e9 / HBM_PEAK_GBS) if traffic else None,
            "kernel": "k_bins_scale (BinSoftAssign+ScanBinMomentMatch+kappa+MF terms)",
            "algorithmic_bytes_per_launch": rd + wr, "algorithmic_read_bytes": rd, "algorithmic_write_bytes": wr,
            "kernel_us": kernel_ms * 1e3}


# ---------------------------------------------------------------- CPU baseline (numpy oracle)
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_scans(N, B, mode, n_scans, seconds, seed0=0, core=None):
    """Time full 14-step oracle scans from the identity prior; returns (scans, seconds)."""
    if core is not None:
        os.sched_setaffinity(0, {core})
    from threadpoolctl import threadpool_limits
    sys.path.insert(0, ROOT)
    from gcslam import synthetic
    from oracle import ops, pipeline as opipe
    with threadpool_limits(1):
        bins = ops.fibonacci_atlas(B)
        knn = ops.bin_knn_table(bins, 16) if mode == "scale" else None
        pc = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode=mode, lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
        b = ops.Belief.identity_prior()
        Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
        ms = opipe.MapState.empty(B)
        scans = [synthetic.make_scan(N, seed0 + k) for k in range(2)]
        n, t_tot = 0, 0.0
        while n < 2 or (t_tot < seconds and n < n_scans):
            t0 = time.perf_counter()
            r = opipe.process_scan_bin_path(b, scans[n % 2], Q, pc, bins, knn, ms)
            t_tot += time.perf_counter() - t0
            b, ms = r["belief"], r["map"]
            n += 1
    return n, t_tot


def _pool_worker(args):
    core, N, B, barrier = args
    os.sched_setaffinity(0, {core})
    from threadpoolctl import threadpool_limits
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "gc-slam_amd"))
    from gcslam import synthetic
    from oracle import ops, pipeline as opipe
    # setup outside the timed window (imports, atlas, scan); all workers start at the barrier
    with threadpool_limits(1):
        bins = ops.fibonacci_atlas(B)
        knn = ops.bin_knn_table(bins, 16)
        pc = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
        Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
        sc = synthetic.make_scan(N, core % 64)
        barrier.wait()
        t0 = time.perf_counter()
        b, ms = ops.Belief.identity_prior(), opipe.MapState.empty(B)
        for _ in range(2):
            r = opipe.process_scan_bin_path(b, sc, Q, pc, bins, knn, ms)
            b, ms = r["belief"], r["map"]
        return 2, time.perf_counter() - t0


def cpu_baseline(cfg):
    """The numpy oracle (`port`: the reference restatement; the JAX reference itself cannot run
    here) on bounded samples of the same workload, on this host's cores."""
    import multiprocessing as mp
    N, B = cfg["N"], cfg["B"]
    allowed = process_cpus()  # the job's CPUs, not the rank's NUMA-local share
    prev = set(allowed)
    n1, t1 = _oracle_scans(N, B, "scale", 12, 8.0, core=allowed[0])
    os.sched_setaffinity(0, prev)
    out = dict(value=n1 / t1, unit="scans/s", cores=1, kind="port",
               sample=f"{n1} full 14-step scans (numpy oracle, scale mode) at N={N}, B={B}, K={cfg['K']} on 1 "
                      f"pinned host core (threadpoolctl limit 1), {t1:.1f} s",
               cpu_model=_cpu_model(), cpu_count=os.cpu_count(), cpus_allowed=len(allowed))
    # multi-core: one independent hypothesis stream per core (processes pinned one per core), on the
    # box's CPU share per GPU (16: os.cpu_count() reports the whole host's CPUs there)
    P = min(len(allowed), int(os.environ.get("GCS_BASELINE_PROCS", "16")))
    try:
        ctx = mp.get_context("spawn")
        mgr = ctx.Manager()
        barrier = mgr.Barrier(P)
        with ctx.Pool(P) as pool:
            t0 = time.perf_counter()
            res = pool.map(_pool_worker, [(allowed[i], N, B, barrier) for i in range(P)])
            wall = time.perf_counter() - t0
        nsc = sum(r[0] for r in res)
        tmax = max(r[1] for r in res)
        out["multi_core"] = dict(value=nsc / tmax, unit="scans/s", cores=P,
                                 sample=f"{P} processes x 2 scans (one hypothesis stream per pinned core, {P} of the "
                                        f"{len(allowed)} CPUs this process may use: the GPU box's per-GPU CPU "
                                        f"share), timed from a common barrier; {wall:.1f} s wall incl. setup")
        mgr.shutdown()
    except Exception as e:  # the baseline is reported, never the thing measured
        out["multi_core"] = dict(value=None, error=repr(e)[:200])
    n3, t3 = _oracle_scans(8192, 48, "dense", 40, 3.0, core=allowed[0])
    os.sched_setaffinity(0, prev)
    out["c1_equivalent"] = dict(value=n3 / t3, unit="scans/s", cores=1,
                                sample=f"{n3} scans at N=8192 (N_POINTS_CAP), B=48 dense (the reference's own "
                                       f"budget, SURVEY 8 C1) on 1 core, {t3:.1f} s")
    return out


# ---------------------------------------------------------------- GPU runs
def make_ctx(cfg, device):
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    return HypothesisContext(n_bins=cfg["B"], n_points_cap=cfg["N"], max_raw_points=cfg["N"], mode="scale",
                             k_cand=cfg["K"], lidar_origin=tuple(synthetic.LIDAR_ORIGIN), device=device)


def resident_scans(N, device, n=N_SCANS):
    import torch
    from gcslam import synthetic
    scans = []
    for k in range(n):
        sc = synthetic.make_scan(N, k)
        scans.append((sc, torch.from_numpy(sc["xyz_record"]).to(device), torch.from_numpy(sc["timestamps"]).to(device),
                      torch.from_numpy(sc["weights"]).to(device)))
    torch.cuda.synchronize()
    return scans


def h2d_ms(scans, device, reps=20):
    """One raw scan (f32 xyz record + f64 t + f64 w) from pinned host memory to HBM."""
    import torch
    sc = scans[0][0]
    host = [torch.from_numpy(np.ascontiguousarray(sc[k])).pin_memory() for k in ("xyz_record", "timestamps", "weights")]
    dev = [torch.empty_like(h, device=device) for h in host]
    s = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for d, h in zip(dev, host):
        d.copy_(h, non_blocking=True)
    e0.record(s)
    for _ in range(reps):
        for d, h in zip(dev, host):
            d.copy_(h, non_blocking=True)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, sum(h.numel() * h.element_size() for h in host)


def pmc_traffic(config):
    """HBM bytes per launch of k_bins_scale from the committed rocprofv3 --pmc passes
    (profiles/pmc_bins_<cfg>.json, tools/pmc_summary.py; FETCH/WRITE_SIZE need their own runs)."""
    path = os.path.join(ROOT, "profiles", f"pmc_bins_{config}.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    return d.get("hbm_bytes_per_launch"), f"profiles/pmc_bins_{config}.json ({d.get('round', 'r01')})"


def c3_roofline(device, steps=16, warmup=3):
    """The roofline kernel at the north-star target config (BASELINE.json configs[2]) in this run."""
    from gcslam.synthetic import scan_kwargs
    cfg = CONFIGS["c3"]
    ctx = make_ctx(cfg, device)
    scans = resident_scans(cfg["N"], f"cuda:{device}", n=2)
    for k in range(warmup):
        sc, rec, t, w = scans[k % 2]
        ctx.scan(rec, 16, t, w, cfg["N"], **scan_kwargs(sc))
    ctx.synchronize()
    ctx.enable_timing(True, stages=["budget", "points", "bins", "bins_fold"])
    ctx.stage_times(reset=True)
    # each scan followed by the hypothesis combine (host form: one rank here) and a device sync: the
    # chain's kernels are timed alone, not under the previous scan's pushforward (at C3 a 55 us kernel on
    # the push stream that the step's 20 us of host work does not cover: k_points 41 us alone, ~52 us
    # under it -- a pipelining cost of the step, which ms_per_step at --config c3 carries)
    combine = ctx.combine_call(None, 1.0, 1.0)
    t0 = time.perf_counter()
    for k in range(steps):
        sc, rec, t, w = scans[k % 2]
        ctx.scan(rec, 16, t, w, cfg["N"], **scan_kwargs(sc))
        combine(k)
        ctx.synchronize()
    el = time.perf_counter() - t0
    ms_sum, cnt = ctx.stage_times(reset=True)
    ctx.close()
    avg = {name: (float(ms_sum[i] / cnt[i]) if cnt[i] else None) for i, name in enumerate(ctx.STAGES)}
    r = roofline(cfg["N"], cfg["B"], avg["bins"], *pmc_traffic("c3"))
    label = "c3: 262144-pt scans vs 1048576-bin map, K=16"
    if r:
        r.update(config=label, timed_launches=int(cnt[2]), scans_per_s_with_chain_stamps=steps / el)
    return r, roofline_chain(cfg["N"], cfg["B"], avg, label, config="c3")


def pin_main_and_worker(ctx, share):
    """The main thread on the share's last core, the context's launch worker on the rest of it (disjoint):
    the worker spins 2 ms after each job, and a worker woken onto the main thread's core (wake-affine
    placement) time-slices with it for up to a scheduler slice -- the multi-millisecond calls of the
    round-5 driver line.  Returns the placement for the line, or {} when the share
    is too small (fewer than 4 CPUs) or the kernel refuses."""
    if os.environ.get("GCSLAM_BENCH_PIN_MAIN", "1") == "0" or len(share) < 4:
        return {}
    main = share[-1]
    # the worker stays off the main thread's physical core too (its SMT siblings share the core's pipes)
    sib = {main}
    try:
        from gcslam.topology import parse_cpulist
        with open(f"/sys/devices/system/cpu/cpu{main}/topology/thread_siblings_list") as f:
            sib |= set(parse_cpulist(f.read()))
    except (OSError, ValueError, ImportError):
        pass
    rest = [c for c in share if c not in sib] or share[:-1]
    try:
        os.sched_setaffinity(threading.get_native_id(), {main})
        out = dict(main_thread_cpu=main, main_core_siblings=sorted(sib - {main}))
        wt = ctx.worker_tid()
        if wt:
            os.sched_setaffinity(wt, set(rest))
            out["worker_cpus"] = f"{len(rest)} of the share, not the main thread's core"
        return out
    except OSError:
        return {}


def live_path_bench(device, steps=30, warmup=10):
    """The live primitive path -- the LiDAR evidence the reference runs today (surfels, recency + atlas
    view, OT association, visual pose evidence, fusion, step 12b; pipeline.py:778-926, 980-1011,
    1232-1492) -- through the drop-in process_scan_single_hypothesis(..., primitive_map=) at the
    reference's sizes (PipelineConfig defaults = constants.py: N_POINTS_CAP 8,192, m_tile 50,000, 7
    active / stencil tiles, M_TILE_VIEW 1,024, n_surfel 1,024 + n_feat 512, k_assoc 8, 50 Sinkhorn
    iterations), one hypothesis over consecutive synthetic scans along the trajectory (the map fills as
    it would).  The call takes the reference's numpy inputs (its H2D included).  ms per call over the
    timed scans (the one-call path, gcs_live_scan), the same count of following scans through the
    per-operator path (GCSLAM_LIVE_CHAIN=0) beside it, then a diagnostic pass with config.enable_timing
    for the stage split."""
    import torch
    from gcslam import synthetic, primitive_map as gpm
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, datasheet_process_noise_state,
                                 process_noise_state_to_Q, process_scan_single_hypothesis)
    N = 8192
    cfg = PipelineConfig(K_HYP=1, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense",
                         lidar_origin_base=tuple(synthetic.LIDAR_ORIGIN), max_raw_points=N, device=device)
    ctx = cfg.make_context()
    # the reference's AtlasMap is a dict of tiles; this one preallocates: 512 tiles x 50,000 slots hold
    # the synthetic trajectory's coverage over the run (its z hovers at a tile boundary, so the one-slab
    # stencil alternates between two layers of tiles)
    am = gpm.create_empty_atlas_map(m_tile=cfg.primitive_map_max_size, max_tiles=512, device=device)
    Q = process_noise_state_to_Q(datasheet_process_noise_state())
    n_total = warmup + 2 * steps + 10
    scans = [synthetic.make_scan(N, k) for k in range(n_total)]
    state = dict(belief=BeliefGaussianInfo.create_identity_prior(), seq=0)

    def one(sc):
        r = process_scan_single_hypothesis(
            belief_prev=state["belief"], raw_points=sc["points"], raw_timestamps=sc["timestamps"],
            raw_weights=sc["weights"], raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8),
            imu_stamps=sc["imu_stamps"], imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
            odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"], scan_end_time=sc["scan_end_time"],
            dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"], t_scan=sc["t_scan"], Q=Q, config=cfg,
            odom_twist=sc["odom_twist"], odom_twist_cov=sc["odom_twist_cov"], camera_batch=None,
            scan_seq=state["seq"], primitive_map=am, map_bins=ctx)
        state["belief"] = r.belief_updated
        state["seq"] += 1
        return r

    share = sorted(os.sched_getaffinity(0))
    placement = {}
    for k in range(warmup):
        one(scans[k])
        if k == 0:  # the first call started the context's worker (step 12b's launches)
            placement = pin_main_and_worker(ctx, share)
    torch.cuda.synchronize()
    # The start-up heap (torch, numpy, the earlier passes) into the collector's permanent generation: a
    # full collection in the timed calls then scans only this loop's objects.  The serving loop of the
    # drop-in does the same after start-up.  Every collection that still runs during a
    # timed call is clocked (gc.callbacks) and charged to that call.
    import gc
    import resource
    from gcslam import pipeline as GP
    gc.collect()
    gc.freeze()
    gc_ev = []

    def _gc_cb(phase, info):
        if phase == "start":
            gc_ev.append([time.perf_counter(), None, info.get("generation", -1)])
        elif gc_ev and gc_ev[-1][1] is None:
            gc_ev[-1][1] = time.perf_counter()
    gc.callbacks.append(_gc_cb)
    stamps_prev = GP._STAMPS_ON
    GP._STAMPS_ON = True  # the drop-in's phase stamps (GCSLAM_LIVE_STAMPS): a list append per phase
    ru0 = resource.getrusage(resource.RUSAGE_THREAD)
    per = np.zeros(steps)
    cpu = np.zeros(steps)
    bounds = []
    phases = []
    for i in range(steps):
        GP.LIVE_STAMPS.clear()
        c0 = time.thread_time()
        t0 = time.perf_counter()
        r = one(scans[warmup + i])
        t1 = time.perf_counter()
        per[i] = t1 - t0
        cpu[i] = time.thread_time() - c0
        bounds.append((t0, t1))
        st = [(n, t) for n, t in GP.LIVE_STAMPS]
        phases.append({st[k][0]: (st[k][1] - (st[k - 1][1] if k else t0)) * 1e3 for k in range(len(st))})
    ru1 = resource.getrusage(resource.RUSAGE_THREAD)
    GP._STAMPS_ON = stamps_prev
    gc.callbacks.remove(_gc_cb)
    gc_ms = np.zeros(steps)
    for ta, tb, _ in gc_ev:
        if tb is None:
            continue
        for i, (t0, t1) in enumerate(bounds):
            if t0 <= ta < t1:
                gc_ms[i] += (tb - ta) * 1e3
    med = float(np.median(per))
    slow = np.nonzero(per > 2.0 * med)[0]
    names = list(phases[0].keys()) if phases else []
    pct = lambda a, q: float(np.percentile(a, q))  # noqa: E731
    attribution = dict(
        phase_ms={n: dict(p50=pct([p.get(n, 0.0) for p in phases], 50), p90=pct([p.get(n, 0.0) for p in phases], 90),
                          max=float(max(p.get(n, 0.0) for p in phases))) for n in names},
        phase_note="drop-in phase clocks per call: h2d (host arrays staged), args (the C call's arguments), "
                   "live_scan (the one C call: begin, surfels .. pose evidence, finish, step 12b queued), "
                   "live_results (result objects, step 12b running), result, collect (step 12b's wait)",
        calls_over_2x_median=int(len(slow)), slow_calls=[dict(call=int(i), ms=float(per[i] * 1e3),
                                                            gc_ms=float(gc_ms[i]),
                                                            offcpu_ms=float((per[i] - cpu[i]) * 1e3),
                                                            phases=phases[i]) for i in slow[:5]],
        gc=dict(collections=len(gc_ev), ms_total=float(gc_ms.sum()), ms_max=float(gc_ms.max()) if steps else 0.0,
                frozen_objects=gc.get_freeze_count()),
        offcpu_ms=dict(p50=pct((per - cpu) * 1e3, 50), p90=pct((per - cpu) * 1e3, 90),
                       max=float(((per - cpu) * 1e3).max())),
        offcpu_note="wall - this thread's CPU time per call: waiting that is not a spin (sleeps, descheduling)",
        ctx_switches=dict(voluntary=int(ru1.ru_nvcsw - ru0.ru_nvcsw), involuntary=int(ru1.ru_nivcsw - ru0.ru_nivcsw)))
    chain_on = r.stage_ms == {} and os.environ.get("GCSLAM_LIVE_CHAIN", "1") != "0"
    prev = os.environ.get("GCSLAM_LIVE_CHAIN")
    os.environ["GCSLAM_LIVE_CHAIN"] = "0"
    per_op = np.zeros(steps)
    try:
        for i in range(3):  # its own warm-up: the per-operator calls' first-use allocations
            one(scans[warmup + steps + i])
        for i in range(steps):
            t0 = time.perf_counter()
            one(scans[warmup + steps + i])
            per_op[i] = time.perf_counter() - t0
    finally:
        if prev is None:
            os.environ.pop("GCSLAM_LIVE_CHAIN")
        else:
            os.environ["GCSLAM_LIVE_CHAIN"] = prev
    # diagnostic pass: every stage synced and timed (config.enable_timing, the reference's _record_timing)
    cfg.enable_timing = True
    split = []
    for k in range(warmup + 2 * steps, n_total):
        split.append(one(scans[k]).stage_ms)
    cfg.enable_timing = False
    mu = r.map_update_cert
    out = dict(ms_per_call=float(per.mean() * 1e3), ms_median=float(np.median(per) * 1e3),
               ms_p90=float(np.percentile(per, 90) * 1e3), ms_max=float(per.max() * 1e3), calls=int(steps),
               attribution=attribution, placement=placement or "share (not pinned)",
               path="gcs_live_scan (one C call per scan)" if chain_on else "per-operator C calls",
               per_operator_ms_per_call=float(per_op.mean() * 1e3),
               per_operator_ms_median=float(np.median(per_op) * 1e3),
               per_operator_ms_max=float(per_op.max() * 1e3),
               stage_ms={k: float(np.mean([s[k] for s in split])) for k in split[0]},
               stage_note="diagnostic pass: a device sync before each stage clock (the reference's enable_timing)",
               sizes=dict(n_points_cap=N, m_tile=cfg.primitive_map_max_size, n_active_tiles=cfg.N_ACTIVE_TILES,
                          n_stencil_tiles=cfg.N_STENCIL_TILES, m_tile_view=cfg.M_TILE_VIEW, n_surfel=cfg.n_surfel,
                          n_feat=cfg.n_feat, k_assoc=cfg.k_assoc, k_sinkhorn=cfg.k_sinkhorn),
               map_primitives=int(am.total_count), last_scan_inserted=int(mu.insert_count_total),
               last_scan_fused=int(mu.fused_count), n_valid_measurements=int(r.measurement_batch.n_valid))
    gc.unfreeze()  # (frozen for the per-operator pass too)
    am.close()
    ctx.close()
    os.sched_setaffinity(threading.get_native_id(), set(share))
    return out


def primitive_path_main(args, rank, world, local_rank, pin):
    """`--path primitive`: the live primitive path (live_path_bench's sizes) as the multi-hypothesis node
    runs it, one hypothesis per rank: each step every rank runs process_scan_single_hypothesis on the same
    synthetic scan and the ranks exchange the combine payload.  --map-mode shared keeps the reference's
    one map, hypothesis 0's (backend_node.py:2036-2083): rank 0 updates the node map and broadcasts the
    update record (gcslam.distributed.MapRecordChannel: RCCL, or gloo with --share-device); the other
    ranks scan with update_map=False and replay the lead's record on their copy of the node map
    (primitive_map_follow) -- with the bin path's declared one-scan lag (a follower's scan s reads the
    map after the lead's scan s - 1, so the ranks run concurrently).  At the end every follower replays
    the last record and the ranks compare map hashes: `map_bitwise_equal`.  --share-device puts every
    rank on device 0 with a gloo transport (a rehearsal on one GPU; RCCL needs one GPU per rank)."""
    import hashlib
    import torch
    import torch.distributed as dist
    from gcslam import synthetic, primitive_map as gpm
    from gcslam.distributed import HypothesisComm, MapRecordChannel, hypothesis_weights
    from gcslam.pipeline import (BeliefGaussianInfo, PipelineConfig, datasheet_process_noise_state,
                                 primitive_map_follow, process_noise_state_to_Q, process_scan_single_hypothesis)
    dev = 0 if args.share_device else local_rank
    torch.cuda.set_device(dev)
    if world > 1:
        # gloo in both cases: the RCCL communicator is the library's (HypothesisComm), not torch's
        dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = HypothesisComm(rank, world, dev) if (world > 1 and not args.share_device) else None
    N = 8192
    cfg = PipelineConfig(K_HYP=world, N_POINTS_CAP=N, B_BINS=48, soft_assign_mode="dense",
                         lidar_origin_base=tuple(synthetic.LIDAR_ORIGIN), max_raw_points=N, device=dev)
    ctx = cfg.make_context()
    am = gpm.create_empty_atlas_map(m_tile=cfg.primitive_map_max_size, max_tiles=256, device=dev)
    shared = args.map_mode == "shared"
    lead = rank == 0
    from gcslam.surfels import GC_VMF_N_LOBES
    chan = (MapRecordChannel(cfg.n_feat + cfg.n_surfel, GC_VMF_N_LOBES, cfg.k_assoc, dev, comm)
            if (shared and world > 1) else None)
    Q = process_noise_state_to_Q(datasheet_process_noise_state())
    rng = np.random.default_rng(1000 + rank)
    belief = BeliefGaussianInfo.create_identity_prior()
    if rank > 0:  # hypothesis priors perturbed by N(0, (0.05 m, 0.5 deg))
        belief.X_anchor = np.concatenate([rng.normal(0, 0.05, 3), rng.normal(0, np.deg2rad(0.5), 3)])
    w_iw, w_bary = (float(x[rank]) for x in hypothesis_weights(world))
    combine = ctx.combine_call(comm.h if comm is not None else None, w_iw, w_bary)
    n_total = args.warmup + args.steps
    scans = [synthetic.make_scan(N, k) for k in range(n_total)]
    st = dict(belief=belief, pending=None)
    comb_ms, follow_ms, bcast_ms = [], [], []

    def step(s):
        if shared and not lead and st["pending"] is not None:  # the lead's update of scan s - 1
            t0 = time.perf_counter()
            primitive_map_follow(am, st["pending"], cfg)
            follow_ms.append((time.perf_counter() - t0) * 1e3)
        sc = scans[s]
        r = process_scan_single_hypothesis(
            belief_prev=st["belief"], raw_points=sc["points"], raw_timestamps=sc["timestamps"],
            raw_weights=sc["weights"], raw_ring=np.zeros(N, np.uint8), raw_tag=np.zeros(N, np.uint8),
            imu_stamps=sc["imu_stamps"], imu_gyro=sc["imu_gyro"], imu_accel=sc["imu_accel"], odom_pose=sc["odom_pose"],
            odom_cov_se3=sc["odom_cov_se3"], scan_start_time=sc["scan_start_time"], scan_end_time=sc["scan_end_time"],
            dt_sec=sc["dt_sec"], t_last_scan=sc["t_last_scan"], t_scan=sc["t_scan"], Q=Q, config=cfg,
            odom_twist=sc["odom_twist"], odom_twist_cov=sc["odom_twist_cov"], camera_batch=None, scan_seq=s,
            primitive_map=am, map_bins=ctx, update_map=(lead or not shared))
        st["belief"] = r.belief_updated
        if chan is not None:
            t0 = time.perf_counter()
            if lead:
                chan.pack(r.map_record)
            chan.broadcast(root=0)
            if not lead:
                st["pending"] = chan.unpack()
            bcast_ms.append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        if comm is not None or world == 1:
            combine(s)
        else:  # gloo transport of the library-packed payload (ranks sharing one device)
            from gcslam.distributed import combine_allreduce
            combine_allreduce(ctx, rank, world, s, want_belief=False)
        comb_ms.append((time.perf_counter() - t0) * 1e3)

    for s in range(args.warmup):
        step(s)
    comb_ms.clear(); follow_ms.clear(); bcast_ms.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, n_total):
        step(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el_rank = time.perf_counter() - t0
    el = el_rank
    if world > 1:  # the slowest rank's clock
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    if shared and not lead and st["pending"] is not None:  # catch up with the lead's last update
        primitive_map_follow(am, st["pending"], cfg)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in sorted(am.tile_ids):
        for k, v in sorted(am.read_tile(int(t)).items()):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v).tobytes())
    med = lambda x: float(np.median(x)) if x else None  # noqa: E731
    me = dict(rank=rank, affinity=pin, ms_per_step=el_rank / args.steps * 1e3, map_sha=h.hexdigest()[:16],
              map_primitives=int(am.total_count), combine_ms=med(comb_ms), follow_ms=med(follow_ms),
              record_bcast_ms=med(bcast_ms))
    per_rank = [me]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, me)
    if rank == 0:
        line = {"metric": "live primitive path: hypothesis-scans/s (process_scan_single_hypothesis, primitive_map=)",
                "value": world * args.steps / el, "unit": "scans/s", "n_gpus": 1 if args.share_device else world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic (seeded VLP-16-like scans along the trajectory; numpy inputs per call)",
                "config": {"workload": f"live path at the reference sizes, {world} hypotheses, map {args.map_mode}",
                           "path": "primitive", "map_mode": args.map_mode, "hypotheses": world,
                           "transport": ("gloo (shared device)" if args.share_device else "rccl") if world > 1 else None},
                "map_bitwise_equal": len({p["map_sha"] for p in per_rank}) == 1 if shared else None,
                "record_bytes": chan.nbytes if chan is not None else None, "per_rank": per_rank}
        print(json.dumps(line), flush=True)
    am.close()
    ctx.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, cpu):
    """`bench.py --gpus N` with no launcher: start N rank processes of this script (the one-process-per-GPU
    layout torch.distributed.run gives) and return their exit status.  Nothing here touches a GPU: the
    visible GPUs are counted from the KFD topology in sysfs (gcslam.topology, the enumeration the HIP
    runtime itself does; no torch.cuda call, which can fall back to hipGetDeviceCount), and each rank
    initialises only its own device."""
    import subprocess
    if not cpu:
        from gcslam import topology
        vis = topology.visible_gpu_count() or 0  # no KFD topology: no AMD GPU driver here
        if n > vis:
            print(f"bench.py: --gpus {n} but only {vis} visible GPU(s)", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GCS_ALLOWED_CPUS=_allowed_str())
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.1)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # one rank failed: the others would block in the next collective
                    q.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def _allowed_str():
    return ",".join(str(c) for c in sorted(os.sched_getaffinity(0)))


def process_cpus():
    """The CPUs this job may use (the launcher's set, passed down before the ranks pin themselves)."""
    s = os.environ.get("GCS_ALLOWED_CPUS")
    return sorted(int(c) for c in s.split(",")) if s else sorted(os.sched_getaffinity(0))


def cpu_rehearsal(args, rank, world, pin):
    """The multi-rank path without GPUs (gloo): each rank packs its hypothesis' payload with the library
    (gcs_payload_pack: IW statistics with the raw weights, barycenter sums with the floor-renormalised
    ones, backend_node.py:1999-2002,2085-2090, hypothesis.py:83-99), the payloads are summed over
    torch.distributed, and every rank applies the sum (gcs_payload_apply: barycenter, both IW applies,
    Q), carrying the IW states to the next step.  The per-rank payloads are all-gathered once to check
    the sum.  A rehearsal of the launcher and the exchange, not a benchmark."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from gcslam import _lib as L
    from gcslam.distributed import allreduce_payload, hypothesis_weights
    lib = L.load()
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    w, wn = hypothesis_weights(world)
    rng = np.random.default_rng(1000 + rank)
    nu, Psi = np.zeros(7), np.zeros(252)
    mnu, mPsi = np.zeros(3), np.zeros(27)
    assert lib.gcs_datasheet_noise_states(nu.ctypes.data, Psi.ctypes.data, mnu.ctypes.data, mPsi.ctypes.data) == 0
    err, payloads, rec_ok = 0.0, None, True
    t0 = time.perf_counter()
    for step in range(args.warmup + args.steps):
        if step == args.warmup:
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
        A = rng.normal(size=(22, 22))
        Lm = A @ A.T + 22.0 * np.eye(22)
        bs = L.belief_to_struct(rng.normal(0, 0.05, 6), float(step), rng.normal(0, 1e-3, 22), Lm, rng.normal(size=22))
        dPsi = np.ascontiguousarray(np.stack([np.outer(v, v) for v in rng.normal(0, 1e-2, (7, 6))]).reshape(252))
        dnu = np.ones(7)
        mdPsi = np.ascontiguousarray(np.stack([np.outer(v, v) for v in rng.normal(0, 1e-3, (3, 3))]).reshape(27))
        mdnu = np.array([1.0, 1.0, 0.0])
        shared = args.map_mode == "shared"
        p = np.zeros(840 + (L.MAP_REC_LEN if shared else 0))
        assert lib.gcs_payload_pack(C.byref(bs), dPsi.ctypes.data, dnu.ctypes.data, mdPsi.ctypes.data,
                                    mdnu.ctypes.data, float(w[rank]), float(wn[rank]), p.ctypes.data) == 0
        if shared:  # the lead's map-update record rides the payload; the followers add zeros
            lead_rec = np.random.default_rng(7 + step).normal(size=L.MAP_REC_LEN)
            if rank == 0:
                p[840:] = lead_rec
        if step == 0:  # every rank's own payload, gathered before the sum (the transport reduces in place)
            if world > 1:
                got = [torch.zeros(p.shape[0], dtype=torch.float64) for _ in range(world)]
                dist.all_gather(got, torch.from_numpy(p.copy()))
                payloads = np.stack([g.numpy() for g in got])
            else:
                payloads = p[None].copy()
        tot = np.ascontiguousarray(allreduce_payload(p))
        if step == 0:
            err = float(np.abs(payloads.sum(0) - tot).max())
        if shared:  # every rank received the lead's record bit for bit
            rec_ok = rec_ok and bool(np.array_equal(tot[840:], lead_rec))
            tot = np.ascontiguousarray(tot[:840])
        comb = L.GcsBelief()
        out = [np.zeros(n) for n in (7, 252, 484, 3, 27, 4)]
        assert lib.gcs_payload_apply(tot.ctypes.data, step, np.zeros(6).ctypes.data, 0.0, nu.ctypes.data,
                                     Psi.ctypes.data, mnu.ctypes.data, mPsi.ctypes.data, C.byref(comb),
                                     *[o.ctypes.data for o in out]) == 0
        nu, Psi, _, mnu, mPsi, _ = out
    el = time.perf_counter() - t0
    ranks = [rank]
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        allr = [None] * world
        dist.all_gather_object(allr, dict(rank=rank, pid=os.getpid(), Q_sum=float(out[2].sum()), map_record_ok=rec_ok,
                                          affinity=pin))
        ranks = allr
    if rank == 0:
        print(json.dumps({
            "metric": "payload exchanges/s (CPU rehearsal of the multi-rank path; not the benchmark)",
            "value": args.steps / el, "unit": "exchanges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "rehearsal": True, "transport": "gloo" if world > 1 else None,
            "ranks": ranks, "payload_sum_max_abs_err": err,
            "payload_sum_check": bool(err <= 1e-12 * max(1.0, float(np.abs(payloads).sum(0).max())))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c3", action="store_true")
    ap.add_argument("--no-live", action="store_true", help="skip the live primitive path's timing (live_path)")
    ap.add_argument("--map-mode", default="own", choices=["own", "shared"],
                    help="own: a map per hypothesis (default); shared: one map, hypothesis 0's (rank 0 leads, "
                         "the other ranks replay its update: gcslam_hip.h GCS_MAP_FOLLOW); at one GPU the rank "
                         "follows itself, which times a follower's scan")
    ap.add_argument("--path", default="bins", choices=["bins", "primitive"],
                    help="bins: the 14-step bin path (the headline metric); primitive: the live primitive path "
                         "through the drop-in, one hypothesis per rank (primitive_path_main)")
    ap.add_argument("--share-device", action="store_true",
                    help="--path primitive: every rank on device 0, gloo transport (a rehearsal on one GPU)")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N = 1 only: combine on the host without a world-1 RCCL communicator (A/B of the collective)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="launcher + payload exchange over gloo on CPU (test of the multi-rank path)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # before any GPU call in this process
        sys.exit(launch_ranks(args.gpus, args.cpu_rehearsal or args.share_device))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # each rank on its GPU's NUMA-local host cores, before any GPU call (threads started later -- the
    # HIP runtime's, the context's launch worker -- inherit the mask); cpu_baseline restores the job's set
    from gcslam import topology
    pin = topology.pin_rank(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    if args.cpu_rehearsal:
        return cpu_rehearsal(args, rank, world, pin)
    if args.path == "primitive":
        return primitive_path_main(args, rank, world, local_rank, pin)

    import torch
    import torch.distributed as dist

    if world > 1:
        # torch.distributed over gloo (host): it broadcasts the RCCL id and carries the bench's barriers and
        # per-rank clocks; the one RCCL communicator is the library's (HypothesisComm), which runs the
        # per-scan all-reduce -- no second (torch NCCL) communicator on the GPUs
        torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = f"cuda:{local_rank}"
    torch.cuda.set_device(local_rank)

    from gcslam import _lib as L
    from gcslam.distributed import HypothesisComm
    from gcslam.synthetic import scan_kwargs

    # the per-scan exchange runs in the library over RCCL (torch.distributed only broadcasts the id); at
    # N = 1 too (a world-1 communicator), so the timed step runs the ncclAllReduce path of the N-GPU run
    comm = HypothesisComm(rank, world, local_rank) if (world > 1 or not args.no_rccl) else None
    rccl = None
    if comm is not None:
        n_comm, r_comm = comm.count()
        allc = [(n_comm, r_comm)]
        if world > 1:
            cnt = torch.tensor([n_comm, r_comm], dtype=torch.int64)
            allc = [torch.zeros_like(cnt) for _ in range(world)]
            dist.all_gather(allc, cnt)
            allc = [(int(c[0]), int(c[1])) for c in allc]
        rccl = dict(comm_count=n_comm, user_ranks=[c[1] for c in allc], counts=[c[0] for c in allc],
                    collective="ncclAllReduce(sum, f64) of the 840-word payload per scan on the context's combine "
                               "stream, inside the timed step")
        if any(c[0] != world for c in allc):
            raise RuntimeError(f"RCCL communicator holds {rccl['counts']} ranks, expected {world}")
    cfg = CONFIGS[args.config]
    N, B, K = cfg["N"], cfg["B"], cfg["K"]
    ctx = make_ctx(cfg, local_rank)
    # hypothesis prior perturbed per rank (N(0, (0.05 m, 0.5 deg)))
    rng = np.random.default_rng(1000 + rank)
    X0 = np.concatenate([rng.normal(0, 0.05, 3) * (rank > 0), rng.normal(0, np.deg2rad(0.5), 3) * (rank > 0)])
    ctx.set_belief(X0, 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
    # each pass over the N_SCANS resident scans restarts from this prior: the scans are one short stretch of
    # a trajectory, so cycling them under a running belief feeds the filter a jump back every N_SCANS
    # scans, and the reference's own restatement diverges on that (the translation doubling per scan from
    # ~100 scans on, oracle and library alike: tools/long_run.py); restarting the
    # belief makes every pass the same closed loop over a map that keeps accumulating the same views
    import ctypes as C
    prior = L.belief_to_struct(X0, 0.0, np.zeros(22), 1e-6 * np.eye(22), np.zeros(22))
    prior_ref, set_belief, ctx_h = C.byref(prior), ctx.lib.gcs_ctx_set_belief, ctx.h
    scans = resident_scans(N, device)
    # each resident scan's gcs_scan_inputs (device pointers + its host IMU / odometry arrays) filled
    # once, as a C caller fills the struct per scan; the step is then one C-ABI call
    prepared = [ctx.prepare_scan(rec, 16, t, w, N, **scan_kwargs(sc)) for sc, rec, t, w in scans]
    from gcslam.distributed import hypothesis_weights
    w_iw, w_bary = (float(x[rank]) for x in hypothesis_weights(world))
    comm_h = comm.h if comm is not None else None

    # gcs_combine_allreduce (RCCL sum of the payload at N > 1, combine, IW updates) and gcs_scan bound once
    combine = ctx.combine_call(comm_h, w_iw, w_bary)
    follow = None
    if args.map_mode == "shared":
        # one map (backend_node.py:2079-2083): rank 0 leads; a follower skips its own map update and
        # replays the lead's from the record the all-reduce carried; a single rank follows itself
        ctx.set_map_mode("lead" if (rank == 0 and world > 1) else "follow")
        if not (rank == 0 and world > 1):
            follow = ctx.map_follow_call()

    scan_out = L.GcsScanOutputs()  # one output record for every scan (the caller-owned buffer form)
    scan_fn = ctx.scan_call(scan_out)
    # the step as one C call (gcs_scan_combine: scan + all-reduce combine, no Python between them);
    # GCSLAM_BENCH_FUSED=0 times the two calls instead (also reported as a variant)
    fused_on = os.environ.get("GCSLAM_BENCH_FUSED", "1") != "0" and follow is None
    fused = ctx.scan_combine_call(scan_out, comm_h, w_iw, w_bary) if fused_on else None
    state = dict(count=0, sample=False, sampled=0, stamp=True, combine=combine, fused=fused, warm_stamp=True,
                 timing_on=False)
    comb_ms = []  # every timed step's combine (pack, all-reduce, IW / Q apply), for SCALE's attribution

    TIMING_STRIDE = timing_stride(args.steps)

    def step():
        try:
            _step()
        except (RuntimeError, ValueError) as e:  # name the failing scan (its index in the bench's sequence)
            raise type(e)(f"{e} [bench scan {state['count']}, scan {state['count'] % N_SCANS} of the cycle]") from e

    def _step():
        combine = state["combine"]
        if state["count"] and state["count"] % N_SCANS == 0:  # a pass over the resident scans restarts
            rc = set_belief(ctx_h, prior_ref)
            if rc:
                ctx._chk(rc, "set_belief")
        # roofline-kernel event stamps on every TIMING_STRIDE-th scan (also in the warm-up, so the timed
        # region's first stamped scan does not pay the events' first use)
        if (state["sample"] or state["warm_stamp"]) and state["stamp"]:
            phase = state["count"] % TIMING_STRIDE
            if phase == 0 and not state["timing_on"]:  # (a call only where the stamping switches)
                ctx.enable_timing(True, stages=["bins"])
                state["timing_on"] = True
            elif phase == 1 and state["timing_on"]:
                ctx.enable_timing(False)
                state["timing_on"] = False
        if state["fused"] is not None:
            dc = state["fused"](prepared[state["count"] % N_SCANS], state["count"])
        else:
            scan_fn(prepared[state["count"] % N_SCANS])
            tc = time.perf_counter()
            combine(state["count"])
            dc = (time.perf_counter() - tc) * 1e3
        out = scan_out
        if state["sample"]:
            comb_ms.append(dc)
        if follow is not None:
            follow(prepared[state["count"] % N_SCANS])
        state["count"] += 1

    share = sorted(os.sched_getaffinity(0))
    for wi in range(args.warmup):
        step()
        # after the warm-up's first scan (which starts the launch worker; it keeps the whole share) the
        # main thread runs on one core of the rank's share -- the last one, away from the low CPUs that
        # take interrupts: the scan's serial host numerics stop migrating between cores, and the rest of
        # the warm-up warms that core (GCSLAM_BENCH_PIN_MAIN=0: the share for every thread, for A/B)
        # (pin_main_and_worker: the launch worker keeps the rest of the share, never the main thread's core)
        if wi == 0:
            pin = dict(pin, **pin_main_and_worker(ctx, share))
    state["warm_stamp"] = False
    state["sample"] = True
    ctx.synchronize()
    ctx.enable_timing(False)
    state["timing_on"] = False
    ctx.stage_times(reset=True)
    ctx.host_split(reset=True)  # the library sums every timed scan's host split (gcs_ctx_host_split)
    per_step = np.zeros(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_THREAD)  # the main thread's context switches over the region
    t0 = time.perf_counter()
    for i in range(args.steps):
        ts = time.perf_counter()
        step()
        per_step[i] = time.perf_counter() - ts
    ru1 = resource.getrusage(resource.RUSAGE_THREAD)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_rank = elapsed
    per_rank_s = [elapsed]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        allt = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(allt, tt)
        per_rank_s = [float(x.item()) for x in allt]
        elapsed = max(per_rank_s)  # the slowest rank's clock
    state["sample"] = False
    hist = ctx.host_split_history(args.steps)  # (before the reset) every timed scan's own split
    hsum, (n_scans_h, n_calls_h) = ctx.host_split(reset=True)
    ms_sum, counts = ctx.stage_times(reset=True)
    bins_in_region = int(counts[2])
    ctx.enable_timing(False)

    def side_loop(name):  # the same steps again, a variant of the step (not `value`)
        # its own warm-up after the switch (round 5's single 20-step mean met one stall: 0.241 vs 0.10 ms),
        # then the mean and the median of the per-step times
        for _ in range(max(5, args.warmup)):
            step()
        ctx.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        per = np.zeros(args.steps)
        ta = time.perf_counter()
        for i in range(args.steps):
            ts = time.perf_counter()
            step()
            per[i] = time.perf_counter() - ts
        ctx.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        variants[name + "_ms_per_step"] = (time.perf_counter() - ta) / args.steps * 1e3
        variants[name + "_median_ms"] = float(np.median(per) * 1e3)
    # the decomposition of ms_per_step: without the roofline stamps, and (N = 1) with the host-only
    # combine instead of the world-1 RCCL all-reduce -- what round 4's line measured
    state["stamp"] = False
    variants = {}
    side_loop("unstamped")
    if fused is not None:  # the same step as two C calls (gcs_scan, then gcs_combine_allreduce)
        state["fused"] = None
        side_loop("two_call_unstamped")
    if world == 1 and comm is not None:
        state["combine"] = ctx.combine_call(None, w_iw, w_bary)
        if fused is not None:
            state["fused"] = ctx.scan_combine_call(scan_out, None, w_iw, w_bary)
        side_loop("host_combine_unstamped")
        state["combine"] = combine
    state["fused"] = fused
    # the step with the IMU / odometry branch on the device (k_imu_odom on its own stream
    # beside the bin path's kernels) instead of the host C++ branch, same box, its own warm-up
    try:
        if os.environ.get("GCSLAM_BENCH_NO_DEVIO") == "1":
            raise RuntimeError("skipped (GCSLAM_BENCH_NO_DEVIO=1)")
        ctx.set_debug(L.DEBUG_DEVICE_IMU_ODOM, 1)
    except (RuntimeError, ValueError) as e:  # an older library in a same-box A/B
        variants["device_imu_odom_unstamped_error"] = str(e)[:200]
    else:
        try:
            side_loop("device_imu_odom_unstamped")
        finally:
            ctx.set_debug(L.DEBUG_DEVICE_IMU_ODOM, 0)
    state["stamp"] = True
    if "main_thread_cpu" in pin:  # the share again (the C3 pass, the live path, the CPU baseline's processes)
        os.sched_setaffinity(threading.get_native_id(), set(share))
    # the roofline kernel's duration: the timed region's stamped launches (every TIMING_STRIDE-th scan)
    # plus, when those are fewer than ROOFLINE_MIN (short runs), a pass stamping it on every scan
    if bins_in_region < ROOFLINE_MIN:
        ctx.enable_timing(True, stages=["bins"])
        for _ in range(ROOFLINE_MIN - bins_in_region):
            step()
        ctx.synchronize()
        ctx.enable_timing(False)
        ms2, c2 = ctx.stage_times(reset=True)
        ms_sum, counts = ms_sum + ms2, counts + c2
    bins_ms = float(ms_sum[2] / counts[2]) if counts[2] else None
    bins_samples = int(counts[2])
    # every timed step's host split, summed by the library (not a sample): its parts add up to the
    # C call, and python_other is the rest of ms_per_step (the Python loop around the call)
    host_avg = {k: v / max(n_scans_h, 1) for k, v in hsum.items() if k not in ("combine", "scan_combine_call")}
    host_avg["combine"] = (hsum["combine"] / n_calls_h) if n_calls_h else float(np.mean(comb_ms)) if comb_ms else 0.0
    if n_calls_h:
        host_avg["scan_combine_call"] = hsum["scan_combine_call"] / n_calls_h
    call_ms = host_avg.get("scan_combine_call", host_avg["gcs_scan"] + host_avg["combine"])
    host_avg["python_other"] = elapsed_rank / args.steps * 1e3 - call_ms
    host_avg["scans_counted"] = n_scans_h
    host_avg["note"] = ("every timed step (gcs_ctx_host_split sums in the library): pre_device + device_wait + tail "
                        "= gcs_scan; gcs_scan + combine = the C call; + python_other = ms_per_step of this rank")
    if hist is not None and len(hist):
        # the per-step distribution of the same split (the library's per-scan record), and the steps
        # over twice the median step with their own split: a host stall names its phase
        q = lambda a, p: float(np.percentile(a, p))  # noqa: E731
        host_avg["per_step"] = {n: dict(p50=q(hist[:, k], 50), p90=q(hist[:, k], 90), max=float(hist[:, k].max()))
                                for k, n in enumerate(ctx.HOST_HIST) if hist[:, k].any()}
        med_step = float(np.median(per_step))
        slow = np.nonzero(per_step > 2.0 * med_step)[0]
        host_avg["steps_over_2x_median"] = int(len(slow))
        host_avg["ctx_switches"] = dict(voluntary=int(ru1.ru_nvcsw - ru0.ru_nvcsw),
                                        involuntary=int(ru1.ru_nivcsw - ru0.ru_nivcsw),
                                        note="main thread, over the timed region: a preempted step shows as "
                                             "an involuntary switch, a device-side delay as device_wait alone")
        if len(hist) == len(per_step):
            host_avg["slow_steps"] = [dict(step=int(i), ms=float(per_step[i] * 1e3),
                                           split={n: float(hist[i, k]) for k, n in enumerate(ctx.HOST_HIST)})
                                      for i in slow[:5]]
    cm = np.array(comb_ms) if comb_ms else np.zeros(1)
    me = dict(rank=rank, affinity=pin, host_ms=host_avg, ms_per_step=elapsed_rank / args.steps * 1e3,
              combine_ms=dict(median=float(np.median(cm)), p90=float(np.percentile(cm, 90)), mean=float(cm.mean()),
                              max=float(cm.max()), n=int(len(comb_ms))))
    per_rank = [me]
    if world > 1:  # every rank's host split and combine latency, so SCALE can attribute a loss
        per_rank = [None] * world
        dist.all_gather_object(per_rank, me)
    # diagnostic pass after the timed region: every device stage stamped (not part of `value`)
    ctx.enable_timing(True)
    for _ in range(min(args.steps, 20)):
        step()
    ctx.synchronize()
    ms_sum, counts = ctx.stage_times(reset=True)
    stage_avg = {name: (float(ms_sum[i] / counts[i]) if counts[i] else None) for i, name in enumerate(ctx.STAGES)}
    ctx.enable_timing(False)
    manifest = ctx.describe()
    ms_ = ctx.mirror_stats()
    mirror = dict(scan_mirrors=ms_[0], scan_rereads=ms_[1], scan_sync_fallbacks=ms_[2], allreduces=ms_[3],
                  allreduce_rereads=ms_[4], allreduce_sync_fallbacks=ms_[5],
                  note="host hand-offs accepted by sequence word + checksum (gcs_layout.h Mirror); a re-read is a "
                       "buffer whose data reached host memory after its sequence word")
    ctx.close()

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        h2d, h2d_bytes = h2d_ms(scans, device)
        host_avg["h2d"] = h2d
        line = {
            "metric": METRIC if args.config == "c2" else "scans/sec (14-step pipeline) at 256k pts/scan",
            "value": world * args.steps / elapsed, "unit": "scans/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded VLP-16-like scans, box room, IMU 200 Hz, odometry; inputs resident in HBM)",
            "config": {"workload": f"{args.config}: {N}-pt scans vs {B}-bin map, K={K} candidates, "
                                   f"1 hypothesis per GPU ({world} hypotheses), payload all-reduce per scan"
                                   + ("; one shared map (hypothesis 0's; followers replay its update)"
                                      if args.map_mode == "shared" else ""),
                       "map_mode": args.map_mode,
                       "n_points": N, "n_bins": B, "k_cand": K, "hypotheses": world, "parallelism": f"hyp{world}"},
            "value_definition": "hypothesis-scans/s of the whole job: every GPU runs its own hypothesis of each scan "
                                "(weak scaling); the node's scans/s is scans_per_s_node = value / n_gpus",
            "scans_per_s_node": args.steps / elapsed,
            # the per-GPU rate SCALE compares across N (value / n_gpus; at N = 1 it equals value)
            "value_per_gpu": args.steps / elapsed,
            "per_rank_ms_per_step": [t / args.steps * 1e3 for t in per_rank_s],
            # per rank: host pinning, sampled host split (host_ms keys), every timed step's combine latency
            "per_rank": per_rank,
            "rccl": rccl,
            "mirror": mirror,
            "step_variants": dict(variants, step_call="gcs_scan_combine (one C call)" if fused is not None
                                  else "gcs_scan + gcs_combine_allreduce",
                                  note="the same step count again after the timed region, not `value`, each "
                                  "after its own warm-up (mean and median): without the roofline kernel's event "
                                  "stamps, as two C calls (scan, then combine), (N = 1) with the host-only combine "
                                  "in place of the world-1 ncclAllReduce, and with the IMU / odometry branch on the "
                                  "device (k_imu_odom) instead of the host"),
            "step_ms": {"median": float(np.median(per_step) * 1e3), "p90": float(np.percentile(per_step, 90) * 1e3),
                        "min": float(per_step.min() * 1e3), "max": float(per_step.max() * 1e3)},
            "roofline": dict(roofline(N, B, bins_ms, *pmc_traffic(args.config)) or {}, timed_launches=bins_samples,
                             timed_launches_in_region=bins_in_region, stamp_stride=TIMING_STRIDE),
            "roofline_chain": roofline_chain(N, B, stage_avg, f"{args.config} (diagnostic pass, every stage stamped)",
                                             config=args.config),
            "stage_ms": stage_avg,
            "host_ms": host_avg,
            "pcie_inclusive": {"h2d_bytes_per_scan": h2d_bytes, "scans_per_s": 1e3 / (ms_step / world + h2d) * world,
                               "note": "not `value`: a caller holding the raw scan in pinned host memory adds one H2D"},
            "manifest": manifest,
        }
        if world == 1 and args.config == "c2" and not args.no_c3:
            line["roofline_c3"], line["roofline_chain_c3"] = c3_roofline(local_rank)
        if world == 1 and not args.no_live:
            line["live_path"] = live_path_bench(local_rank)
        line["cpu_baseline"] = cpu_baseline(cfg) if (world == 1 and not args.no_cpu_baseline) else None
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
