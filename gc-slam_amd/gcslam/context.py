"""One hypothesis on one GPU: owns the device map-bin statistics, the atlas lookup structures and
the host belief / IW state (wraps gcs_ctx, include/gcslam_hip.h).

Device memory for scans is plain torch CUDA tensors (HIP on ROCm); the context runs on torch's
current stream so ordering with torch producers is implicit.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _addr(a):
    """Address of a C-contiguous f64 array: through the buffer protocol (about half the cost of
    ndarray.ctypes.data per call), ndarray.ctypes for read-only or empty arrays."""
    try:
        return C.addressof(C.c_char.from_buffer(a))
    except (TypeError, ValueError):
        return a.ctypes.data


def _torch():
    import torch
    return torch


def tau_for_bins(n_bins: int, tau_48: float = 0.1) -> float:
    """DECLARED soft-assign temperature: tau_B = tau_48 * 48 / B (DESIGN.md "temperature")."""
    return tau_48 * 48.0 / float(n_bins)


class HypothesisContext:
    def __init__(self, n_bins=48, n_points_cap=8192, max_raw_points=None, mode="dense", k_cand=16, tau=None,
                 lidar_origin=(0.0, 0.0, 0.0), deskew_rotation_only=False, forgetting_factor=0.99,
                 gravity_W=(0.0, 0.0, -9.81), device=0, use_torch_stream=True, use_imu_odom=True,
                 imu_gravity_scale=1.0, planar_z_ref=0.0, planar_z_sigma=0.1, planar_vz_sigma=0.01, alpha_min=1.0,
                 alpha_max=1.0, c0_cond=1e6):
        self.lib = L.load()
        cfg = L.GcsConfig()
        L.check(self.lib.gcs_config_defaults(C.byref(cfg)), None, "gcs_config_defaults")
        cfg.device = int(device)
        cfg.n_bins = int(n_bins)
        cfg.n_points_cap = int(n_points_cap)
        cfg.max_raw_points = int(max_raw_points if max_raw_points is not None else max(n_points_cap, 1) * 8)
        cfg.mode = L.MODE_SCALE if mode == "scale" else L.MODE_DENSE
        cfg.k_cand = int(k_cand)
        cfg.tau = float(tau if tau is not None else tau_for_bins(n_bins))
        cfg.lidar_origin[:] = [float(x) for x in lidar_origin]
        cfg.deskew_rotation_only = int(bool(deskew_rotation_only))
        cfg.forgetting_factor = float(forgetting_factor)
        cfg.gravity_W[:] = [float(x) for x in gravity_W]
        cfg.use_imu_odom = int(bool(use_imu_odom))
        cfg.imu_gravity_scale = float(imu_gravity_scale)
        cfg.planar_z_ref = float(planar_z_ref)
        cfg.planar_z_sigma = float(planar_z_sigma)
        cfg.planar_vz_sigma = float(planar_vz_sigma)
        cfg.alpha_min = float(alpha_min)
        cfg.alpha_max = float(alpha_max)
        cfg.c0_cond = float(c0_cond)
        self.cfg = cfg
        self.mode = mode
        self.device = int(device)
        h = C.c_void_p()
        rc = self.lib.gcs_ctx_create(C.byref(cfg), C.byref(h))
        L.check(rc, None, "gcs_ctx_create")
        self.h = h
        self.stream_ptr = None  # the torch stream the context runs on (None: its own)
        if use_torch_stream:
            torch = _torch()
            with torch.cuda.device(self.device):
                s = torch.cuda.current_stream().cuda_stream
            L.check(self.lib.gcs_ctx_set_stream(self.h, C.c_void_p(s)), self.h, "set_stream")
            self.stream_ptr = int(s)

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "h", None):
            self.lib.gcs_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_bins(self):
        return self.cfg.n_bins

    @property
    def cap(self):
        return self.cfg.n_points_cap

    def _chk(self, rc, what):
        L.check(rc, self.h, what)

    # ------------------------------------------------------------------ state
    def atlas(self):
        B = self.n_bins
        dirs = np.zeros((B, 3))
        knn = np.zeros((B, max(1, self.cfg.k_cand)), np.int32)
        self._chk(self.lib.gcs_ctx_get_atlas(self.h, L.dptr(dirs), L.iptr(knn)), "get_atlas")
        return dirs, (knn if self.mode == "scale" else None)

    def set_atlas(self, dirs):
        d = np.ascontiguousarray(dirs, np.float64)
        self._chk(self.lib.gcs_ctx_set_atlas(self.h, L.dptr(d)), "set_atlas")

    def set_belief(self, X_anchor, stamp, z_lin, Lm, h):
        b = L.belief_to_struct(X_anchor, stamp, z_lin, Lm, h)
        self._chk(self.lib.gcs_ctx_set_belief(self.h, C.byref(b)), "set_belief")

    def get_belief(self):
        b = L.GcsBelief()
        self._chk(self.lib.gcs_ctx_get_belief(self.h, C.byref(b)), "get_belief")
        return L.struct_to_arrays(b)

    def get_map(self):
        B = self.n_bins
        m = np.zeros(L.MAP_FIELDS * B)
        d = np.zeros(L.DERIVED_FIELDS * B)
        self._chk(self.lib.gcs_ctx_get_map(self.h, L.dptr(m), L.dptr(d)), "get_map")
        return m.reshape(L.MAP_FIELDS, B), d.reshape(L.DERIVED_FIELDS, B)

    def set_map(self, map_fields):
        m = np.ascontiguousarray(map_fields, np.float64).reshape(-1)
        self._chk(self.lib.gcs_ctx_set_map(self.h, L.dptr(m)), "set_map")

    def get_scan_stats(self):
        B = self.n_bins
        s = np.zeros(L.SCAN_FIELDS * B)
        self._chk(self.lib.gcs_ctx_get_scan_stats(self.h, L.dptr(s)), "get_scan_stats")
        return s.reshape(L.SCAN_FIELDS, B)

    def iw_state(self):
        nu, Psi, Q = np.zeros(7), np.zeros(252), np.zeros(484)
        self._chk(self.lib.gcs_ctx_get_iw_state(self.h, L.dptr(nu), L.dptr(Psi), L.dptr(Q)), "get_iw_state")
        return nu, Psi.reshape(7, 6, 6), Q.reshape(22, 22)

    def meas_iw_state(self):
        """Measurement-noise IW state: nu (3,), Psi (3,3,3), cert [psd_delta, nu_delta] of the last apply."""
        nu, Psi, cert = np.zeros(3), np.zeros(27), np.zeros(2)
        self._chk(self.lib.gcs_ctx_get_meas_iw_state(self.h, L.dptr(nu), L.dptr(Psi), L.dptr(cert)),
                  "get_meas_iw_state")
        return nu, Psi.reshape(3, 3, 3), cert

    def set_meas_iw_state(self, nu, Psi):
        n = np.ascontiguousarray(nu, np.float64).reshape(3)
        P = np.ascontiguousarray(Psi, np.float64).reshape(27)
        self._chk(self.lib.gcs_ctx_set_meas_iw_state(self.h, L.dptr(n), L.dptr(P)), "set_meas_iw_state")

    STAGES = ("points", "sort_bucket", "bins", "matrix_fisher", "planar", "pushforward", "budget", "bins_fold")

    def enable_timing(self, on=True, stages=None):
        """Device stage timing (hipEvents stamped by the stage kernels).  stages: names from
        STAGES to time (default all); on=False turns timing off."""
        mask = 0
        if on:
            names = self.STAGES if stages is None else stages
            for s in names:
                mask |= 1 << self.STAGES.index(s)
        self._chk(self.lib.gcs_ctx_enable_timing(self.h, mask), "enable_timing")

    def stage_times(self, reset=False):
        ms = np.zeros(len(self.STAGES))
        cnt = np.zeros(len(self.STAGES), np.int64)
        self._chk(self.lib.gcs_ctx_stage_times(self.h, L.dptr(ms), cnt.ctypes.data_as(L.c_int64_p), int(reset)),
                  "stage_times")
        return ms, cnt

    def describe(self):
        """gcs_ctx_describe: the library's runtime description of this context (RuntimeManifest)."""
        import json
        buf = C.create_string_buffer(4096)
        self._chk(self.lib.gcs_ctx_describe(self.h, buf, len(buf)), "describe")
        return json.loads(buf.value.decode())

    def set_debug(self, key, value):
        """gcs_ctx_set_debug (test knobs: L.DEBUG_SCAN_SPIN_LIMIT, L.DEBUG_INJECT_SCAN_FAIL)."""
        self._chk(self.lib.gcs_ctx_set_debug(self.h, int(key), int(value)), "set_debug")

    HOST_SPLIT = ("pre_device", "device_wait", "tail", "gcs_scan", "pre_predict", "launch_calls", "tail_numerics",
                  "push_launch", "combine", "scan_combine_call")

    def host_split(self, reset=False):
        """gcs_ctx_host_split: the host split of every scan since the last reset, summed in the library
        (ms; HOST_SPLIT names), and (scans, gcs_scan_combine calls) counted."""
        ms = np.zeros(10)
        n = np.zeros(2, np.int64)
        if not hasattr(self.lib, "gcs_ctx_host_split"):  # an older build in a same-box A/B
            return dict(zip(self.HOST_SPLIT, ms.tolist())), (0, 0)
        self._chk(self.lib.gcs_ctx_host_split(self.h, L.dptr(ms), n.ctypes.data_as(L.c_int64_p), int(reset)),
                  "host_split")
        return dict(zip(self.HOST_SPLIT, ms.tolist())), (int(n[0]), int(n[1]))

    HOST_HIST = ("pre_device", "device_wait", "tail", "gcs_scan", "combine", "scan_combine_call")

    def host_split_history(self, n_max=4096):
        """gcs_ctx_host_split_history: the per-scan host split of the latest scans since the last reset
        (oldest first), an (n, 6) float32 array with columns HOST_HIST (ms); None from an older build."""
        if not hasattr(self.lib, "gcs_ctx_host_split_history"):
            return None
        out = np.zeros((int(n_max), 6), np.float32)
        n = C.c_int32(0)
        self._chk(self.lib.gcs_ctx_host_split_history(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), int(n_max),
                                                      C.byref(n)), "host_split_history")
        return out[:n.value]

    def worker_tid(self):
        """gcs_ctx_worker_tid: the OS thread id of the context's launch worker (0: not started)."""
        return int(self.lib.gcs_ctx_worker_tid(self.h)) if hasattr(self.lib, "gcs_ctx_worker_tid") else 0

    def mirror_stats(self):
        """gcs_ctx_mirror_stats: (scan mirrors accepted, of them re-read at least once, via stream sync,
        all-reduces run, re-read, via stream sync)."""
        out = np.zeros(6, np.int64)
        self._chk(self.lib.gcs_ctx_mirror_stats(self.h, out.ctypes.data_as(L.c_int64_p)), "mirror_stats")
        return tuple(int(x) for x in out)

    def state_checksums(self):
        """gcs_debug_state_checksums: FNV-1a of [ScanBinStats, map, derived, touched, flags, bin-kernel
        partial rows, device scalars, host mirror scalars] after the context's streams drain."""
        out = np.zeros(8, np.uint64)
        self._chk(self.lib.gcs_debug_state_checksums(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64))),
                  "state_checksums")
        return tuple(int(x) for x in out)

    def synchronize(self):
        self._chk(self.lib.gcs_ctx_synchronize(self.h), "synchronize")

    # ------------------------------------------------------------------ per-operator stages
    def point_stage(self, xyz_dev, point_step, t_dev, w_dev, n_points, t0, t1, xi_body, want_outputs=True):
        """Fused PointBudgetResample + DeskewConstantTwist + directions + soft-assign normalisers."""
        torch = _torch()
        cap = self.cap
        dev = f"cuda:{self.device}"
        p0 = torch.zeros((cap, 3), dtype=torch.float64, device=dev) if want_outputs else None
        wo = torch.zeros(cap, dtype=torch.float64, device=dev) if want_outputs else None
        wb = torch.zeros(cap, dtype=torch.float64, device=dev) if want_outputs else None
        nearest = torch.zeros(cap, dtype=torch.int32, device=dev) if want_outputs else None
        xi = np.ascontiguousarray(xi_body, np.float64)
        cert = np.zeros(8)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        rc = self.lib.gcs_point_stage(self.h, C.c_void_p(xyz_dev.data_ptr()), int(point_step),
                                      C.c_void_p(t_dev.data_ptr()), C.c_void_p(w_dev.data_ptr()), int(n_points),
                                      float(t0), float(t1), L.dptr(xi), ptr(p0), ptr(wo), ptr(wb), ptr(nearest),
                                      L.dptr(cert))
        self._chk(rc, "point_stage")
        return dict(points=p0, weights=wo, budget_weights=wb, nearest=nearest, cert=cert)

    def bin_soft_assign(self):
        torch = _torch()
        dev = f"cuda:{self.device}"
        if self.mode == "scale":
            ids = torch.zeros((self.cap, self.cfg.k_cand), dtype=torch.int32, device=dev)
            r = torch.zeros((self.cap, self.cfg.k_cand), dtype=torch.float64, device=dev)
        else:
            ids = None
            r = torch.zeros((self.cap, self.n_bins), dtype=torch.float64, device=dev)
        rc = self.lib.gcs_bin_soft_assign(self.h, C.c_void_p(ids.data_ptr()) if ids is not None else None,
                                          C.c_void_p(r.data_ptr()))
        self._chk(rc, "bin_soft_assign")
        return ids, r

    def scan_bin_moment_match(self):
        cert = np.zeros(5)
        self._chk(self.lib.gcs_scan_bin_moment_match(self.h, L.dptr(cert)), "scan_bin_moment_match")
        return cert

    def matrix_fisher_rotation(self):
        out = np.zeros(42)
        self._chk(self.lib.gcs_matrix_fisher_rotation(self.h, L.dptr(out)), "matrix_fisher_rotation")
        return dict(H=out[0:9].reshape(3, 3), N_eff=out[9], map_scatter_total=out[10:19].reshape(3, 3),
                    map_N_dir_total=out[19], scan_N_total=out[20], R_mf=out[21:30].reshape(3, 3),
                    svd_s=out[30:33], V=out[33:42].reshape(3, 3))

    def planar_translation(self, R_hat):
        R = np.ascontiguousarray(R_hat, np.float64).reshape(9)
        out = np.zeros(13)
        self._chk(self.lib.gcs_planar_translation(self.h, L.dptr(R), L.dptr(out)), "planar_translation")
        return dict(L_full=out[0:9].reshape(3, 3), h_full=out[9:12], N_eff=out[12])

    def pushforward(self, z_t, Sigma_pose6, gamma):
        z = np.ascontiguousarray(z_t, np.float64)
        S = np.ascontiguousarray(Sigma_pose6, np.float64).reshape(36)
        self._chk(self.lib.gcs_pushforward(self.h, L.dptr(z), L.dptr(S), float(gamma)), "pushforward")

    # ------------------------------------------------------------------ the scan
    def _scan_inputs(self, xyz_dev, point_step, t_dev, w_dev, n_points, imu_stamps, imu_gyro, imu_accel,
                     scan_start_time, scan_end_time, dt_sec, Q=None, L_ext=None, h_ext=None, t_last_scan=None,
                     t_scan=None, xyz_f64=False, odom_pose=None, odom_cov_se3=None, odom_twist=None,
                     odom_twist_cov=None, Sigma_g=None, Sigma_a=None):
        """gcs_scan_inputs for gcs_scan / gcs_scan_begin; returns (struct, arrays to keep alive)."""
        imu_stamps = np.ascontiguousarray(imu_stamps, np.float64)
        imu_gyro = np.ascontiguousarray(imu_gyro, np.float64).reshape(-1)
        imu_accel = np.ascontiguousarray(imu_accel, np.float64).reshape(-1)
        inp = L.GcsScanInputs()
        inp.xyz_dev = xyz_dev.data_ptr()
        inp.point_step = int(point_step)
        inp.timestamps_dev = t_dev.data_ptr()
        inp.weights_dev = w_dev.data_ptr()
        inp.n_points = int(n_points)
        inp.imu_stamps = _addr(imu_stamps)
        inp.imu_gyro = _addr(imu_gyro)
        inp.imu_accel = _addr(imu_accel)
        inp.imu_len = int(imu_stamps.shape[0])
        inp.scan_start_time = float(scan_start_time)
        inp.scan_end_time = float(scan_end_time)
        inp.dt_sec = float(dt_sec)
        inp.t_last_scan = float(scan_start_time if t_last_scan is None else t_last_scan)
        inp.t_scan = float(scan_end_time if t_scan is None else t_scan)
        inp.xyz_format = 1 if xyz_f64 else 0
        keep = [imu_stamps, imu_gyro, imu_accel]
        for name, arr in (("Q", Q), ("L_ext", L_ext), ("h_ext", h_ext), ("odom_pose", odom_pose),
                          ("odom_cov_se3", odom_cov_se3), ("odom_twist", odom_twist), ("odom_twist_cov", odom_twist_cov),
                          ("Sigma_g", Sigma_g), ("Sigma_a", Sigma_a)):
            if arr is not None:
                a = np.ascontiguousarray(arr, np.float64).reshape(-1)
                keep.append(a)
                setattr(inp, name, _addr(a))
        return inp, keep

    def scan_begin(self, *args, **kw):
        """gcs_scan_begin (the live primitive path's first half; same arguments as scan()): returns a
        GcsScanBeginOutputs with z_lin_pose, pose_pred and the device arrays of the deskewed points,
        budget timestamps and deskewed weights (context-owned, valid until the next scan)."""
        import torch
        bufs = kw.pop("buffers", None)
        inp, keep = self._scan_inputs(*args, **kw)
        out = L.GcsScanBeginOutputs()
        if bufs is not None:  # caller-owned (points (cap,3), timestamps (cap,), weights (cap,)) f64 tensors
            p, t, w = bufs
            for x, n in ((p, 3 * self.cfg.n_points_cap), (t, self.cfg.n_points_cap), (w, self.cfg.n_points_cap)):
                if x.dtype != torch.float64 or not x.is_contiguous() or x.numel() != n:
                    raise ValueError("scan_begin buffers: contiguous f64 tensors of N_POINTS_CAP rows")
            out.points_dev, out.timestamps_dev, out.weights_dev = p.data_ptr(), t.data_ptr(), w.data_ptr()
        self._chk(self.lib.gcs_scan_begin(self.h, C.byref(inp), C.byref(out)), "gcs_scan_begin")
        del keep
        return out

    def scan_finish(self, L_lidar, h_lidar, trigger_sum, ess_sum, n_certs, nll_sum, out=None):
        """gcs_scan_finish with the live path's LiDAR evidence (visual_pose_evidence L_pose / h_pose) and
        the terms of its certificates (gcs_lidar_evidence)."""
        Lm = np.ascontiguousarray(L_lidar, np.float64).reshape(-1)
        hv = np.ascontiguousarray(h_lidar, np.float64).reshape(-1)
        ev = L.GcsLidarEvidence(_addr(Lm), _addr(hv), float(trigger_sum), float(ess_sum), int(n_certs), float(nll_sum))
        if out is None:
            out = L.GcsScanOutputs()
        self._chk(self.lib.gcs_scan_finish(self.h, C.byref(ev), C.byref(out)), "gcs_scan_finish")
        return out

    def prepare_scan(self, *args, **kw):
        """The gcs_scan_inputs of one scan (same arguments as scan()), built once: a caller that holds a
        scan's host arrays fills the C struct once and hands it to scan_prepared (a C caller fills it in
        a few hundred nanoseconds; ctypes takes microseconds per field)."""
        inp, keep = self._scan_inputs(*args, **kw)
        return (inp, C.byref(inp), keep)

    def scan_call(self, out):
        """gcs_scan bound once for prepare_scan() structs into the caller-owned out; returns
        call(prepared) -> None, raising on failure."""
        fn, h, po = self.lib.gcs_scan, self.h, C.byref(out)

        def call(prepared):
            rc = fn(h, prepared[1], po)
            if rc:
                self._chk(rc, "gcs_scan")
        return call

    def scan_prepared(self, prepared, out):
        """gcs_scan on a prepare_scan() struct into a caller-owned GcsScanOutputs (one ctypes call)."""
        rc = self.lib.gcs_scan(self.h, prepared[1], C.byref(out))
        if rc:
            self._chk(rc, "gcs_scan")
        return out

    def scan(self, xyz_dev, point_step, t_dev, w_dev, n_points, imu_stamps, imu_gyro, imu_accel,
             scan_start_time, scan_end_time, dt_sec, Q=None, L_ext=None, h_ext=None, t_last_scan=None, t_scan=None,
             xyz_f64=False, odom_pose=None, odom_cov_se3=None, odom_twist=None, odom_twist_cov=None, Sigma_g=None,
             Sigma_a=None, out=None):
        """gcs_scan.  t_last_scan / t_scan bound the scan-to-scan IMU window of the measurement-noise
        IW statistics and the IMU evidence (pipeline.py:331-332); default: the scan window.  xyz_f64:
        xyz_dev holds f64 x, y, z per point_step record (gcs_parse_pointcloud2 output, point_step 24).
        Odometry arguments left None take the node's "no odometry yet" inputs (backend_node.py:
        2047-2051); Sigma_g / Sigma_a None take the IW modes of the context's measurement state.
        out: a GcsScanOutputs to fill (the caller's, reused across scans); default a fresh one."""
        imu_stamps = np.ascontiguousarray(imu_stamps, np.float64)
        imu_gyro = np.ascontiguousarray(imu_gyro, np.float64).reshape(-1)
        imu_accel = np.ascontiguousarray(imu_accel, np.float64).reshape(-1)
        inp = L.GcsScanInputs()
        inp.xyz_dev = xyz_dev.data_ptr()
        inp.point_step = int(point_step)
        inp.timestamps_dev = t_dev.data_ptr()
        inp.weights_dev = w_dev.data_ptr()
        inp.n_points = int(n_points)
        inp.imu_stamps = _addr(imu_stamps)
        inp.imu_gyro = _addr(imu_gyro)
        inp.imu_accel = _addr(imu_accel)
        inp.imu_len = int(imu_stamps.shape[0])
        inp.scan_start_time = float(scan_start_time)
        inp.scan_end_time = float(scan_end_time)
        inp.dt_sec = float(dt_sec)
        inp.t_last_scan = float(scan_start_time if t_last_scan is None else t_last_scan)
        inp.t_scan = float(scan_end_time if t_scan is None else t_scan)
        inp.xyz_format = 1 if xyz_f64 else 0
        keep = []
        for name, arr in (("Q", Q), ("L_ext", L_ext), ("h_ext", h_ext), ("odom_pose", odom_pose),
                          ("odom_cov_se3", odom_cov_se3), ("odom_twist", odom_twist), ("odom_twist_cov", odom_twist_cov),
                          ("Sigma_g", Sigma_g), ("Sigma_a", Sigma_a)):
            if arr is not None:
                a = np.ascontiguousarray(arr, np.float64).reshape(-1)
                keep.append(a)
                setattr(inp, name, _addr(a))
        if out is None:
            out = L.GcsScanOutputs()
        self._chk(self.lib.gcs_scan(self.h, C.byref(inp), C.byref(out)), "gcs_scan")
        return out

    # ------------------------------------------------------------------ one map for all hypotheses
    def set_map_mode(self, mode):
        """"own" (default: this hypothesis' own map), "lead" (hypothesis 0: its map is the node's map)
        or "follow" (skips its own map update; map_follow replays the lead's), gcslam_hip.h GCS_MAP_*."""
        m = {"own": L.MAP_OWN, "lead": L.MAP_LEAD, "follow": L.MAP_FOLLOW}[mode]
        self._chk(self.lib.gcs_ctx_set_map_mode(self.h, m), "set_map_mode")

    def map_record(self):
        """The last scan's map-update record [deskew twist 6 | z_t 6 | pose covariance 36]."""
        r = np.empty(L.MAP_REC_LEN)
        self._chk(self.lib.gcs_ctx_map_record(self.h, r.ctypes.data), "map_record")
        return r

    def map_follow(self, prepared, rec=None):
        """Replay the lead's map update of this scan (prepared: prepare_scan() of the same scan; rec: the
        lead's map_record(), None = the record the last combine_allreduce carried)."""
        r = None if rec is None else np.ascontiguousarray(rec, np.float64)
        self._chk(self.lib.gcs_map_follow(self.h, prepared[1], None if r is None else r.ctypes.data), "map_follow")

    def map_follow_call(self):
        """gcs_map_follow bound once for prepare_scan() structs, with the record the last combine carried;
        returns call(prepared) -> None, raising on failure."""
        fn, h = self.lib.gcs_map_follow, self.h

        def call(prepared):
            rc = fn(h, prepared[1], None)
            if rc:
                self._chk(rc, "map_follow")
        return call

    # ------------------------------------------------------------------ hypotheses
    def hypothesis_payload(self, w_iw, w_bary):
        """Packed 840-f64 all-reduce payload of this hypothesis (a fresh array per call)."""
        p = np.empty(L.PAYLOAD_LEN)
        self._chk(self.lib.gcs_hypothesis_payload(self.h, float(w_iw), float(w_bary), p.ctypes.data), "payload")
        return p

    def combine_allreduce(self, comm, w_iw, w_bary, scan_count, want_belief=True):
        """gcs_combine_allreduce: payload pack + RCCL sum all-reduce on the context stream (comm =
        HypothesisComm handle; None = single rank) + combine and IW updates."""
        b = L.GcsBelief() if want_belief else None
        cert = np.empty(4)
        self._chk(self.lib.gcs_combine_allreduce(self.h, comm, float(w_iw), float(w_bary), int(scan_count),
                                                 C.addressof(b) if want_belief else None, cert.ctypes.data),
                  "combine_allreduce")
        return (L.struct_to_arrays(b) if want_belief else None), cert

    def combine_call(self, comm, w_iw, w_bary):
        """gcs_combine_allreduce bound once (the caller's per-scan loop: arguments converted and the cert
        buffer allocated here, not per call); returns call(scan_count) -> None, raising on failure."""
        fn, h, cert = self.lib.gcs_combine_allreduce, self.h, (C.c_double * 4)()
        comm, w_iw, w_bary = comm, float(w_iw), float(w_bary)

        def call(scan_count):
            rc = fn(h, comm, w_iw, w_bary, scan_count, None, cert)
            if rc:
                self._chk(rc, "combine_allreduce")
        return call

    def scan_combine_call(self, out, comm, w_iw, w_bary):
        """gcs_scan_combine (gcs_scan + gcs_combine_allreduce in one C call) bound once: returns
        call(prepared, scan_count) -> the combine's host ms, raising on failure."""
        fn, h, po = self.lib.gcs_scan_combine, self.h, C.byref(out)
        cert, cms = (C.c_double * 4)(), C.c_double()
        comm, w_iw, w_bary, pc = comm, float(w_iw), float(w_bary), C.byref(cms)

        def call(prepared, scan_count):
            rc = fn(h, prepared[1], po, comm, w_iw, w_bary, scan_count, None, cert, pc)
            if rc:
                self._chk(rc, "gcs_scan_combine")
            return cms.value
        return call

    def hypothesis_combine(self, payload_sum, scan_count, want_belief=True):
        """Barycenter + IW update from the summed payload; returns (belief arrays or None, cert)."""
        p = np.ascontiguousarray(payload_sum, np.float64)
        b = L.GcsBelief() if want_belief else None  # combined_out may be NULL (gcslam_hip.h)
        cert = np.empty(4)
        self._chk(self.lib.gcs_hypothesis_combine(self.h, p.ctypes.data, int(scan_count),
                                                  C.addressof(b) if want_belief else None, cert.ctypes.data),
                  "combine")
        return (L.struct_to_arrays(b) if want_belief else None), cert
