"""The live primitive path's OT association on the MI355X:
associate_primitives_ot with the reference's calling convention
(FS/backend/operators/primitive_association.py:239-553 -> (PrimitiveAssociationResult, CertBundle,
ExpectedEffect)), running gcs_associate_primitives_ot (libgcslam_hip.so).  The measurement side is
gcslam.surfels.MeasurementBatch (device tensors); the map side is an AtlasMapView
(FS/backend/structures/primitive_map.py:270-300) whose arrays the caller builds from its primitive
map (the map itself -- fuse / insert / cull -- is not part of this library)."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from enum import Enum
from typing import Optional

import numpy as np

from . import _lib as L
from .certificates import CertBundle, ComputeCert, ExpectedEffect, InfluenceCert, OTCert, SupportCert

CHART_ID = "GC-RIGHT-01"
GC_EPS_LIFT = 1e-9
GC_EPS_MASS = 1e-12


class MeasurementMassPolicy(Enum):   # primitive_association.py:40-48
    UNIFORM = "uniform"
    WEIGHT_PROPORTIONAL = "weight_proportional"
    FEATURE_CONFIDENCE = "feature_confidence"


class MapMassPolicy(Enum):           # primitive_association.py:51-59
    UNIFORM = "uniform"
    PRIMITIVE_MASS = "primitive_mass"
    MASS_TEMPERED = "mass_tempered"


_A_CODE = {MeasurementMassPolicy.UNIFORM: 0, MeasurementMassPolicy.WEIGHT_PROPORTIONAL: 1,
           MeasurementMassPolicy.FEATURE_CONFIDENCE: 2}
_B_CODE = {MapMassPolicy.UNIFORM: 0, MapMassPolicy.PRIMITIVE_MASS: 1, MapMassPolicy.MASS_TEMPERED: 2}


@dataclass
class AssociationConfig:
    """primitive_association.py:206-236 (same fields and defaults)."""
    k_assoc: int = 8
    k_sinkhorn: int = 50
    beta: float = 0.5
    epsilon: float = 0.1
    tau_a: float = 0.5
    tau_b: float = 0.5
    cost_subtract_row_min: bool = True
    cost_scale_by_median: bool = False
    a_policy: MeasurementMassPolicy = MeasurementMassPolicy.UNIFORM
    b_policy: MapMassPolicy = MapMassPolicy.UNIFORM
    eps_mass: float = GC_EPS_MASS
    h_tile: float = 2.0
    r_stencil_tiles_xy: int = 1
    r_stencil_tiles_z: int = 0
    scan_seq: int = 0
    recency_decay_lambda: float = 0.02


@dataclass
class AtlasMapView:
    """primitive_map.py:270-300 (device tensors; the fields association reads are required)."""
    candidate_tile_ids: object   # (M,) int64
    candidate_slots: object      # (M,) int32
    valid_mask: object           # (M,) bool
    tile_ids: object             # (n_tiles,) int64
    m_tile_view: int
    positions: object            # (M, 3)
    directions: object           # (M, 3)
    kappas: object               # (M,)
    last_supported_scan_seq: object  # (M,) int64
    primitive_ids: object = None
    covariances: object = None
    weights: object = None
    etas: object = None
    colors: object = None

    @property
    def count(self) -> int:
        return int(self.positions.shape[0])


@dataclass
class PrimitiveAssociationResult:
    """primitive_association.py:71-92."""
    responsibilities: object       # (N, K) f64
    candidate_pool_indices: object  # (N, K) int32
    candidate_tile_ids: object     # (N, K) int64
    candidate_slots: object        # (N, K) int64
    row_masses: object             # (N,)
    cost_matrix: object            # (N, K)
    # this build's addition: the MapUpdateCert's candidate statistics (pipeline.py:879-905: distinct
    # candidate tiles and valid candidates per valid measurement, their means and the counts' p95),
    # computed by the library beside the Sinkhorn, so the pipeline needs no device round trip for them
    candidate_stats: tuple = (0.0, 0.0, 0.0)


def _torch():
    import torch
    return torch


class Associator:
    """A gcs_assoc_ctx: workspace for up to max_meas rows, max_pool view entries, k_assoc <= max_k."""

    def __init__(self, max_meas=1536, max_pool=7 * 1024, max_k=8, device=0):
        self.lib = L.load()
        h = C.c_void_p()
        rc = self.lib.gcs_assoc_ctx_create(int(max_meas), int(max_pool), int(max_k), int(device), C.byref(h))
        if rc != 0:
            raise (ValueError if rc == -1 else RuntimeError)(f"gcs_assoc_ctx_create failed ({rc})")
        self.h = h
        self.device, self.max_meas, self.max_pool, self.max_k = int(device), int(max_meas), int(max_pool), int(max_k)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gcs_assoc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.gcs_assoc_last_error(self.h).decode(errors="replace")
            raise (ValueError if rc in (-1, -3) else RuntimeError)(f"{what} failed ({rc}): {msg}")

    def run(self, batch, view: AtlasMapView, config: AssociationConfig, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
        """Result tensors (fresh device tensors) + the cert scalars (dict) + exact flag."""
        call = self.prepare(batch, view, config, eps_lift, eps_mass)
        o = call()
        cert = {k: float(o.cert[i]) for i, k in enumerate(L.ASSOC_CERT_FIELDS)}
        return call.out, cert, bool(o.exact)

    def prepare(self, batch, view: AtlasMapView, config: AssociationConfig, eps_lift=GC_EPS_LIFT,
                eps_mass=GC_EPS_MASS):
        """The C-ABI call of `run` with its argument structs and device tensors built: call() runs
        gcs_associate_primitives_ot again on the same inputs into the same outputs (call.out) and
        returns the outputs struct -- the boundary call a C caller makes, without the Python argument
        marshalling (tools/assoc_bench.py times both)."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        f64 = lambda x: torch.as_tensor(x, device=dev).to(torch.float64).contiguous()  # noqa: E731
        u8 = lambda x: torch.as_tensor(x, device=dev).to(torch.uint8).contiguous()  # noqa: E731
        i64 = lambda x: torch.as_tensor(x, device=dev).to(torch.int64).contiguous()  # noqa: E731
        keep = [f64(batch.Lambdas), f64(batch.thetas), f64(batch.etas), f64(batch.weights), u8(batch.valid_mask),
                i64(view.tile_ids), f64(view.positions), f64(view.directions), f64(view.kappas), u8(view.valid_mask),
                i64(view.last_supported_scan_seq), i64(view.candidate_tile_ids),
                torch.as_tensor(view.candidate_slots, device=dev).to(torch.int32).contiguous()]
        N = int(keep[0].shape[0])
        etas = keep[2]
        m = L.GcsAssocMeas()
        m.Lambdas, m.thetas, m.etas, m.weights, m.valid_mask = (t.data_ptr() for t in keep[:5])
        m.n_total, m.n_lobes = N, int(etas.shape[1]) if etas.dim() == 3 else 1
        m.n_valid = int(batch.n_valid)
        v = L.GcsAssocView()
        v.tile_ids = keep[5].data_ptr()
        v.n_tiles, v.m_tile_view = int(keep[5].shape[0]), int(view.m_tile_view)
        (v.positions, v.directions, v.kappas, v.valid_mask, v.last_supported_scan_seq, v.candidate_tile_ids,
         v.candidate_slots) = (t.data_ptr() for t in keep[6:])
        out, o = assoc_outputs(N, int(config.k_assoc), dev)
        c = assoc_config_struct(config, eps_lift, eps_mass)
        self._chk(self.lib.gcs_assoc_ctx_set_stream(self.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                  "gcs_assoc_ctx_set_stream")
        lib, h, chk = self.lib, self.h, self._chk
        args = (h, C.byref(c), C.byref(m), C.byref(v), C.byref(o))

        def call():
            chk(lib.gcs_associate_primitives_ot(*args), "gcs_associate_primitives_ot")
            return o
        call.out, call.keep = out, (keep, c, m, v, o)
        return call


    def pose_evidence(self, batch, view: AtlasMapView, result, k_assoc: int, z_lin_pose, eps_lift=GC_EPS_LIFT,
                      eps_mass=GC_EPS_MASS):
        """gcs_visual_pose_evidence: the 22-D pose evidence of an association result (host struct)."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        f64 = lambda x: torch.as_tensor(x, device=dev).to(torch.float64).contiguous()  # noqa: E731
        u8 = lambda x: torch.as_tensor(x, device=dev).to(torch.uint8).contiguous()  # noqa: E731
        keep = [f64(batch.Lambdas), f64(batch.thetas), f64(batch.etas), u8(batch.valid_mask), f64(view.positions),
                f64(view.directions), f64(view.kappas), u8(view.valid_mask), f64(result.responsibilities),
                torch.as_tensor(result.candidate_pool_indices, device=dev).to(torch.int32).contiguous(),
                f64(result.row_masses)]
        N = int(keep[0].shape[0])
        m = L.GcsAssocMeas()
        m.Lambdas, m.thetas, m.etas, m.valid_mask = (t.data_ptr() for t in keep[:4])
        m.n_total = N
        m.n_lobes = int(keep[2].reshape(N, -1, 3).shape[1])
        m.n_valid = int(batch.n_valid)
        v = L.GcsAssocView()
        v.positions, v.directions, v.kappas, v.valid_mask = (t.data_ptr() for t in keep[4:8])
        v.n_tiles, v.m_tile_view = 1, int(keep[7].shape[0])
        o = L.GcsVpeOutputs()
        z = np.ascontiguousarray(np.asarray(z_lin_pose, dtype=np.float64).ravel()[:6])
        self._chk(self.lib.gcs_assoc_ctx_set_stream(self.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                  "gcs_assoc_ctx_set_stream")
        self._chk(self.lib.gcs_visual_pose_evidence(self.h, C.byref(m), C.byref(v), C.c_void_p(keep[8].data_ptr()),
                                                    C.c_void_p(keep[9].data_ptr()), C.c_void_p(keep[10].data_ptr()),
                                                    int(k_assoc), L.dptr(z), float(eps_lift), float(eps_mass),
                                                    C.byref(o)), "gcs_visual_pose_evidence")
        return o


def assoc_outputs(N: int, K: int, dev: str):
    """Fresh PrimitiveAssociationResult tensors (N x K) and the gcs_assoc_outputs struct naming them."""
    torch = _torch()
    out = dict(responsibilities=torch.empty((N, K), dtype=torch.float64, device=dev),
               candidate_pool_indices=torch.empty((N, K), dtype=torch.int32, device=dev),
               candidate_tile_ids=torch.empty((N, K), dtype=torch.int64, device=dev),
               candidate_slots=torch.empty((N, K), dtype=torch.int64, device=dev),
               row_masses=torch.empty((N,), dtype=torch.float64, device=dev),
               cost_matrix=torch.empty((N, K), dtype=torch.float64, device=dev))
    o = L.GcsAssocOutputs()
    for k, t in out.items():
        setattr(o, k, t.data_ptr())
    return out, o


def assoc_config_struct(config: AssociationConfig, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """gcs_assoc_config of an AssociationConfig and the operator's eps_lift / eps_mass arguments."""
    c = L.GcsAssocConfig()
    L.check(L.load().gcs_assoc_config_defaults(C.byref(c)), None, "gcs_assoc_config_defaults")
    c.k_assoc, c.k_sinkhorn = int(config.k_assoc), int(config.k_sinkhorn)
    c.beta, c.epsilon, c.tau_a, c.tau_b = float(config.beta), float(config.epsilon), float(config.tau_a), \
        float(config.tau_b)
    c.cost_subtract_row_min, c.cost_scale_by_median = int(bool(config.cost_subtract_row_min)), \
        int(bool(config.cost_scale_by_median))
    c.a_policy, c.b_policy = _A_CODE[config.a_policy], _B_CODE[config.b_policy]
    c.eps_mass, c.eps_lift, c.eps_mass_dir = float(config.eps_mass), float(eps_lift), float(eps_mass)
    c.h_tile = float(config.h_tile)
    c.r_stencil_tiles_xy, c.r_stencil_tiles_z = int(config.r_stencil_tiles_xy), int(config.r_stencil_tiles_z)
    c.scan_seq, c.recency_decay_lambda = int(config.scan_seq), float(config.recency_decay_lambda)
    return c


def association_result(out: dict, o) -> "PrimitiveAssociationResult":
    """The PrimitiveAssociationResult of filled outputs (candidate statistics from the cert slots)."""
    cs = (float(o.cert[18]), float(o.cert[19]), float(o.cert[20]))
    return PrimitiveAssociationResult(**out, candidate_stats=cs)


def association_cert(o, config: AssociationConfig, N: int, chart_id: str = CHART_ID, anchor_id: str = "primitive_ot"):
    """(CertBundle, ExpectedEffect) of an association call's host results (o: gcs_assoc_outputs)."""
    if o.exact:
        cert = CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id)
        return cert, ExpectedEffect(objective_name="primitive_association_ot", predicted=0.0, realized=0.0)
    cv = {k: float(o.cert[i]) for i, k in enumerate(L.ASSOC_CERT_FIELDS)}
    K = int(config.k_assoc)
    compute = ComputeCert(alloc_bytes_est=int(N * K * 8 * 4), largest_tensor_shape=(N, K), segment_sum_k=K,
                          psd_projection_count=0, chol_solve_count=0)
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id, triggers=["sinkhorn_fixed_iter", "sinkhorn_unbalanced_kl_relax"],
        frobenius_applied=False, support=SupportCert(ess_total=cv["ess_total"], support_frac=cv["support_frac"]),
        influence=InfluenceCert.identity().with_overrides(mass_epsilon_ratio=cv["mass_epsilon_ratio"]),
        compute=compute)
    cert.ot = OTCert(marginal_defect_a=cv["marginal_defect_a"], marginal_defect_b=cv["marginal_defect_b"],
                     transport_mass_total=cv["transport_mass_total"], dual_gap_proxy=0.0, sum_a=cv["sum_a"],
                     sum_b=cv["sum_b"], sum_m=cv["sum_m"], sum_novel=cv["sum_novel"], p95_a=cv["p95_a"],
                     p95_b=cv["p95_b"], nonzero_a=int(cv["nonzero_a"]), nonzero_b=int(cv["nonzero_b"]),
                     epsilon=float(config.epsilon), tau_a=float(config.tau_a), tau_b=float(config.tau_b),
                     n_iters=int(config.k_sinkhorn), b_policy=str(config.b_policy.value),
                     b_recency_decay_lambda=float(config.recency_decay_lambda), b_recency_p95=cv["b_recency_p95"])
    effect = ExpectedEffect(objective_name="primitive_association_ot", predicted=cv["total_cost"],
                            realized=cv["total_cost"])
    return cert, effect


_associators = {}


def _associator_for(n, pool, k, device):
    key = device
    a = _associators.get(key)
    if a is None or a.max_meas < n or a.max_pool < pool or a.max_k < k:
        if a is not None:
            a.close()
        mk = max(k, 8)
        a = Associator(max_meas=max(n, 1536 if mk <= 8 else 1024), max_pool=max(pool, 7 * 1024), max_k=mk,
                       device=device)
        _associators[key] = a
    return a


def associate_primitives_ot(measurement_batch, map_view: AtlasMapView, config: Optional[AssociationConfig] = None,
                            eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS, chart_id: str = CHART_ID,
                            anchor_id: str = "primitive_ot", device: int = 0, associator: Associator = None):
    """primitive_association.py:239-553.  Fixed-cost operator: output shape (n_total, k_assoc)."""
    if config is None:
        config = AssociationConfig()
    N = int(measurement_batch.n_total)
    K = int(config.k_assoc)
    pool = int(np.asarray(map_view.tile_ids.shape)[0]) * int(map_view.m_tile_view)
    a = associator or _associator_for(N, pool, K, device)
    call = a.prepare(measurement_batch, map_view, config, eps_lift, eps_mass)
    o = call()
    cert, effect = association_cert(o, config, N, chart_id, anchor_id)
    return association_result(call.out, o), cert, effect


@dataclass
class VisualPoseEvidenceResult:      # visual_pose_evidence.py:46-66
    L_pose: np.ndarray
    h_pose: np.ndarray
    L_trans: np.ndarray
    h_trans: np.ndarray
    L_rot: np.ndarray
    h_rot: np.ndarray
    total_weighted_cost: float
    n_associations: int
    mean_transported_mass: float


def visual_pose_evidence(association_result: PrimitiveAssociationResult, measurement_batch, map_view: AtlasMapView,
                         belief_pred=None, eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS,
                         chart_id: str = CHART_ID, anchor_id: str = "visual_pose_evidence", z_lin_pose=None,
                         device: int = 0, associator: Associator = None):
    """visual_pose_evidence.py:260-412: 22-D pose evidence from the OT soft correspondences at
    z_lin_pose (or belief_pred.mean_world_pose()).  Returns (VisualPoseEvidenceResult, CertBundle,
    ExpectedEffect); the sums run on the GPU (gcs_visual_pose_evidence), the 3x3 SVD on the host."""
    if z_lin_pose is None:
        if belief_pred is None:
            raise ValueError("visual_pose_evidence needs z_lin_pose or belief_pred")
        z_lin_pose = belief_pred.mean_world_pose(eps_lift=eps_lift)
    torch = _torch()
    r = association_result.responsibilities
    N, K = (int(x) for x in (r.shape if torch.is_tensor(r) else np.asarray(r).shape))
    pool = int(np.asarray(map_view.valid_mask.shape)[0])
    a = associator or _associator_for(max(N, 1), pool, max(K, 1), device)
    o = a.pose_evidence(measurement_batch, map_view, association_result, K, z_lin_pose, eps_lift, eps_mass)
    return visual_pose_result(o, eps_lift, chart_id, anchor_id)


def visual_pose_result(o, eps_lift=GC_EPS_LIFT, chart_id: str = CHART_ID, anchor_id: str = "visual_pose_evidence"):
    """(VisualPoseEvidenceResult, CertBundle, ExpectedEffect) of gcs_visual_pose_evidence's outputs."""
    view = np.ctypeslib.as_array
    res = VisualPoseEvidenceResult(L_pose=view(o.L_pose).reshape(22, 22).copy(), h_pose=view(o.h_pose).copy(),
                                   L_trans=view(o.L_trans).reshape(3, 3).copy(), h_trans=view(o.h_trans).copy(),
                                   L_rot=view(o.L_rot).reshape(3, 3).copy(), h_rot=view(o.h_rot).copy(),
                                   total_weighted_cost=float(o.total_weighted_cost),
                                   n_associations=int(o.n_associations),
                                   mean_transported_mass=float(o.mean_transported_mass))
    if o.exact:
        return res, CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id), ExpectedEffect(
            objective_name="visual_pose_evidence", predicted=0.0, realized=0.0)
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id,
                                    triggers=["linearization", "ot_soft_correspondence"], frobenius_applied=True,
                                    support=SupportCert(ess_total=float(o.ess_total), support_frac=float(o.support_frac)),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=eps_lift))
    c = float(o.total_weighted_cost)
    return res, cert, ExpectedEffect(objective_name="visual_pose_evidence", predicted=c, realized=c)


def build_visual_pose_evidence_22d(visual_result: VisualPoseEvidenceResult):
    """visual_pose_evidence.py:420-433."""
    return visual_result.L_pose, visual_result.h_pose
