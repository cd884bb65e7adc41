"""Certificate structures mirroring FS/common/certificates.py (the fields that are numerically live
on the bin path: influence magnitudes feed the Frobenius strength, support feeds tempering)."""

from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import List, Optional


@dataclass
class ConditioningCert:          # certificates.py:22-35
    eig_min: float = 1.0
    eig_max: float = 1.0
    cond: float = 1.0
    near_null_count: int = 0


@dataclass
class SupportCert:               # certificates.py:39-49
    ess_total: float = 0.0
    support_frac: float = 1.0


@dataclass
class MismatchCert:              # certificates.py:52-62
    nll_per_ess: float = 0.0
    directional_score: float = 1.0


@dataclass
class InfluenceCert:             # certificates.py:78-109
    lift_strength: float = 0.0
    psd_projection_delta: float = 0.0
    nu_projection_delta: float = 0.0
    mass_epsilon_ratio: float = 0.0
    anchor_drift_rho: float = 0.0
    dt_scale: float = 1.0
    extrinsic_scale: float = 1.0
    trust_alpha: float = 1.0
    power_beta: float = 1.0

    @classmethod
    def identity(cls):
        return cls()

    def with_overrides(self, **kw):
        return replace(self, **kw)


@dataclass
class ComputeCert:               # certificates.py:318-329 (shape / allocation accounting)
    alloc_bytes_est: int = 0
    largest_tensor_shape: tuple = (0, 0)
    segment_sum_k: int = 0
    psd_projection_count: int = 0
    chol_solve_count: int = 0


@dataclass
class OTCert:                    # certificates.py:152-181 (association diagnostics)
    marginal_defect_a: float = 0.0
    marginal_defect_b: float = 0.0
    transport_mass_total: float = 0.0
    dual_gap_proxy: float = 0.0
    sum_a: float = 0.0
    sum_b: float = 0.0
    sum_m: float = 0.0
    sum_novel: float = 0.0
    p95_a: float = 0.0
    p95_b: float = 0.0
    nonzero_a: int = 0
    nonzero_b: int = 0
    epsilon: float = 0.0
    tau_a: float = 0.0
    tau_b: float = 0.0
    n_iters: int = 0
    b_policy: str = ""
    b_recency_decay_lambda: float = 0.0
    b_recency_p95: float = 0.0


@dataclass
class CertBundle:                # certificates.py:349-486
    chart_id: str
    anchor_id: str
    exact: bool
    approximation_triggers: List[str] = field(default_factory=list)
    frobenius_applied: bool = False
    conditioning: ConditioningCert = field(default_factory=ConditioningCert)
    support: SupportCert = field(default_factory=SupportCert)
    mismatch: MismatchCert = field(default_factory=MismatchCert)
    influence: InfluenceCert = field(default_factory=InfluenceCert)
    compute: ComputeCert = field(default_factory=ComputeCert)
    ot: Optional[OTCert] = None  # populated by the association operator

    @classmethod
    def create_exact(cls, chart_id, anchor_id, **kw):
        return cls(chart_id=chart_id, anchor_id=anchor_id, exact=True, **kw)

    @classmethod
    def create_approx(cls, chart_id, anchor_id, triggers, **kw):
        return cls(chart_id=chart_id, anchor_id=anchor_id, exact=False, approximation_triggers=list(triggers), **kw)

    def total_trigger_magnitude(self) -> float:
        i = self.influence
        return (i.lift_strength + i.psd_projection_delta + i.nu_projection_delta + i.mass_epsilon_ratio
                + i.anchor_drift_rho + abs(1.0 - i.dt_scale) + abs(1.0 - i.extrinsic_scale)
                + abs(1.0 - i.trust_alpha) + abs(1.0 - i.power_beta))


@dataclass
class ExpectedEffect:            # certificates.py:488-505
    objective_name: str
    predicted: float
    realized: Optional[float] = None


def aggregate_certificates(certs: List[CertBundle]) -> CertBundle:
    """certificates.py:511-700 restricted to the fields carried here."""
    if not certs:
        return CertBundle.create_exact("GC-RIGHT-01", "unknown")
    t = certs[0]
    n = len(certs)
    # one pass over the certs; every sum in list order from 0 and every min / max from the first cert,
    # as the per-field generator expressions (sum(), min(), max()) take them
    c0 = certs[0]
    cd, sp, mm, inf = c0.conditioning, c0.support, c0.mismatch, c0.influence
    exact, frob, trig = c0.exact, c0.frobenius_applied, list(c0.approximation_triggers)
    e_min, e_max, cond, nn = cd.eig_min, cd.eig_max, cd.cond, 0 + cd.near_null_count
    ess, sfr, nll, dsc = 0 + sp.ess_total, 0 + sp.support_frac, 0 + mm.nll_per_ess, 0 + mm.directional_score
    ls, pd, nd = 0 + inf.lift_strength, 0 + inf.psd_projection_delta, 0 + inf.nu_projection_delta
    me, ad, dts, ext, ta, pb = (inf.mass_epsilon_ratio, inf.anchor_drift_rho, inf.dt_scale, inf.extrinsic_scale,
                                inf.trust_alpha, inf.power_beta)
    for c in certs[1:]:
        cd, sp, mm, inf = c.conditioning, c.support, c.mismatch, c.influence
        exact = exact and c.exact
        frob = frob or c.frobenius_applied
        trig.extend(c.approximation_triggers)
        e_min, e_max, cond = min(e_min, cd.eig_min), max(e_max, cd.eig_max), max(cond, cd.cond)
        nn += cd.near_null_count
        ess += sp.ess_total
        sfr += sp.support_frac
        nll += mm.nll_per_ess
        dsc += mm.directional_score
        ls += inf.lift_strength
        pd += inf.psd_projection_delta
        nd += inf.nu_projection_delta
        me, ad = max(me, inf.mass_epsilon_ratio), max(ad, inf.anchor_drift_rho)
        dts, ext = min(dts, inf.dt_scale), min(ext, inf.extrinsic_scale)
        ta, pb = min(ta, inf.trust_alpha), min(pb, inf.power_beta)
    return CertBundle(
        chart_id=t.chart_id, anchor_id=t.anchor_id, exact=bool(exact), approximation_triggers=trig,
        frobenius_applied=bool(frob), conditioning=ConditioningCert(e_min, e_max, cond, nn),
        support=SupportCert(ess / n, sfr / n), mismatch=MismatchCert(nll, dsc / n),
        influence=InfluenceCert(lift_strength=ls, psd_projection_delta=pd, nu_projection_delta=nd,
                                mass_epsilon_ratio=me, anchor_drift_rho=ad, dt_scale=dts, extrinsic_scale=ext,
                                trust_alpha=ta, power_beta=pb))
