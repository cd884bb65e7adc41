"""numpy restatement of the live path's LiDAR/visual pose evidence -- TEST INFRASTRUCTURE ONLY.

FS = fl_ws/src/fl_slam_poc/fl_slam_poc.  Follows FS/backend/operators/visual_pose_evidence.py:
  * _compute_translation_evidence_wls   :87-147
  * _compute_rotation_evidence_vmf      :150-240
  * visual_pose_evidence                :260-412 (valid-row filter, 22-D embedding, certificate)
with measurement_batch_mean_positions / _directions / _kappas (measurement_batch.py:389-411).
The product path never imports this; it is the checker of tests/test_gpu_primitive_evidence.py.
np.linalg.svd stands in for jnp.linalg.svd (LAPACK gesdd in both); U V^T and the singular values
do not depend on the SVD's sign convention for distinct singular values.  Parity unpinned: the
reference holds no outputs for this operator (tests/test_visual_lidar_plan.py checks only the
manifest's backend names).
"""

from __future__ import annotations

import numpy as np

from . import se3

GC_EPS_LIFT = 1e-9
GC_EPS_MASS = 1e-12


def visual_pose_evidence(batch, view, assoc, z_lin_pose, eps_lift=GC_EPS_LIFT, eps_mass=GC_EPS_MASS):
    """batch: Lambdas (N,3,3), thetas, etas (N,B,3), valid_mask, n_valid; view: positions, directions,
    kappas, valid_mask; assoc: responsibilities (N,K), candidate_pool_indices, row_masses.
    Returns a dict with the VisualPoseEvidenceResult fields plus ess_total / support_frac / exact."""
    N_meas = int(batch["n_valid"])
    N_assoc, K = np.asarray(assoc["responsibilities"]).shape
    if N_meas == 0 or N_assoc == 0 or int(np.sum(np.asarray(view["valid_mask"]).astype(np.int32))) == 0:
        return dict(L_pose=eps_lift * np.eye(22), h_pose=np.zeros(22), L_trans=np.zeros((3, 3)), h_trans=np.zeros(3),
                    L_rot=np.zeros((3, 3)), h_rot=np.zeros(3), total_weighted_cost=0.0, n_associations=0,
                    mean_transported_mass=0.0, exact=True)
    z = np.asarray(z_lin_pose, np.float64).ravel()[:6]
    t_pred, R = z[:3], se3.so3_exp(z[3:6])
    Lam = np.asarray(batch["Lambdas"], np.float64)
    Lreg = Lam + eps_lift * np.eye(3)[None]
    pos = np.linalg.solve(Lreg, np.asarray(batch["thetas"], np.float64)[..., None])[..., 0]
    es = np.sum(np.asarray(batch["etas"], np.float64), axis=1)
    kap = np.linalg.norm(es, axis=1)
    dirs = es / (kap[:, None] + eps_mass)
    vi = np.where(np.asarray(batch["valid_mask"]).astype(bool))[0][:N_meas]
    pos, dirs, kap, Lreg = pos[vi], dirs[vi], kap[vi], Lreg[vi]
    resp = np.asarray(assoc["responsibilities"], np.float64)[vi]
    cvi = np.asarray(assoc["candidate_pool_indices"]).astype(np.int64)[vi]
    rmass = np.asarray(assoc["row_masses"], np.float64)[vi]
    N_assoc = resp.shape[0]
    mpos = np.asarray(view["positions"], np.float64)
    mdir = np.asarray(view["directions"], np.float64)
    mkap = np.asarray(view["kappas"], np.float64)
    # translation (:121-147)
    mw = np.einsum("ij,nj->ni", R, pos)
    mp = mpos[cvi]
    resid = mp - mw[:, None, :] - t_pred[None, None, :]
    L_t = np.einsum("n,nij->ij", np.sum(resp, axis=1), Lreg)
    wt = np.einsum("nk,nkj->nj", resp, mp - mw[:, None, :])
    h_t = np.einsum("nij,nj->i", Lreg, wt)
    Lr = np.einsum("nij,nkj->nki", Lreg, resid)
    cost_t = float(np.sum(resp * np.einsum("nki,nki->nk", resid, Lr)))
    L_t = L_t + eps_lift * np.eye(3)
    # rotation (:209-240)
    md, mk = mdir[cvi], mkap[cvi]
    w = resp * np.sqrt(kap[:, None] * mk + 1e-12)
    S = np.einsum("nk,nki,nj->ij", w, md, dirs)
    dots = np.einsum("ni,nki->nk", np.einsum("ij,nj->ni", R, dirs), md)
    cost_r = float(np.sum(w * (1.0 - dots)))
    U, s, Vt = np.linalg.svd(S)
    L_rot = np.diag(s + eps_lift)
    Rs = U @ Vt
    if np.linalg.det(Rs) < 0:
        Rs = U @ np.diag([1.0, 1.0, -1.0]) @ Vt
    h_rot = L_rot @ se3.so3_log(Rs @ R.T)
    L = eps_lift * np.eye(22)
    h = np.zeros(22)
    L[0:3, 0:3], L[3:6, 3:6] = L_t, L_rot
    h[0:3], h[3:6] = h_t, h_rot
    return dict(L_pose=L, h_pose=h, L_trans=L_t, h_trans=h_t, L_rot=L_rot, h_rot=h_rot,
                total_weighted_cost=cost_t + cost_r, n_associations=int(N_assoc * K),
                mean_transported_mass=float(np.mean(rmass)), ess_total=float(np.sum(rmass)),
                support_frac=float(N_assoc) / float(max(N_meas, 1)), exact=False)
