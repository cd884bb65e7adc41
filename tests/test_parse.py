"""PointCloud2 parse: parse_pointcloud2_vlp16 (backend_node.py:377-468) +
the base transform (:1677-1680).  CPU: the oracle restatement on known answers.  GPU: the device
parse (gcs_parse_pointcloud2) against the oracle on messages with non-finite coordinates, several
time-field types and unaligned layouts, and a scan fed from the parse against the oracle pipeline."""

import math

import numpy as np
import pytest

from oracle import ops
from gcslam.synthetic import scan_kwargs

F32, F64, U16, U32 = 7, 8, 4, 6
NP = {F32: "<f4", F64: "<f8", U16: "<u2", U32: "<u4"}


def make_msg(xyz, ring, t=None, t_type=F32, step=None, layout="vlp16"):
    """Pack a PointCloud2-like byte buffer.  layout 'vlp16': x y z intensity ring t (aligned);
    'odd': a 3-byte pad before x and an unaligned ring / t (point_step 23 + t)."""
    n = xyz.shape[0]
    if layout == "vlp16":
        offs = dict(x=0, y=4, z=8, intensity=12, ring=16)
        tt = 18 if t is not None else None
        size = 18 + (np.dtype(NP[t_type]).itemsize if t is not None else 0)
    else:
        offs = dict(x=3, y=7, z=11, ring=15)
        tt = 17 if t is not None else None
        size = 17 + (np.dtype(NP[t_type]).itemsize if t is not None else 0) + 2
    step = step or size
    names, fmts, offsets = ["x", "y", "z", "ring"], ["<f4", "<f4", "<f4", "<u2"], [offs["x"], offs["y"], offs["z"], offs["ring"]]
    if t is not None:
        names.append("t"); fmts.append(NP[t_type]); offsets.append(tt)
    arr = np.zeros(n, dtype=np.dtype({"names": names, "formats": fmts, "offsets": offsets, "itemsize": step}))
    arr["x"], arr["y"], arr["z"], arr["ring"] = xyz[:, 0], xyz[:, 1], xyz[:, 2], ring
    if t is not None:
        arr["t"] = t
    fields = {k: (o, {"<f4": F32, "<f8": F64, "<u2": U16, "<u4": U32}[f]) for k, f, o in zip(names, fmts, offsets)}
    return arr.tobytes(), fields, step


def _cloud(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = rng.uniform(0.1, 80.0, n)
    xyz = (d * r[:, None]).astype(np.float32)
    xyz[::97, 0] = np.nan
    xyz[5::101, 1] = np.inf
    xyz[7::103, 2] = -np.inf
    return xyz, (np.arange(n) % 16).astype(np.uint16)


# ------------------------------------------------------------------ CPU: the oracle restatement
def test_oracle_parse_known_answers():
    xyz = np.array([[np.nan, 0.0, 0.0], [np.inf, -np.inf, 1.0], [0.5, 0.0, 0.0], [3.0, 4.0, 0.0]], np.float32)
    data, fields, step = make_msg(xyz, np.array([1, 2, 300, 4], np.uint16), t=np.array([1e9, 2e9, 3e9, 4e9]),
                                  t_type=U32)
    p, t, w, ring, tag = ops.parse_pointcloud2_vlp16(data, fields, step, 4, 7.0)
    assert p[0, 0] == 1e6 and p[1, 0] == 1e6 and p[1, 1] == -1e6                 # non-finite sentinel
    assert np.array_equal(t, np.array([1.0, 2.0, 3.0, 4.0]))                     # ns -> s (any > 1e6)
    assert np.array_equal(ring, np.array([1, 2, 44, 4], np.uint8))              # astype(uint8) wraps
    assert np.all(tag == 0)
    # range 0.5 m: w_min = 1/2, w_max = sigmoid(198) = 1 -> w = 0.5 (1 - 1e-12) + 1e-12
    assert w[2] == pytest.approx(0.5 * (1 - 1e-12) + 1e-12, rel=1e-15)
    assert w[3] == pytest.approx(1.0 / (1.0 + math.exp(-18.0)), rel=1e-15)       # range 5 m
    _, t2, _, _, _ = ops.parse_pointcloud2_vlp16(*make_msg(xyz, np.zeros(4, np.uint16))[:1],
                                                 make_msg(xyz, np.zeros(4, np.uint16))[1], step - 4, 4, 7.0)
    assert np.all(t2 == 7.0)                                                      # no time field: header stamp
    with pytest.raises(RuntimeError):
        ops.parse_pointcloud2_vlp16(data, {k: v for k, v in fields.items() if k != "ring"}, step, 4, 0.0)


def test_oracle_base_transform():
    p = np.array([[1.0, 2.0, 3.0]])
    R = np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    assert np.allclose(ops.lidar_to_base(p, R, [0.1, 0.2, 0.3]), [[-1.9, 1.2, 3.3]], atol=1e-15)


# ------------------------------------------------------------------ GPU: device parse vs oracle
def _msg_obj(data, fields, step, n, stamp):
    from gcslam.parse import PointCloud2Like, PointFieldLike
    return PointCloud2Like(data=data, fields=[PointFieldLike(k, o, d) for k, (o, d) in fields.items()], point_step=step,
                           width=n, stamp_sec=stamp)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["f32_s", "f64_ns", "u32_ns", "none", "odd_f32"])
def test_gpu_parse_matches_oracle(case):
    from gcslam.context import HypothesisContext
    from gcslam.parse import parse_pointcloud2_vlp16
    n = 20000
    xyz, ring = _cloud(n, 3)
    t = {"f32_s": (np.linspace(0.0, 0.1, n).astype(np.float32), F32),
         "f64_ns": (1.7e18 + np.arange(n) * 5000.0, F64),
         "u32_ns": ((np.arange(n) * 4999) % 2**32, U32),
         "none": (None, F32),
         "odd_f32": (np.linspace(100.0, 100.1, n).astype(np.float32), F32)}[case]
    data, fields, step = make_msg(xyz, ring, t=t[0], t_type=t[1], layout="odd" if case.startswith("odd") else "vlp16")
    ang = 0.3
    R = np.array([[math.cos(ang), -math.sin(ang), 0.0], [math.sin(ang), math.cos(ang), 0.0], [0.0, 0.0, 1.0]])
    tb = np.array([0.1, -0.2, 0.5])
    ctx = HypothesisContext(n_bins=48, n_points_cap=1024, mode="dense", max_raw_points=n)
    pts, tt, w, rg, tag = parse_pointcloud2_vlp16(_msg_obj(data, fields, step, n, 42.5), ctx, R, tb)
    p_ref, t_ref, w_ref, ring_ref, _ = ops.parse_pointcloud2_vlp16(data, fields, step, n, 42.5)
    assert np.array_equal(tt.cpu().numpy(), t_ref)                          # bit-exact times
    assert np.array_equal(rg.cpu().numpy(), ring_ref)
    np.testing.assert_allclose(w.cpu().numpy(), w_ref, rtol=2e-16 * 8, atol=0)
    pb = ops.lidar_to_base(p_ref, R, tb)
    np.testing.assert_allclose(pts.cpu().numpy(), pb, rtol=1e-15, atol=1e-15 * np.abs(pb).max())
    assert int(tag.sum().item()) == 0
    ctx.close()


@pytest.mark.gpu
def test_gpu_scan_from_parsed_cloud_matches_oracle():
    """The 14-step scan fed by the device parse (f64 base-frame points) against the oracle pipeline
    fed by the oracle parse + base transform (dense B=48, two scans)."""
    import torch
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.parse import parse_pointcloud2_vlp16
    from oracle import pipeline as opipe
    origin = (0.0, 0.0, 0.5)
    ctx = HypothesisContext(n_bins=48, n_points_cap=2048, mode="dense", lidar_origin=origin, max_raw_points=4096)
    dirs, knn = ctx.atlas()
    cfg = opipe.BinPathConfig(n_points_cap=2048, n_bins=48, mode="dense", lidar_origin=origin, tau=ctx.cfg.tau)
    b = ops.Belief.identity_prior()
    nu, Psi = ops.datasheet_process_noise_state()
    Q = ops.process_noise_Q(nu, Psi)
    ms = opipe.MapState.empty(48)
    tb = np.array([0.0, 0.0, 0.05])
    for k in range(2):
        sc = synthetic.make_scan(4096, 40 + k)
        xyz = sc["xyz_record"][:, :3]
        data, fields, step = make_msg(xyz, np.zeros(4096, np.uint16), t=sc["timestamps"], t_type=F64)
        pts, t, w, _, _ = parse_pointcloud2_vlp16(_msg_obj(data, fields, step, 4096, 0.0), ctx, np.eye(3), tb)
        p_ref, t_ref, w_ref, _, _ = ops.parse_pointcloud2_vlp16(data, fields, step, 4096, 0.0)
        sref = dict(sc, points=ops.lidar_to_base(p_ref, np.eye(3), tb), timestamps=t_ref, weights=w_ref)
        ref = opipe.process_scan_bin_path(b, sref, Q, cfg, dirs, knn, ms)
        out = ctx.scan(pts, 24, t, w, 4096, **scan_kwargs(sc), Q=Q,
                       xyz_f64=True)
        np.testing.assert_allclose(np.array(out.z_t[:]), ref["z_t"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(ctx.get_scan_stats()[0], ref["scan_bins"]["N"], rtol=1e-11, atol=1e-14)
        b, ms = ref["belief"], ref["map"]
    ctx.close()
