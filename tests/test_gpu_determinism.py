"""Run-to-run determinism of the whole node loop on the GPU (docs/GC_SLAM.md:1150: the backend is
deterministic), beyond one scan on an empty map:

* fresh contexts run the same scale-mode scan sequence -- populated map, the hypothesis combine and
  the IW applies after every scan -- and must agree bit for bit after every scan: z_t, the belief,
  the certificates, and checksums of the device state the next scan reads (ScanBinStats, map,
  derived stats, touched bytes, both active-flag buffers, the bin kernel's persistent partial rows,
  the device scalar block and the host mirror the tail reads);
* the scan mirror's guard (gcs_layout.h Mirror): with the PT fold's data stores held back behind its
  sequence word (GCS_DEBUG_MIRROR_TORN) the host must re-read until the checksum matches and return
  the same results as the ordinary hand-off.

The sequence is the trajectory test's (B = 5,000, N = 4,096, 12 scans), in which round 4 saw one
run-to-run drift.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from golden_util import ORIGIN
from gcslam.synthetic import scan_kwargs

pytestmark = pytest.mark.gpu

N_SCANS = 12


def _run(n_bins, cap, n_pts, n_scans, torn_us=0, checksums=True):
    from gcslam import _lib as L
    from gcslam import synthetic
    from gcslam.context import HypothesisContext
    from gcslam.distributed import combine_allreduce
    ctx = HypothesisContext(n_bins=n_bins, n_points_cap=cap, max_raw_points=n_pts, mode="scale",
                            lidar_origin=tuple(ORIGIN))
    if torn_us:
        ctx.set_debug(L.DEBUG_MIRROR_TORN, torn_us)
    seq = []
    try:
        for s in range(n_scans):
            sc = synthetic.make_scan(n_pts, s)
            rec = torch.from_numpy(sc["xyz_record"]).cuda()
            t = torch.from_numpy(sc["timestamps"]).cuda()
            w = torch.from_numpy(sc["weights"]).cuda()
            out = ctx.scan(rec, 16, t, w, n_pts, **scan_kwargs(sc))
            row = [np.array(out.z_t[:]), np.array(out.belief.L[:]), np.array(out.belief.h[:]),
                   np.array(out.cert[:]), np.array(out.iw_process_dPsi[:])]
            combine_allreduce(ctx, 0, 1, s, want_belief=False)
            if checksums:
                row.append(np.array(ctx.state_checksums(), np.uint64))
            seq.append(row)
        stats = ctx.mirror_stats()
    finally:
        ctx.close()
    return seq, stats


def _first_difference(a, b):
    names = ["z_t", "belief.L", "belief.h", "cert", "iw_process_dPsi", "state checksums"]
    for s, (ra, rb) in enumerate(zip(a, b)):
        for k, (x, y) in enumerate(zip(ra, rb)):
            if x.tobytes() != y.tobytes():
                return f"scan {s}: {names[k]}" + (f" component {np.flatnonzero(x != y).tolist()}" if k == 5 else "")
    return None


def test_scan_sequence_bitwise_across_contexts():
    """Four fresh contexts, 12 scans each with the combine: every per-scan output and every device
    state checksum bitwise equal; every scan's mirror accepted (none through the sync fallback)."""
    runs = [_run(5000, 4096, 4096, N_SCANS) for _ in range(4)]
    for r, (seq, stats) in enumerate(runs):
        assert stats[0] == N_SCANS, stats
        assert stats[2] == 0, f"mirror accepted only after a stream synchronize: {stats}"
        if r:
            diff = _first_difference(runs[0][0], seq)
            assert diff is None, f"run {r} differs from run 0 first at {diff}"


def test_scan_sequence_bitwise_c2_shape():
    """The benchmark's shape (65,536 points, 100,000 bins: 64-bin tiles, direct buckets): two fresh
    contexts, six scans with the combine, bitwise equal including the state checksums."""
    a, _ = _run(100_000, 65536, 65536, 6)
    b, _ = _run(100_000, 65536, 65536, 6)
    assert _first_difference(a, b) is None, _first_difference(a, b)


def test_scan_sequence_bitwise_c3_shape():
    """The north-star shape (262,144 points, 1,048,576 bins: 128-bin tiles, two finalizing waves): four
    fresh contexts, three scans each, bitwise equal including the ScanBinStats checksum -- the round-6
    race (a tile's dirty word cleared by wave 0 before wave 1 read it: wave 1 took the clean-tile exit and
    left its 64 bins' rows unwritten) showed here in 6 of 9 runs."""
    runs = [_run(1_048_576, 262_144, 262_144, 3)[0] for _ in range(4)]
    for r in range(1, 4):
        diff = _first_difference(runs[0], runs[r])
        assert diff is None, f"run {r} differs from run 0 first at {diff}"


def test_torn_mirror_is_reread_not_consumed():
    """The PT fold stores the mirror's sequence word and checksum 300 us before its data: the host sees
    a mirror of the right scan whose data have not arrived, must re-read it until the checksum
    matches, and must return exactly the ordinary hand-off's results."""
    ref, _ = _run(5000, 4096, 4096, 4, checksums=False)
    torn, stats = _run(5000, 4096, 4096, 4, torn_us=300, checksums=False)
    assert _first_difference(ref, torn) is None, _first_difference(ref, torn)
    assert stats[0] == 4 and stats[1] >= 1, stats
