"""The drop-in's host-array staging (gcslam.pipeline._as_device_scan): one pinned + device buffer pair
per (device, stream), grown to the largest scan seen -- real LiDAR scans change their point count
almost every scan, and a buffer per count would grow without bound over a long run."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def test_staging_cache_one_entry_per_stream_over_varying_counts():
    from gcslam import pipeline as P
    rng = np.random.default_rng(5)
    P._pinned.clear()
    for n in (5000, 7000, 6000, 12000, 3000, 12000):
        p = rng.normal(size=(n, 3))
        ts = rng.uniform(0.0, 0.1, n)
        ws = rng.uniform(0.5, 1.5, n)
        xyz, t, w = P._as_device_scan(p, ts, ws, 0)
        torch.cuda.synchronize()
        assert xyz.shape == (n, 3) and xyz.dtype == torch.float32
        assert np.array_equal(xyz.cpu().numpy(), p.astype(np.float32))
        assert np.array_equal(t.cpu().numpy(), ts) and np.array_equal(w.cpu().numpy(), ws)
        keys = [k for k in P._pinned if k[0] == "scan"]
        assert len(keys) == 1, keys
    assert P._pinned[keys[0]][0] >= 12000
