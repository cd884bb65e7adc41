"""gcslam: MI355X-native (gfx950) GC-SLAM bin-path per-scan backend.

Host-side mirror of the reference operator / pipeline interface
(fl_ws/src/fl_slam_poc/fl_slam_poc/backend/pipeline.py) over the C-ABI library
libgcslam_hip.so (include/gcslam_hip.h).  There is no CPU fallback.
"""

from . import _lib  # noqa: F401

__version__ = "0.1.0"


def library():
    """Load libgcslam_hip.so (raises RuntimeError if missing)."""
    return _lib.load()
