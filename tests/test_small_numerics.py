"""gcs_small.h's fixed-size PSD projection (shared by the host IMU / odometry branch and its device kernel)
against the host numerics' run-time-n projection, bitwise, over 200,000 random matrices with zero rows
(tools/psd_small_check.cpp, built here with hipcc's host compiler)."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_small_psd_project_equals_host_bitwise(tmp_path):
    exe = str(tmp_path / "psd_small_check")
    src = os.path.join(ROOT, "tools", "psd_small_check.cpp")
    csrc = os.path.join(ROOT, "gc-slam_amd", "csrc")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", csrc, "-I", os.path.join(ROOT, "include"), src,
                    os.path.join(csrc, "gcs_host.cpp"), "-o", exe], check=True, capture_output=True, timeout=300)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    assert out.startswith("bad 0 "), out
