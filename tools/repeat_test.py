"""Run one GPU test function N times in one process (a flaky-vs-deterministic check of a parity failure):
    python tools/repeat_test.py tests/test_gpu_fullsize.py test_c3_full_scans_value_parity 2"""
import importlib.util
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "gc-slam_amd")]
path, name, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
spec = importlib.util.spec_from_file_location("t", os.path.join(ROOT, path))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
fails = 0
for i in range(n):
    try:
        getattr(mod, name)()
        print(f"run {i}: pass", flush=True)
    except AssertionError as e:
        fails += 1
        print(f"run {i}: FAIL {str(e)[:300]}", flush=True)
    except Exception:
        fails += 1
        traceback.print_exc()
print(f"{n - fails}/{n} passed", flush=True)
