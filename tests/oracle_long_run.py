# The numpy oracle over bench.py's cycled sequence (8 synthetic scans, C2 size, no restart) -- the
# reference restatement's own divergence (profiles/r06/longrun/oracle_cycled_c2.txt); test infrastructure,
# like tools/long_run.py for the library (kept under tests/: only tests may run the oracle).
# Usage: python tests/oracle_long_run.py N_SCANS
import sys, time, json
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gc-slam_amd')]
import numpy as np
from threadpoolctl import threadpool_limits
from gcslam import synthetic
from oracle import ops, pipeline as opipe
N, B = 65536, 100000
with threadpool_limits(4):
    bins = ops.fibonacci_atlas(B)
    knn = ops.bin_knn_table(bins, 16)
    pc = opipe.BinPathConfig(n_points_cap=N, n_bins=B, mode="scale", lidar_origin=tuple(synthetic.LIDAR_ORIGIN))
    b = ops.Belief.identity_prior()
    Q = ops.process_noise_Q(*ops.datasheet_process_noise_state())
    ms = opipe.MapState.empty(B)
    scans = [synthetic.make_scan(N, k) for k in range(8)]
    t0 = time.time()
    for n in range(int(sys.argv[1])):
        r = opipe.process_scan_bin_path(b, scans[n % 8], Q, pc, bins, knn, ms)
        b, ms = r["belief"], r["map"]
        if n % 10 == 0 or n > 95:
            print(n, [float('%.3g' % x) for x in r["z_t"]], round(time.time() - t0, 1), flush=True)
