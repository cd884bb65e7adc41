#!/bin/bash
# live path host profile (cProfile over the timed calls of tools/live_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/r08d}; mkdir -p "$O"
timeout -k 10 300 python -c "
import cProfile, pstats, sys, io
sys.argv = ['live_bench.py', '30']
sys.path[:0] = ['tools', 'gc-slam_amd', '.']
import live_bench
pr = cProfile.Profile()
pr.enable()
live_bench.main()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(45)
open('$O/profile_tottime.txt', 'w').write(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats('cumulative').print_stats(70)
open('$O/profile_cum.txt', 'w').write(s.getvalue())
" > "$O/live.log" 2>&1
