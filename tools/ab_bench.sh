#!/bin/bash
# Same-box A/B of bench.py argument / environment variants, alternated REPS times (C2, short runs).
#   VARIANTS="name|ENV=V ENV2=V|--bench-args ;; name2|...|..."  O=gpurun_out/x  REPS=2  STEPS=100
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${O:-gpurun_out/ab}; REPS=${REPS:-2}; STEPS=${STEPS:-100}
mkdir -p "$O"
IFS=';;' read -r -a VS <<< "$VARIANTS"
for r in $(seq 1 "$REPS"); do
  for v in "${VS[@]}"; do
    [ -z "${v// }" ] && continue
    name=$(echo "$v" | cut -d'|' -f1 | xargs); envs=$(echo "$v" | cut -d'|' -f2); args=$(echo "$v" | cut -d'|' -f3)
    echo "[ab] $r $name" >&2
    env $envs timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 10 --no-cpu-baseline --no-c3 --no-live $args \
      > "$O/${name}_$r.log" 2>&1 || exit $?
  done
done
python3 - "$O" <<'PY'
import glob, json, os, sys
o = sys.argv[1]
rows = {}
for f in sorted(glob.glob(os.path.join(o, "*.log"))):
    name = os.path.basename(f)[:-4]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            rows[name] = (d["ms_per_step"], d["step_ms"]["median"], d["roofline"].get("kernel_us"),
                          d["per_rank"][0]["combine_ms"]["median"], d.get("mirror", {}))
for k, v in rows.items():
    print(f"{k:24s} ms/step {v[0]:.4f} median {v[1]:.4f} bins_us {v[2]} combine_med {v[3]:.4f} mirror {v[4].get('scan_rereads')},{v[4].get('allreduce_rereads')}")
PY
