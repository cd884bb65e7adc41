#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (`tools/gpu.sh pmc`) into per-kernel HBM bytes per launch and write
profiles/pmc_bins_<cfg>.json for bench.py's roofline.traffic.

Correction (MI355X_MICROARCH.md, section HBM): FETCH_SIZE and WRITE_SIZE are reported in KiB;
on gfx950 FETCH_SIZE counts one half of the bytes of a 16-B-per-lane coalesced streaming read, so
the read bytes are FETCH_SIZE x 2.  WRITE_SIZE is exact for 16-B-per-lane streaming stores.

Usage: python tools/pmc_summary.py gpurun_out/pmc [c2 c3]   (PMC_ROUND=r02 labels the round)
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path_glob, counter):
    per = defaultdict(list)
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                per[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    cfgs = sys.argv[2:] or ["c2", "c3"]
    for cfg in cfgs:
        fdir = f"{cfg}_FETCH_SIZE" if os.path.isdir(os.path.join(base, f"{cfg}_FETCH_SIZE")) else f"{cfg}_fetch"
        wdir = f"{cfg}_WRITE_SIZE" if os.path.isdir(os.path.join(base, f"{cfg}_WRITE_SIZE")) else f"{cfg}_write"
        fetch, nf = load(os.path.join(base, fdir, "**", "*counter_collection.csv"), "FETCH_SIZE")
        write, nw = load(os.path.join(base, wdir, "**", "*counter_collection.csv"), "WRITE_SIZE")
        if not fetch and not write:
            print(f"{cfg}: no counter files under {base}")
            continue
        kernels = {}
        for k in sorted(set(fetch) | set(write)):
            rd = fetch.get(k, 0.0) * 1024.0 * 2.0
            wr = write.get(k, 0.0) * 1024.0
            kernels[k] = {"fetch_size_kib": fetch.get(k), "write_size_kib": write.get(k),
                          "read_bytes_corrected": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                          "launches": [nf.get(k, 0), nw.get(k, 0)]}
        # the roofline kernel: one k_bins_scale instance runs per pass (C2 64-bin tiles, C3 128-bin tiles)
        name = next((k for k in kernels if "k_bins_scale" in k), None)
        bins = kernels.get(name)
        out = {"config": cfg, "round": os.environ.get("PMC_ROUND", "r03"), "kernel": name,
               "hbm_bytes_per_launch": bins["hbm_bytes"] if bins else None,
               "correction": "read = FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of 16-B/lane reads); "
                             "write = WRITE_SIZE KiB x 1024",
               "kernels": kernels}
        path = os.path.join(ROOT, "profiles", f"pmc_bins_{cfg}.json")
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
        print(path)
        for k, v in kernels.items():
            print(f"  {k:40s} read {v['read_bytes_corrected']/1e6:9.2f} MB  write {v['write_bytes']/1e6:9.2f} MB")


if __name__ == "__main__":
    main()
