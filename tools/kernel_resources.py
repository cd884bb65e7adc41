#!/usr/bin/env python3
"""Per-kernel code-object resources of the built library (VGPR, AGPR, SGPR, spills, private segment,
LDS, and the waves per SIMD the registers allow), read from the AMDGPU metadata notes of the gfx950
code objects inside gc-slam_amd/build/*.o (the objects libgcslam_hip.so links).

  python tools/kernel_resources.py [--json out.json] [--md out.md]

Each object's .hip_fatbin section is a clang offload bundle; its gfx950 code object carries the
metadata the loader uses (`llvm-readelf --notes`).  Waves per SIMD from registers follow
MI355X_MICROARCH.md "Register files": the allocation granule is 8 registers per lane over the unified
512-entry VGPR+AGPR file, min(8, 512 // alloc)."""

import argparse
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def kernels_of(obj):
    with tempfile.TemporaryDirectory() as d:
        bundle, co = os.path.join(d, "b"), os.path.join(d, "co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={bundle}", obj, os.path.join(d, "o")],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={bundle}", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    ks, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*(-\s+)?\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1):  # a new kernel map
            cur = {}
            ks.append(cur)
        if cur is not None:
            cur[m.group(2)] = m.group(3)
    out = []
    for k in ks:
        if "name" not in k or "vgpr_count" not in k:
            continue
        m = re.search(r"target_archE(\d+)", k["name"])
        if m and m.group(1) != "950":  # rocPRIM's dispatch stubs for other targets (never launched here)
            continue
        v, a = int(k["vgpr_count"]), int(k.get("agpr_count", 0))
        alloc = -(-(v + a) // 8) * 8
        out.append(dict(name=k["name"], object=os.path.basename(obj), vgpr=v, agpr=a, sgpr=int(k.get("sgpr_count", 0)),
                        vgpr_spill=int(k.get("vgpr_spill_count", 0)), sgpr_spill=int(k.get("sgpr_spill_count", 0)),
                        private_bytes=int(k.get("private_segment_fixed_size", 0)),
                        lds_bytes=int(k.get("group_segment_fixed_size", 0)),
                        max_threads=int(k.get("max_flat_workgroup_size", 0)),
                        waves_per_simd_regs=min(8, 512 // max(alloc, 8))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--md")
    args = ap.parse_args()
    rows = []
    for obj in sorted(glob.glob(os.path.join(ROOT, "gc-slam_amd", "build", "*.o"))):
        try:
            rows.extend(kernels_of(obj))
        except subprocess.CalledProcessError:  # a host-only object: no device code
            continue
    for r, dn in zip(rows, demangle([r["name"] for r in rows])):
        r["kernel"] = dn.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    if args.json:
        json.dump(rows, open(args.json, "w"), indent=1)
    lines = ["| kernel | VGPR | AGPR | SGPR | spill (V/S) | private B/lane | LDS B | waves/SIMD (regs) |",
             "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{r['kernel']}` | {r['vgpr']} | {r['agpr']} | {r['sgpr']} | {r['vgpr_spill']}/{r['sgpr_spill']} | "
                     f"{r['private_bytes']} | {r['lds_bytes']} | {r['waves_per_simd_regs']} |")
    text = "\n".join(lines) + "\n"
    if args.md:
        open(args.md, "w").write(text)
    else:
        sys.stdout.write(text)


if __name__ == "__main__":
    main()
