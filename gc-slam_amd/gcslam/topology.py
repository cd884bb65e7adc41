"""GPU and CPU topology for the one-process-per-GPU launch, read from sysfs without initialising HIP.

`bench.py --gpus N` starts its rank processes itself, and each rank pins itself to its GPU's
NUMA-local host cores before its first GPU call (the per-scan host work -- the 22-D prologue and
tail, the context's launch worker, the polled ready word -- then runs next to its GPU's memory and
PCIe root).  Neither step may touch HIP in the launching process: an initialised HIP runtime must
not fork or exec (the pool's rule), and `torch.cuda.device_count()` falls back to hipGetDeviceCount
when amdsmi fails.  So both read the KFD topology the ROCr runtime itself enumerates:

  /sys/class/kfd/kfd/topology/nodes/<n>/properties   simd_count > 0 marks a GPU node, in HIP's
                                                      device order; location_id = bus << 8 | dev << 3 | fn,
                                                      domain = PCI domain
  /sys/bus/pci/devices/<dddd:bb:dd.f>/local_cpulist   the GPU's NUMA-local CPUs
  /sys/bus/pci/devices/<...>/numa_node                (fallback: /sys/devices/system/node/node<k>/cpulist)

HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES select and reorder the GPU nodes
the way the runtime does (ROCR first, then HIP / CUDA on top of it).
"""

from __future__ import annotations

import os

SYSFS = "/sys"


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in (text or "").strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def _props(text: str) -> dict:
    d = {}
    for line in (text or "").splitlines():
        kv = line.split()
        if len(kv) == 2:
            try:
                d[kv[0]] = int(kv[1])
            except ValueError:
                pass
    return d


def kfd_gpu_nodes(sysfs: str = SYSFS) -> list[dict] | None:
    """The KFD topology's GPU nodes in node order (HIP's enumeration order), or None without KFD."""
    root = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        names = sorted((n for n in os.listdir(root) if n.isdigit()), key=int)
    except OSError:
        return None
    gpus = []
    for n in names:
        p = _props(_read(os.path.join(root, n, "properties")))
        if p.get("simd_count", 0) > 0:
            p["node"] = int(n)
            gpus.append(p)
    return gpus


def _visible(env_names, n):
    """Apply one visibility variable (the first one set) to n devices: the selected indices."""
    for name in env_names:
        v = os.environ.get(name)
        if v is None:
            continue
        v = v.strip()
        if v == "":
            return []
        idx = []
        for tok in v.split(","):
            tok = tok.strip()
            if not tok.isdigit():  # UUIDs etc.: not resolvable here; keep the count only
                return list(range(min(n, len(v.split(",")))))
            i = int(tok)
            if i >= n or i in idx:
                break  # the runtime stops at the first invalid index
            idx.append(i)
        return idx
    return list(range(n))


def visible_gpus(sysfs: str = SYSFS) -> list[dict] | None:
    """The GPU nodes this process's HIP runtime would enumerate, in device order (None without KFD)."""
    nodes = kfd_gpu_nodes(sysfs)
    if nodes is None:
        return None
    sel = _visible(("ROCR_VISIBLE_DEVICES",), len(nodes))
    nodes = [nodes[i] for i in sel]
    sel = _visible(("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"), len(nodes))
    return [nodes[i] for i in sel]


def visible_gpu_count(sysfs: str = SYSFS) -> int | None:
    g = visible_gpus(sysfs)
    return None if g is None else len(g)


def _pci_name(node: dict) -> str | None:
    loc = node.get("location_id")
    if loc is None:
        return None
    dom = node.get("domain", 0)
    return f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}"


def gpu_local_cpus(device: int, sysfs: str = SYSFS) -> list[int] | None:
    """NUMA-local host CPUs of visible GPU `device` (None when the topology does not say)."""
    gpus = visible_gpus(sysfs)
    if not gpus or device >= len(gpus):
        return None
    name = _pci_name(gpus[device])
    if name is None:
        return None
    dev = os.path.join(sysfs, "bus", "pci", "devices", name)
    cpus = parse_cpulist(_read(os.path.join(dev, "local_cpulist")) or "")
    if cpus:
        return cpus
    numa = (_read(os.path.join(dev, "numa_node")) or "").strip()
    if numa.lstrip("-").isdigit() and int(numa) >= 0:
        cpus = parse_cpulist(_read(os.path.join(sysfs, "devices", "system", "node", f"node{int(numa)}", "cpulist")) or "")
        return cpus or None
    return None


def rank_cpus(local_rank: int, local_world: int, allowed: list[int], sysfs: str = SYSFS) -> tuple[list[int], str]:
    """The host CPUs rank `local_rank` (on visible GPU `local_rank`) should run on, and how they were
    chosen.  The GPU's NUMA-local CPUs this process may use are split evenly between the ranks whose
    GPUs share that CPU set (a socket serving four GPUs gives each rank a quarter of it); with no
    topology, or no allowed CPU near the GPU, the allowed CPUs are split evenly over all local ranks."""
    allowed = sorted(allowed)
    local = gpu_local_cpus(local_rank, sysfs)
    if local:
        mine = [c for c in local if c in set(allowed)]
        if mine:
            key = tuple(local)
            peers = [r for r in range(local_world) if tuple(gpu_local_cpus(r, sysfs) or ()) == key]
            k, n = peers.index(local_rank), len(peers)
            share = mine[k * len(mine) // n:(k + 1) * len(mine) // n] or mine
            return share, f"numa-local ({len(mine)} allowed CPUs near GPU {local_rank}, 1/{n} share)"
    if local_world <= 1 or len(allowed) < local_world:
        return allowed, "allowed (no topology)"
    k, n = local_rank, local_world
    return allowed[k * len(allowed) // n:(k + 1) * len(allowed) // n], "allowed split (no topology)"


def pin_rank(local_rank: int, local_world: int, sysfs: str = SYSFS) -> dict:
    """Pin this process to rank_cpus(...) (os.sched_setaffinity; call before any GPU work: threads
    created later -- the HIP runtime's, the library's worker -- inherit the mask)."""
    allowed = sorted(os.sched_getaffinity(0))
    cpus, how = rank_cpus(local_rank, local_world, allowed, sysfs)
    if len(cpus) < min(2, len(allowed)):  # the main thread and the context's launch worker need two
        return dict(cpus=_fmt(allowed), n_cpus=len(allowed), how=f"unpinned (share {_fmt(cpus)} too small)")
    try:
        os.sched_setaffinity(0, set(cpus))
    except OSError as e:
        return dict(cpus=_fmt(allowed), n_cpus=len(allowed), how=f"unpinned ({e})")
    return dict(cpus=_fmt(cpus), n_cpus=len(cpus), how=how)


def _fmt(cpus):
    """[0, 1, 2, 5] -> '0-2,5'."""
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)
