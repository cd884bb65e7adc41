"""gcslam.topology on a synthetic sysfs tree: the HIP-free GPU count bench.py's launcher uses, the
visibility variables, and the NUMA-local CPU share each rank pins itself to (an 8-GPU node with two
sockets: GPUs 0-3 on CPUs 0-63, GPUs 4-7 on CPUs 64-127)."""

import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gc-slam_amd"))
from gcslam import topology as T  # noqa: E402


def _fake_sysfs(root, n_gpus=8, numa_file=False):
    nodes = os.path.join(root, "class", "kfd", "kfd", "topology", "nodes")
    # two CPU nodes first (simd_count 0), then the GPUs, as KFD lists them
    props = ["cpu_cores_count 64\nsimd_count 0\n"] * 2
    for g in range(n_gpus):
        bus = 0x11 + 0x20 * g
        props.append(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        pci = os.path.join(root, "bus", "pci", "devices", f"0000:{bus:02x}:00.0")
        os.makedirs(pci)
        if numa_file:
            open(os.path.join(pci, "numa_node"), "w").write(f"{g // 4}\n")
        else:
            open(os.path.join(pci, "local_cpulist"), "w").write("0-63\n" if g < 4 else "64-127\n")
    for i, p in enumerate(props):
        os.makedirs(os.path.join(nodes, str(i)))
        open(os.path.join(nodes, str(i), "properties"), "w").write(p)
    for k in range(2):
        d = os.path.join(root, "devices", "system", "node", f"node{k}")
        os.makedirs(d)
        open(os.path.join(d, "cpulist"), "w").write(f"{64 * k}-{64 * k + 63}\n")
    return root


@pytest.fixture
def clean_env(monkeypatch):
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    return monkeypatch


def test_parse_and_format_cpulists():
    assert T.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert T.parse_cpulist("") == []
    assert T._fmt([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"


def test_gpu_count_without_kfd_is_none(tmp_path, clean_env):
    assert T.visible_gpu_count(str(tmp_path)) is None


def test_gpu_count_and_visibility(tmp_path, clean_env):
    root = _fake_sysfs(str(tmp_path))
    assert T.visible_gpu_count(root) == 8
    clean_env.setenv("HIP_VISIBLE_DEVICES", "6,2")
    g = T.visible_gpus(root)
    assert [x["node"] for x in g] == [8, 4]  # CPU nodes 0-1, GPU k = node k + 2
    clean_env.setenv("ROCR_VISIBLE_DEVICES", "4,5,6,7")
    clean_env.setenv("HIP_VISIBLE_DEVICES", "1")
    assert [x["node"] for x in T.visible_gpus(root)] == [7]
    clean_env.setenv("HIP_VISIBLE_DEVICES", "")
    assert T.visible_gpu_count(root) == 0


@pytest.mark.parametrize("numa_file", [False, True])
def test_rank_cpus_split_the_socket_between_its_gpus(tmp_path, clean_env, numa_file):
    root = _fake_sysfs(str(tmp_path), numa_file=numa_file)
    allowed = list(range(128))
    shares = [T.rank_cpus(r, 8, allowed, root)[0] for r in range(8)]
    assert shares[0] == list(range(0, 16)) and shares[3] == list(range(48, 64))
    assert shares[4] == list(range(64, 80)) and shares[7] == list(range(112, 128))
    assert len(set().union(*map(set, shares))) == 128  # disjoint, covering
    # fewer ranks than GPUs: two ranks on GPUs 0 and 1 share socket 0
    assert T.rank_cpus(1, 2, allowed, root)[0] == list(range(32, 64))
    # a restricted allowed set (a cgroup share): only its CPUs near the GPU
    cpus, how = T.rank_cpus(0, 1, list(range(56, 72)), root)
    assert cpus == list(range(56, 64)) and how.startswith("numa-local")


def test_rank_cpus_without_topology_split_the_allowed_set(tmp_path, clean_env):
    cpus, how = T.rank_cpus(2, 4, list(range(8)), str(tmp_path))
    assert cpus == [4, 5] and "no topology" in how
    assert T.rank_cpus(0, 1, list(range(8)), str(tmp_path))[0] == list(range(8))
