"""bench.py's multi-rank launcher on CPU (gloo): `bench.py --gpus N` without a launcher's WORLD_SIZE
starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), before any
GPU call, and exits with their status.  `--cpu-rehearsal` runs each rank's per-scan exchange (library
payload pack, gloo sum, library apply: backend_node.py:1999-2002,2085-2119, hypothesis.py:83-99) so
the test sees both ranks run and the summed payload equal the sum of the ranks' own payloads.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # rank 0 alone prints the JSON line
    return json.loads(lines[0])


def test_launcher_spawns_two_gloo_ranks_and_payload_sums_match():
    r = _run(["--cpu-rehearsal", "--gpus", "2", "--steps", "6", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["rehearsal"] and d["transport"] == "gloo"
    ranks = d["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert ranks[0]["pid"] != ranks[1]["pid"]  # two processes, not one
    assert d["payload_sum_check"] and d["payload_sum_max_abs_err"] == 0.0
    assert ranks[0]["Q_sum"] == ranks[1]["Q_sum"]  # the applied sum gives every rank the same Q


@pytest.mark.parametrize("map_mode", ["own", "shared"])
def test_launcher_eight_gloo_ranks(map_mode):
    """The C4 layout (8 hypotheses, one rank each) rehearsed on CPU: eight processes, each pinned
    to its share of the job's CPUs, the summed payload equal to the sum of the eight payloads, every
    rank applying the same Q, and (shared map) the lead's record reaching every rank bit for bit."""
    r = _run(["--cpu-rehearsal", "--gpus", "8", "--map-mode", map_mode, "--steps", "4", "--warmup", "1"], timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 8 and d["transport"] == "gloo"
    ranks = d["ranks"]
    assert [x["rank"] for x in ranks] == list(range(8))
    assert len({x["pid"] for x in ranks}) == 8
    assert d["payload_sum_check"]
    assert len({x["Q_sum"] for x in ranks}) == 1
    if map_mode == "shared":
        assert all(x["map_record_ok"] for x in ranks)
    # each rank pinned itself (or says why not); with >= 16 CPUs the shares are disjoint
    aff = [x["affinity"] for x in ranks]
    assert all("how" in a for a in aff)
    if len(os.sched_getaffinity(0)) >= 16:
        sets = [set(_cpus(a["cpus"])) for a in aff]
        assert sum(len(s) for s in sets) == len(set().union(*sets))


def _cpus(s):
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def test_single_rank_rehearsal_is_unchanged():
    r = _run(["--cpu-rehearsal", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["ranks"] == [0]


def test_launcher_fails_when_more_gpus_than_visible():
    r = _run(["--gpus", "64", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "visible GPU" in r.stderr


def test_launcher_world_mismatch_fails():
    r = _run(["--cpu-rehearsal", "--gpus", "2", "--steps", "1"], env_extra={"WORLD_SIZE": "1", "RANK": "0",
                                                                           "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_shared_map_record_rides_the_payload_to_every_rank():
    """--map-mode shared: the lead's (rank 0) map-update record is appended to the payload and the
    followers add zeros, so after the sum every rank holds the lead's record bit for bit
    (gcslam_hip.h GCS_MAP_FOLLOW; backend_node.py:2079-2083)."""
    r = _run(["--cpu-rehearsal", "--gpus", "2", "--map-mode", "shared", "--steps", "4", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert [x["map_record_ok"] for x in d["ranks"]] == [True, True]
    assert d["payload_sum_check"]
