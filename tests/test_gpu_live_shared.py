"""The live primitive map shared across hypotheses on separate ranks (bench.py --path primitive
--map-mode shared): rank 0 updates the node map and broadcasts each scan's update record
(gcslam.distributed.MapRecordChannel), rank 1 scans with update_map=False on its copy and replays the
record (primitive_map_follow), the reference's one map, hypothesis 0's (backend_node.py:2036-2083).
Two ranks share the one GPU here (gloo transport; RCCL takes one GPU per rank): after the run the
follower's map is bitwise the lead's."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_share_the_live_map_bitwise():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--path", "primitive", "--map-mode", "shared",
                        "--gpus", "2", "--share-device", "--steps", "4", "--warmup", "2"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["config"]["hypotheses"] == 2 and d["config"]["map_mode"] == "shared"
    assert d["map_bitwise_equal"] is True
    ranks = d["per_rank"]
    assert ranks[0]["map_primitives"] == ranks[1]["map_primitives"] > 0
    assert ranks[1]["follow_ms"] is not None and 0.4e6 < d["record_bytes"] < 0.7e6
