"""bench.py's own multi-rank launcher on the GPU box: `python bench.py --gpus 2` with no launcher
environment starts two ranks (gloo here: RCCL needs a GPU per rank, this box has one), they play
their shards and all-gather the record images, and exactly one JSON line comes back with the
all-gather verified byte for byte."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_spawns_two_ranks():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--envs", "256", "--sims", "8", "--steps", "1", "--warmup", "1", "--no-coach",
                        "--spawn-timeout", "240"], env=env, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["allgather_check"] == "ok" and d["dist_backend"] == "gloo"
    assert d["value"] > 0 and d["expansions_per_episode_batch"] > 0
