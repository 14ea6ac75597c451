"""bench.py's own N-rank launcher on the GPU (VERDICT r05 "Next round" 1): the plain command
`python3 bench.py --gpus 2 ...`, with no torch.distributed.run around it, must measure two ranks.
Both ranks share the box's one GPU (--share-gpu) and exchange their write segments over gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--share-gpu", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--deadline", "240"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["config"]["parallelism"] == "replicas2"
    assert res["value"] > 0 and res["steps"] == 5
    assert res["amdahl"]["predicted_speedup_vs_1gpu"] == pytest.approx(2 * 1.1 / 1.3, abs=1e-3)
