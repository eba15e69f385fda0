"""bench.py's multi-GPU launcher (the driver runs ``python bench.py --gpus N``): without a torchrun
environment it spawns N ranks itself (train_v6.py:465-468 mp.spawn), they form a process group and
rank 0 prints one JSON line whose n_gpus is the size of that group.  ``--dry-run`` replaces the GPU
workload with a CPU stub over gloo so the launcher, rendezvous, barrier and max-over-ranks timing
run here without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2])
def test_bench_launches_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run", "--steps", "4",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n
    assert rec["steps"] == 4 and rec["warmup"] == 1
    assert rec["config"]["backend"] == ("gloo" if n > 1 else "none")
    assert rec["value"] > 0 and rec["scaling"] == "weak"
