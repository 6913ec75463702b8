"""bench.py's launcher on the CPU: `--gpus N` means N ranks (re-launched under
torch.distributed.run when no launcher set WORLD_SIZE), and a launcher's world size that disagrees
with --gpus is refused.  --dry-run stops after the process group (gloo, no GPU)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, env=e)


def test_gpus_n_relaunches_n_ranks():
    r = _bench("--gpus", "2", "--no-other-configs", "--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0]) == {"dry_run": True, "n_gpus": 2}, r.stdout


def test_gpus_one_is_one_rank():
    r = _bench("--dry-run")
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_gpus_disagreeing_with_launcher_is_refused():
    r = _bench("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
