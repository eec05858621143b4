"""bench.py --gpus N without WORLD_SIZE starts N ranks itself (verdict r1:
--gpus was ignored).  CPU check of the launcher: --dry-run joins a gloo group
instead of touching a GPU; rank 0 reports the world size it sees."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=180, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_gpus_2_spawns_two_ranks():
    r = _run("--gpus", "2", "--dry-run")
    assert r == {"dry_run": True, "n_gpus": 2, "requested": 2}


def test_default_is_one_rank():
    assert _run("--dry-run")["n_gpus"] == 1
