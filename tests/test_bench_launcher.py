"""bench.py --gpus N starts N ranks by itself (torch.distributed.run as a
child process, before anything touches a GPU).  Checked here without a GPU
through the --dry-run path: every rank joins a gloo group and rank 0 prints
the world it saw."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--dry-run"], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus_2_launches_two_ranks():
    d = _run(2)
    assert d["world"] == 2 and d["gpus_arg"] == 2
    assert sorted(tuple(x) for x in d["ranks"]) == [(0, 0), (1, 1)]


def test_bench_gpus_1_stays_single_process():
    d = _run(1)
    assert d["world"] == 1 and d["ranks"] == [0]
