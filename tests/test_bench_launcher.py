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


def test_pmc_bytes_per_row_calibration():
    """bench.pmc_bytes_per_row: FETCH_SIZE scaled so the calibration launch
    reads its known bytes; WRITE_SIZE taken as is."""
    import bench
    rows, k = 1 << 20, 64
    known = rows * (2 * k * 4 + 5 * 4 + 2 * 4)
    half_kb = known / 2 / 1024          # gfx950 tallies 128-B requests at 64 B
    fetch = [half_kb, half_kb, 1.5 * half_kb, 1.5 * half_kb, half_kb, half_kb]
    write = [rows * 4 / 1024] * 6
    r = bench.pmc_bytes_per_row(fetch, write, rows, k)
    assert abs(r["calibration"]["factor"] - 2.0) < 1e-12
    assert abs(r["hbm_read_bytes_per_row"] - 1.5 * (2 * k * 4 + 28)) < 1e-9
    assert r["hbm_write_bytes_per_row"] == 4.0
    assert abs(r["w_gather_bytes_per_row"] - 0.5 * (2 * k * 4 + 28)) < 1e-9
