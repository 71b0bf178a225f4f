"""bench.py's launch contract on CPU: `--gpus N` with
no launcher spawns N ranks itself and the line reports the world size the
process group saw; a `--gpus` that disagrees with the launcher's WORLD_SIZE
is refused. `--plumbing` runs the rendezvous, barrier and max-over-ranks
reduction over gloo with no GPU and no combine."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_bench_gpus_n_spawns_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--plumbing"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["world_size_env"] == n, line
    assert line["max_over_ranks"] == n - 1, line


def test_bench_gpus_disagreeing_with_world_size_is_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr, p.stderr


def test_bench_gpus_one_stays_one_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--plumbing"],
                       env=_env(MASTER_ADDR="127.0.0.1", MASTER_PORT="0"),
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1, line
