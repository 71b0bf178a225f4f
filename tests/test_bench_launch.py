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


def test_collective_child_result_keeps_finished_phases(tmp_path):
    """An overrun costs the running phase's entry, never the line (VERDICT r04
    #1): the parent reads back the phases the child saved, marks the one it was
    stopped in as failed, and adds the child's exit status as an error."""
    import json
    import bench
    path = tmp_path / "child.json"
    path.write_text(json.dumps({"c4_rccl_rs_ag_4gib_fp32": {"rs_ms": 1.0},
                                "phase_wall_s": {"c4_rccl_rs_ag_4gib_fp32": 3.0},
                                "running": "c4_oneshot_xgmi_rs_4gib_fp32"}))
    res = bench.read_child_result(str(path), "timeout", "tail")
    assert res["c4_rccl_rs_ag_4gib_fp32"] == {"rs_ms": 1.0}
    assert "stopped inside this phase" in res["c4_oneshot_xgmi_rs_4gib_fp32"]["error"]
    assert res["error"].startswith("collective child exited with timeout")
    assert not path.exists()
    fails = bench.collective_failures(res)
    assert any(f.startswith("c4_oneshot_xgmi_rs_4gib_fp32") for f in fails), fails
    # a clean child: its final file, no error entries
    path.write_text(json.dumps({"c4_rccl_rs_ag_4gib_fp32": {"rs_ms": 1.0}}))
    res = bench.read_child_result(str(path), 0, "")
    assert bench.collective_failures(res) == [] and "running" not in res
    # no file at all
    res = bench.read_child_result(str(tmp_path / "none.json"), 1, "boom")
    assert res["error"] == "collective child exited with 1" and res["tail"] == "boom"


def test_collective_alloc_plan_is_balanced_and_fits():
    """the per-rank allocation plan of the 8-GPU collective
    phases (bench.collective_alloc_plan, also what --collective-dry-alloc
    allocates): every free matches an earlier allocation of the same size,
    nothing goes negative, and the peak stays far below one MI355X's 288 GB."""
    import bench
    plan = bench.collective_alloc_plan(8)
    live = {}
    for phase, act, name, nbytes in plan:
        assert act in ("alloc", "free") and nbytes > 0
        if act == "alloc":
            assert name not in live, name
            live[name] = nbytes
        else:
            assert live.pop(name) == nbytes, name
    peak = bench.plan_peak(plan)
    assert 16 << 30 < peak < 20 << 30, peak          # C4's rounded leg: 17.5 GiB
    assert bench.plan_peak(bench.collective_alloc_plan(2)) > peak   # bigger shards
