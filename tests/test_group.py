"""Multi-rank paths: shard math, the reference recursive-doubling plan over
gloo (CPU, world 2 and 4), and the peer-mapped one-shot kernel (GPU)."""
import os

import pytest

from xucg_amd import group as G
from _launch import launch


def test_shard_bounds_cover_and_align():
    for count in (1, 255, 256, 4096 + 7, 1 << 20, (1 << 30) + 13):
        for size in (1, 2, 4, 8):
            for world in (1, 2, 4, 8):
                bounds = [G.shard_bounds(count, size, world, r) for r in range(world)]
                assert bounds[0][0] == 0 and bounds[-1][1] == count
                for (a, b), (c, d) in zip(bounds, bounds[1:]):
                    assert b == c and a <= b
                for lo, _ in bounds:
                    assert (lo * size) % 256 == 0
    # 4 GiB fp32 over 8 GPUs: 512 MiB shards (config 4)
    assert G.shard_bounds(1 << 30, 4, 8, 3) == (3 << 27, 4 << 27)


def test_recursive_steps_and_peers():
    assert G.recursive_steps(8) == 3 and G.recursive_steps(6) == 0
    assert [G.recursive_peer(5, s) for s in (1, 2, 3)] == [4, 7, 1]


def test_recursive_halving_segments_partition():
    for count in (1, 7, 1001, 1 << 20):
        for world in (1, 2, 4, 8):
            segs = G.recursive_halving_segments(count, world, 32)
            covered = sorted(segs)
            assert covered[0][0] == 0 and covered[-1][1] == count
            assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_recursive_doubling_plan_over_gloo(world):
    codes, outs = launch("_worker_gloo.py", world, timeout=240)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_reduce_scatter_over_ipc(world):
    codes, outs = launch("_worker_ipc.py", world, timeout=300)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.gpu
def test_bench_collective_phases_world1():
    """bench.py's N > 1 collective phases (C4 RCCL RS+AG, one-shot xGMI RS
    with its parity check, C5 recursive doubling with its parity check) run
    under torch.distributed.run at world 1 (only 1-GPU boxes are available to
    the tests; the driver runs N = 2..8)."""
    import json
    import subprocess
    import sys
    from _launch import ROOT, free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-extra", "--collective-force"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    coll = line["collective"]
    assert coll, line
    for name, res in coll.items():
        assert isinstance(res, dict) and "error" not in res, (name, res)
    c4 = coll["c4_oneshot_xgmi_rs_4gib_fp32"]
    assert c4["bit_exact_vs_rccl_on_exact_inputs"] is True, c4
    assert c4["rccl_within_8c_tolerance_on_rounded_inputs"] is True, c4
    assert c4["oneshot_ag_bit_exact_vs_rccl"] is True, c4
    c5 = coll["c5_recursive_allreduce_512mib_fp64"]
    assert c5["doubling"]["bit_exact_vs_oneshot_tree"] is True, c5
    assert c5["halving"]["bit_exact_vs_oneshot_tree"] is True, c5
    assert c5["rccl_allreduce_within_8c_tolerance_of_plan"] is True, c5


@pytest.mark.parametrize("mode,bad", [("ok", 0), ("export", 1), ("import", 2), ("import", 0)])
def test_peer_buffers_failures_are_agreed(mode, bad):
    codes, outs = launch("_worker_peers.py", 3, args=(mode, bad), timeout=120)
    assert codes == [0] * 3, "\n".join(outs)
