"""Multi-rank paths: shard math, the reference recursive-doubling plan over
gloo (CPU, world 2 and 4), and the peer-mapped one-shot kernel (GPU)."""
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


@pytest.mark.parametrize("world", [2, 4])
def test_recursive_doubling_plan_over_gloo(world):
    codes, outs = launch("_worker_gloo.py", world, timeout=240)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_reduce_scatter_over_ipc(world):
    codes, outs = launch("_worker_ipc.py", world, timeout=300)
    assert codes == [0] * world, "\n".join(outs)
