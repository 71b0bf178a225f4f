"""Test helper: the expected one-shot shard (the oracle is the checker; the
product package never imports it)."""
import numpy as np

from xucg_amd.group import is_pow2, shard_bounds


def oracle_shard(op, dt, inputs, rank, world, oracle):
    """Expected one-shot shard: the plan's result on the owner."""
    size = np.dtype(inputs[0].dtype).itemsize
    lo, hi = shard_bounds(inputs[0].size, size, world, rank)
    shards = [x[lo:hi] for x in inputs]
    if is_pow2(len(inputs)):
        return lo, hi, oracle.reduce_multi(op, dt, shards, rank)
    return lo, hi, oracle.tree_reduce(op, dt, shards, root=0)
