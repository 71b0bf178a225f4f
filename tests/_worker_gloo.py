"""One rank of the CPU multi-process test (gloo): runs the reference plan's
recursive-doubling schedule (xucg_amd.group.recursive_doubling_allreduce)
with the oracle as the combine and checks every rank's result bit for bit
against the oracle's own simulation of the plan."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

from oracle import oracle as O
from xucg_amd import group as G
from _shards import oracle_shard  # noqa: E402

CASES = [("float32", "sum", "special"), ("float32", "sum", "round"),
         ("float64", "sum", "round"), ("float32", "prod", "special"),
         ("int32", "prod", "round"), ("float16", "max", "special"),
         ("bfloat16", "sum", "round"), ("uint8", "bxor", "round")]


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    exchange = G.torch_exchange(dist)
    n = 1001
    for dt, op, dist_name in CASES:
        st = O.storage(dt)
        inputs = [O.fill(dt, dist_name, 7000 + r, n) for r in range(world)]
        acc = torch.from_numpy(inputs[rank].view(np.uint8).copy())
        tmp = torch.empty_like(acc)

        def combine(a, t):
            av = a.numpy().view(st)
            av[:] = O.reduce(op, dt, t.numpy().view(st), av)

        G.recursive_doubling_allreduce(acc, tmp, rank, world, combine, exchange)
        want = O.reduce_multi(op, dt, inputs, rank)
        got = acc.numpy().view(st)
        if not (O.bits(got) == O.bits(want)).all():
            print(f"rank {rank}: MISMATCH {dt} {op} {dist_name}", flush=True)
            sys.exit(1)
        # recursive halving: every element equals the plan's result on the
        # member that owns it after the reduce-scatter (all ranks identical)
        acc2 = torch.from_numpy(inputs[rank].view(np.uint8).copy())
        tmp2 = torch.empty_like(acc2)
        size = np.dtype(st).itemsize

        def combine_n(d, t, cnt):
            dv = d.numpy().view(st)
            dv[:] = O.reduce(op, dt, t.numpy().view(st), dv)

        G.recursive_halving_allreduce(acc2, tmp2, rank, world, combine_n, exchange, n, size)
        got2 = acc2.numpy().view(st)
        for owner, (lo, hi) in enumerate(G.recursive_halving_segments(n, world,
                                                                       max(1, 256 // size))):
            want_o = O.reduce_multi(op, dt, inputs, owner)
            if not (O.bits(got2[lo:hi]) == O.bits(want_o[lo:hi])).all():
                print(f"rank {rank}: halving MISMATCH {dt} {op} {dist_name} owner {owner}",
                      flush=True)
                sys.exit(1)
        # the one-shot shard of this rank equals the plan's result on it
        lo, hi, shard = oracle_shard(op, dt, inputs, rank, world, O)
        if not (O.bits(shard) == O.bits(want[lo:hi])).all():
            print(f"rank {rank}: shard mismatch {dt} {op}", flush=True)
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
