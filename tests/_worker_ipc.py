"""One rank of the GPU peer-mapping test: every rank lives on cuda:0 (the
only GPU of the test box), maps every other rank's buffer through the IPC
C-ABI and computes its shard with the one-shot recursive-doubling kernel,
checked bit for bit against the oracle's simulation of the reference plan."""
import os
import sys

import numpy as np
import torch.distributed as dist

import xucg_amd
from oracle import oracle as O
from xucg_amd import group as G

CASES = [("float32", "sum", "special"), ("float64", "sum", "round"),
         ("int32", "prod", "round"), ("float16", "sum", "special"),
         ("bfloat16", "max", "special")]


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = xucg_amd.DevContext(device=0)
    n = 100_003
    for dt, op, dname in CASES:
        st = O.storage(dt)
        sz = np.dtype(st).itemsize
        inputs = [O.fill(dt, dname, 300 + r, n) for r in range(world)]
        buf = ctx.alloc(n * sz)
        buf.upload(inputs[rank])
        out = ctx.alloc(n * sz)
        peers = G.PeerBuffers(ctx, buf.ptr, rank, world, dist)
        ctx.sync()
        dist.barrier()                      # every input is complete
        lo, hi = G.oneshot_reduce_scatter(ctx, peers, out.ptr, n, dt, op, rank, world)
        ctx.sync()
        dist.barrier()                      # every reader is done
        got = out.download(st, hi - lo)
        _, _, want = G.oracle_shard(op, dt, inputs, rank, world, O)
        peers.close()
        if not (O.bits(got) == O.bits(want)).all():
            print(f"rank {rank}: MISMATCH {dt} {op}", flush=True)
            sys.exit(1)
        # one-shot all-gather of the reduced shards, read from every peer
        full = ctx.alloc(n * sz)
        speers = G.PeerBuffers(ctx, out.ptr, rank, world, dist)
        G.oneshot_all_gather(ctx, speers, full.ptr, n, dt, world)
        ctx.sync()
        dist.barrier()
        speers.close()
        allgot = full.download(st, n)
        for r in range(world):
            rlo, rhi, rwant = G.oracle_shard(op, dt, inputs, r, world, O)
            if not (O.bits(allgot[rlo:rhi]) == O.bits(rwant)).all():
                print(f"rank {rank}: all-gather MISMATCH {dt} {op} shard {r}", flush=True)
                sys.exit(1)
        # one-shot allreduce: reduce-scatter into the recv buffer's own shard,
        # then every other shard read from its owner; every member ends with
        # the plan's result on every shard
        ctx.fill(dt, "special", 999, full, n)      # stale contents must not pass
        ctx.sync()
        rpeers = G.PeerBuffers(ctx, full.ptr, rank, world, dist)
        peers = G.PeerBuffers(ctx, buf.ptr, rank, world, dist)

        def barrier():
            ctx.sync()
            dist.barrier()
        G.oneshot_allreduce(ctx, peers, rpeers, n, dt, op, rank, world, barrier)
        allgot = full.download(st, n)
        rpeers.close()
        peers.close()
        for r in range(world):
            rlo, rhi, rwant = G.oracle_shard(op, dt, inputs, r, world, O)
            if not (O.bits(allgot[rlo:rhi]) == O.bits(rwant)).all():
                print(f"rank {rank}: allreduce MISMATCH {dt} {op} shard {r}", flush=True)
                sys.exit(1)
        full.free()
        buf.free()
        out.free()
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
