"""One rank of the GPU peer-mapping test: every rank lives on cuda:0 (the
only GPU of the test box), maps every other rank's buffers through the IPC
C-ABI and runs the one-shot kernels over them, each result checked bit for bit
against the oracle's simulation of the reference plan:

  reduce-scatter  shard r of every member's send buffer -> V(r, log2 N)
  all-gather      every member's reduced shard, read in place
  allreduce       both in one operation into a recv buffer
  push forms      the same reduce-scatter and allreduce with every transfer a
                  write into a peer's buffer (stage slots, recv shards)
  reduce          MPI_Reduce to the last member: the tree fan-in, one launch

Every buffer is exported once, and all mappings are released by every
member (PeerBuffers.close, a collective) before any member frees a buffer."""
import os
import sys

import numpy as np
import torch.distributed as dist

import xucg_amd
from oracle import oracle as O
from xucg_amd import group as G
from _shards import oracle_shard  # noqa: E402

CASES = [("float32", "sum", "special"), ("float64", "sum", "round"),
         ("int32", "prod", "round"), ("float16", "sum", "special"),
         ("bfloat16", "max", "special")]


def fail(rank, what):
    print(f"rank {rank}: MISMATCH {what}", flush=True)
    sys.exit(1)


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = xucg_amd.DevContext(device=0)

    def barrier():
        ctx.sync()
        dist.barrier()

    n = 100_003
    for dt, op, dname in CASES:
        st = O.storage(dt)
        sz = np.dtype(st).itemsize
        inputs = [O.fill(dt, dname, 300 + r, n) for r in range(world)]
        shards = [oracle_shard(op, dt, inputs, r, world, O) for r in range(world)]
        # XUCG_IPC_SHAREABLE=1: every exported buffer is shareable memory
        # (mapped by its physical allocation), else hipMalloc (hipIpc keys)
        sh = os.environ.get("XUCG_IPC_SHAREABLE") == "1"
        buf, out = ctx.alloc(n * sz, shareable=sh), ctx.alloc(n * sz, shareable=sh)
        full = ctx.alloc(n * sz, shareable=sh)
        stage = ctx.alloc(world * G.stage_slot_bytes(n, sz, world), shareable=sh)
        buf.upload(inputs[rank])
        ctx.fill(dt, "special", 999, full, n)      # stale contents must not pass
        ctx.sync()
        peers = G.PeerBuffers(ctx, buf.ptr, rank, world, dist)
        speers = G.PeerBuffers(ctx, out.ptr, rank, world, dist)
        rpeers = G.PeerBuffers(ctx, full.ptr, rank, world, dist)
        tpeers = G.PeerBuffers(ctx, stage.ptr, rank, world, dist)
        dist.barrier()                      # every input is complete

        lo, hi = G.oneshot_reduce_scatter(ctx, peers, out.ptr, n, dt, op, rank, world)
        barrier()                           # every shard reduced, every reader done
        if not (O.bits(out.download(st, hi - lo)) == O.bits(shards[rank][2])).all():
            fail(rank, f"reduce-scatter {dt} {op}")

        G.oneshot_all_gather(ctx, speers, full.ptr, n, dt, world)
        barrier()
        allgot = full.download(st, n)
        for r, (rlo, rhi, rwant) in enumerate(shards):
            if not (O.bits(allgot[rlo:rhi]) == O.bits(rwant)).all():
                fail(rank, f"all-gather {dt} {op} shard {r}")

        ctx.fill(dt, "special", 998, full, n)
        barrier()
        G.oneshot_allreduce(ctx, peers, rpeers, n, dt, op, rank, world, barrier)
        allgot = full.download(st, n)
        for r, (rlo, rhi, rwant) in enumerate(shards):
            if not (O.bits(allgot[rlo:rhi]) == O.bits(rwant)).all():
                fail(rank, f"allreduce {dt} {op} shard {r}")

        # push forms: shards written into the peers' stages, then combined
        # locally; the reduced shard written into every peer's recv buffer
        ctx.fill(dt, "special", 997, out, n)
        barrier()
        G.push_reduce_scatter(ctx, buf.ptr, tpeers, out.ptr, n, dt, op, rank, world, barrier)
        barrier()
        if not (O.bits(out.download(st, hi - lo)) == O.bits(shards[rank][2])).all():
            fail(rank, f"push reduce-scatter {dt} {op}")
        ctx.fill(dt, "special", 996, full, n)
        barrier()
        G.push_allreduce(ctx, buf.ptr, tpeers, rpeers, n, dt, op, rank, world, barrier)
        allgot = full.download(st, n)
        for r, (rlo, rhi, rwant) in enumerate(shards):
            if not (O.bits(allgot[rlo:rhi]) == O.bits(rwant)).all():
                fail(rank, f"push allreduce {dt} {op} shard {r}")

        # MPI_Reduce to the last member: the tree fan-in read in one launch
        root = world - 1
        ctx.fill(dt, "special", 995, full, n)
        barrier()
        if G.oneshot_reduce(ctx, peers, full.ptr, n, dt, op, rank, world, root):
            ctx.sync()
            want = O.tree_reduce(op, dt, inputs, root=root)
            if not (O.bits(full.download(st, n)) == O.bits(want)).all():
                fail(rank, f"reduce to root {root} {dt} {op}")
        barrier()

        for p in (peers, speers, rpeers, tpeers):
            p.close()                       # collective: all mappings gone
        for b in (buf, out, full, stage):
            b.free()
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
