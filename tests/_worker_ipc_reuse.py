"""One rank of the IPC-reuse probe: the allocation pattern of bench.py's
C4 then C5 phases (torch tensors, PeerBuffers on several of them, then
everything freed and the cache emptied, then new tensors exported), with
every imported mapping checked against the value its owner wrote. All ranks
share GPU 0; gloo carries the handles.

    python tests/_worker_ipc_reuse.py SCALE

Every mapping is read by DMA (hipMemcpyAsync) and by a kernel
(ucg_builtin_dev_copy_multi). Prints one line per wrong read (phase, buffer,
peer, how, exporter's VA, segment base and size, offset, the importer's
address) and exits 1 if there is any."""
import ctypes
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xucg_amd  # noqa: E402
from xucg_amd import _lib, group as G  # noqa: E402


def main():
    scale = int(sys.argv[1])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = xucg_amd.DevContext.on_torch_stream(0)
    dev = torch.device("cuda:0")
    bad = 0

    def peek(ptr):
        out = ctypes.c_double()
        _lib.check(_lib.dev().ucg_builtin_dev_memcpy(ctx.handle, ctypes.addressof(out), ptr, 8),
                   "memcpy")
        return out.value

    def info(t):
        """the tensor's address and its caching-allocator segment"""
        va = t.data_ptr()
        for seg in torch.cuda.memory_snapshot():
            if seg["address"] <= va < seg["address"] + seg["total_size"]:
                return va, seg["address"], seg["total_size"]
        return va, 0, 0

    def phase(name, specs):
        nonlocal bad
        tensors, peers = {}, []
        for i, (bname, elems, export) in enumerate(specs):
            t = torch.full((elems,), float(rank * 1000 + i), dtype=torch.float64, device=dev)
            tensors[bname] = t
        torch.cuda.synchronize()
        for i, (bname, elems, export) in enumerate(specs):
            if not export:
                continue
            t = tensors[bname]
            va, base, size = info(t)
            metas = [None] * world
            dist.all_gather_object(metas, (va, base, size))
            pb = G.PeerBuffers(ctx, t.data_ptr(), rank, world, dist)
            peers.append(pb)
            for p in range(world):
                want = float(p * 1000 + i)
                # the same mapping read two ways: a DMA copy (hipMemcpyAsync)
                # and a kernel (copy_multi) into a local buffer
                nk = min(elems, 1 << 13)
                local = torch.full((nk,), -1.0, dtype=torch.float64, device=dev)
                _lib.check(ctx.copy_multi([local.data_ptr()],
                                          [pb.ptrs[p] + (elems - nk) * 8], nk * 8),
                           "copy_multi")
                torch.cuda.synchronize()
                kern = local.cpu()
                for how, off, got in (("dma", 0, peek(pb.ptrs[p])),
                                      ("dma", (elems - 1) * 8, peek(pb.ptrs[p] + (elems - 1) * 8)),
                                      ("kernel", (elems - nk) * 8, kern[0].item()),
                                      ("kernel", (elems - 1) * 8, kern[-1].item())):
                    if got != want:
                        bad += 1
                        print(f"rank {rank} {name} {bname} peer {p} {how} off {off}: got {got} "
                              f"want {want}; exporter va 0x{metas[p][0]:x} base "
                              f"0x{metas[p][1]:x} size {metas[p][2]} offset "
                              f"{metas[p][0] - metas[p][1]}; mapped at 0x{pb.ptrs[p]:x}",
                              flush=True)
        torch.cuda.synchronize()
        dist.barrier()
        for pb in peers:
            pb.close()
        del tensors
        torch.cuda.empty_cache()

    n4 = (1 << 29) // scale          # C4's 4 GiB, as fp64 elements, scaled
    shard = n4 // world
    for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):
        phase(f"c4.{rep}", [("x", n4, True), ("rs_out", shard, False), ("ag_out", n4, True),
                            ("mine", shard, True), ("stage", world * shard, True)])
        n5 = (1 << 26) // scale
        phase(f"c5.{rep}", [("init", n5, True), ("acc", n5, True), ("tmp", n5, False),
                            ("stage5", n5, True)])
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: {'ok' if bad == 0 else f'{bad} wrong mappings'}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
