"""One rank of the stale-key test: every rank exports a
buffer, frees it, allocates a new one of the same size (often at the same
address) and exports that; the peers must read the new contents through the
new key, and an import of the old key must be refused ("stale key",
UCS_ERR_NO_RESOURCE) instead of mapping whatever lives there now.

    python tests/_worker_ipc_churn.py KIND ROUNDS
      KIND  shareable  ucg_builtin_dev_malloc_shareable (HIP VMM, fd keys)
            plain      ucg_builtin_dev_malloc (hipMalloc, hipIpc keys checked
                       against the runtime's buffer id)
            torch      torch tensors with torch's allocator routed through the
                       shim (xucg_amd.use_shareable_torch_memory), freed and
                       the cache emptied between rounds

All ranks share GPU 0; gloo carries the keys. Every mapping is read by DMA
and by a kernel (ucg_builtin_dev_copy_multi)."""
import ctypes
import os
import sys

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

NBYTES = 6 << 20          # three 2 MiB granules


def main():
    kind, rounds = sys.argv[1], int(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if kind == "torch":
        xucg_amd.use_shareable_torch_memory()      # before any device allocation
        import torch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = xucg_amd.DevContext(device=0)
    bad = 0

    def fail(msg):
        nonlocal bad
        bad += 1
        print(f"rank {rank}: FAIL {msg}", flush=True)

    def value(r, rnd):
        return float(1000 * rnd + r + 1)

    def read_back(ptr, n):
        """the mapping's first and last words by DMA, and its tail by a kernel"""
        h = np.empty(2, np.float64)
        for j, off in enumerate((0, (n - 1) * 8)):
            _lib.check(_lib.dev().ucg_builtin_dev_memcpy(ctx.handle, h[j:].ctypes.data,
                                                         ptr + off, 8), "memcpy")
        loc = ctx.alloc(4096)
        try:
            _lib.check(ctx.copy_multi([loc.ptr], [ptr + n * 8 - 4096], 4096), "copy_multi")
            ctx.sync()
            k = loc.download(np.float64, 512)
        finally:
            loc.free()
        return h, k

    old_keys = None
    n = NBYTES // 8
    for rnd in range(rounds):
        if kind == "torch":
            t = torch.full((n,), value(rank, rnd), dtype=torch.float64, device="cuda:0")
            torch.cuda.synchronize()
            ptr, holder = t.data_ptr(), t
            if not _lib.dev().ucg_builtin_dev_is_shareable(ptr):
                fail("a torch tensor is not shareable memory under the shim's allocator")
        else:
            holder = ctx.alloc(NBYTES, shareable=(kind == "shareable"))
            holder.upload(np.full(n, value(rank, rnd)))
            ptr = holder.ptr
            if bool(_lib.dev().ucg_builtin_dev_is_shareable(ptr)) != (kind == "shareable"):
                fail("ucg_builtin_dev_is_shareable disagrees with the allocation")
        key = ctx.ipc_export(ptr)
        if ctx.ipc_export(ptr) != key:
            fail("a second export of the same allocation gave another key")
        keys = [None] * world
        dist.all_gather_object(keys, (bytes(key), ptr))
        if old_keys is not None:
            for p in range(world):
                if keys[p][0] == old_keys[p][0]:
                    fail(f"round {rnd}: member {p}'s new allocation kept the old key")
        maps, first = [], None
        for p in range(world):
            if p == rank:
                continue
            m = ctx.ipc_import(keys[p][0])
            maps.append(m)
            first = p if first is None else first
            h, k = read_back(m, n)
            want = value(p, rnd)
            if not ((h == want).all() and (k == want).all()):
                fail(f"round {rnd}: member {p}'s buffer (exporter address 0x{keys[p][1]:x}, "
                     f"{'same address as the last round' if old_keys and old_keys[p][1] == keys[p][1] else 'new address'}) "
                     f"read {h.tolist()} / {k[[0, -1]].tolist()}, want {want}")
        # a second import of the same key is the same mapping
        if maps:
            again = ctx.ipc_import(keys[first][0])
            if again != maps[0]:
                fail("a second import of one key gave another mapping")
            ctx.ipc_release(again)
        ctx.sync()
        dist.barrier()
        for m in maps:
            ctx.ipc_release(m)
        dist.barrier()
        # every member frees its buffer; then the old keys must be refused
        if kind == "torch":
            del t, holder
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        else:
            holder.free()
        dist.barrier()
        for p in range(world):
            if p == rank:
                continue
            try:
                m = ctx.ipc_import(keys[p][0])
            except xucg_amd.UcsError as e:
                if e.status != -2:               # UCS_ERR_NO_RESOURCE: stale key
                    fail(f"round {rnd}: a freed key of member {p} failed with {e}")
            else:
                ctx.ipc_release(m)
                fail(f"round {rnd}: a freed key of member {p} was imported")
        old_keys = keys
        dist.barrier()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: {'ok' if bad == 0 else f'{bad} failures'}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
