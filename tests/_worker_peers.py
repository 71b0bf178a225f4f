"""PeerBuffers agreement over gloo with a stand-in context: a member whose
export or import fails must make every member raise (nobody left waiting).

    _worker_peers.py <mode: ok|export|import> <failing rank>"""
import os
import sys

import torch.distributed as dist

from xucg_amd import group as G


class FakeCtx:
    def __init__(self, rank, mode, bad):
        self.rank, self.mode, self.bad = rank, mode, bad
        self.released = []

    def ipc_export(self, ptr):
        if self.mode == "export" and self.rank == self.bad:
            raise RuntimeError("export failed")
        return b"blob%d" % self.rank

    def ipc_import(self, blob):
        if self.mode == "import" and self.rank == self.bad:
            raise RuntimeError("import failed")
        return 0x1000 + int(blob[4:])

    def ipc_release(self, p):
        self.released.append(p)


def main():
    mode, bad = sys.argv[1], int(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = FakeCtx(rank, mode, bad)
    try:
        peers = G.PeerBuffers(ctx, 0xABC, rank, world, dist)
        raised = False
    except RuntimeError:
        raised = True
    if mode == "ok":
        assert not raised and peers.ptrs[rank] == 0xABC
        assert [p for r, p in enumerate(peers.ptrs) if r != rank] == \
            [0x1000 + r for r in range(world) if r != rank]
        peers.close()
        assert len(ctx.released) == world - 1
    else:
        assert raised, "every member must raise"
    dist.barrier()           # nobody is stuck inside PeerBuffers
    dist.destroy_process_group()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
