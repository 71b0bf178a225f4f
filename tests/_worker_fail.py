"""One member of a group in which one member fails: no
survivor may hang or be killed; every survivor's op and close end with a
status, and the survivor exits 0.

    _worker_fail.py <shm-name> <mode> <victim>

modes (the victim is member <victim>):
  exit-before   the victim exits right after the set-up barrier, before it
                starts the op: the survivors' op ends with
                UCS_ERR_CONNECTION_RESET, their close with the same status
  exit-during   the victim starts the op (a 2-cell ring: it stops at
                UCS_ERR_NO_RESOURCE), then exits in the middle of it
  cancel        the victim starts the op and destroys it while it runs
                (UCS_ERR_CANCELED, published as abandoned): the survivors'
                op ends with UCS_ERR_CANCELED; every member is alive, so the
                last barrier and the close succeed
Each survivor prints one JSON line: its op status, its close status and how
long the failed op took to end."""
import json
import os
import sys
import time

import numpy as np

from xucg_amd import _lib, host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES  # noqa: E402


def main():
    name, mode, victim = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    iface = ops.ShmIface(name, world, rank, max_short=256, ring_cells=2)
    group = ops.Group(iface, 3, world, rank, cmb)
    count = 64 * 1024                     # 256 KiB fp32: ~1,000 fragments per peer
    x = np.full(count, float(rank + 1), dtype=np.float32)
    out = np.zeros_like(x)
    coll = group.allreduce(x, out, count, DTYPES["float32"], OPS["sum"])
    assert coll.status == 0, coll.status
    iface.barrier()
    if rank == victim:
        if mode == "exit-before":
            os._exit(0)
        st = coll.start()
        if mode == "exit-during":
            for _ in range(200):
                group.progress()
            os._exit(0)
        # cancel: destroy the running op (finish -> UCS_ERR_CANCELED,
        # published), then meet the others at the last barrier
        assert st == _lib.UCS_INPROGRESS, st
        coll.close()
        group.close()
        cst = iface.close()
        print(json.dumps({"rank": rank, "victim": True, "close": cst}), flush=True)
        cmb.close()
        sys.exit(0 if cst == 0 else 1)
    t0 = time.monotonic()
    st = coll.start()
    if st == _lib.UCS_INPROGRESS:
        st = coll.wait()
    took = time.monotonic() - t0
    coll.close()
    group.close()
    cst = iface.close()
    cmb.close()
    print(json.dumps({"rank": rank, "status": st, "close": cst, "took_s": round(took, 3)}),
          flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
