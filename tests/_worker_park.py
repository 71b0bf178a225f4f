"""One member of the parking test: member 0 starts an allreduce
on device buffers that member 1 never joins, so member 0's op exposes its
buffer (READY sent, a reader outstanding) and then times out; destroying its
group must park that buffer - keys retired, memory never handed out again
(ucg_builtin_dev_park, rma_group_free) - instead of returning it to the
reuse cache under the reader. Member 1 only opens the transport and the
group and waits for member 0 to finish.

    _worker_park.py <shm-name>
"""
import os
import sys
import time

import numpy as np

from xucg_amd import _lib, host, ops
import xucg_amd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402


def main():
    name = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ctx = xucg_amd.DevContext(device=0)
    cmb = host.BuiltinCombine(MockMPI().callbacks(), host.make_config(device=0),
                              op_classifier=op_classifier, dt_classifier=dt_classifier)
    iface = ops.ShmIface(name, world, rank, max_short=256)
    group = ops.Group(iface, 11, world, rank, cmb)
    rc = 0
    n = 1 << 16
    flag = f"/dev/shm/{name.strip('/')}_m0_done"
    if rank == 0:
        s = ctx.alloc(n * 8)
        r = ctx.alloc(n * 8)
        s.upload(np.arange(n, dtype=np.float64))
        coll = group.allreduce(s.ptr, r.ptr, n, DTYPES["float64"], OPS["sum"])
        p0 = _lib.mem_stats()["parked_bytes"]
        st = coll.run()                        # member 1 never starts: times out
        coll.close()
        group.close()
        parked = _lib.mem_stats()["parked_bytes"] - p0
        print(f"rank 0: status {st} parked {parked}", flush=True)
        if st != _lib.UCS_ERR_TIMED_OUT or parked <= 0:
            print("rank 0: FAIL: the op did not time out, or nothing was parked", flush=True)
            rc = 1
        s.free()
        r.free()
        open(flag, "w").close()
    else:
        t0 = time.time()
        while not os.path.exists(flag) and time.time() - t0 < 60:
            time.sleep(0.05)
        group.close()
        try:
            os.unlink(flag)
        except OSError:
            pass
    iface.close()
    cmb.close()
    ctx.close()
    print(f"rank {rank}: {'ok' if rc == 0 else 'FAILED'}", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
