"""One member of the group-churn test: groups on device buffers created and
destroyed again and again in one process, with buffers of a few recurring
sizes freed and allocated between them, so that addresses and sizes - and
with them HIP IPC keys, which are (pid, address, size) - recur. Every
allreduce is checked whole against the oracle's recursive-doubling
association (ucg_oracle_reduce_multi). Half the groups take the send buffer
from the group's registered memory (exported pool buffers).

    _worker_churn.py <shm-name> <rounds>
"""
import os
import sys

import numpy as np

from oracle import oracle as O
from xucg_amd import host, ops
import xucg_amd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402

SIZES = (1 << 16, 3 << 15, 1 << 17)


def main():
    name, rounds = sys.argv[1], int(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ctx = xucg_amd.DevContext(device=0)
    cmb = host.BuiltinCombine(MockMPI().callbacks(), host.make_config(device=0),
                              op_classifier=op_classifier, dt_classifier=dt_classifier)
    rc = 0
    for it in range(rounds):
        n = SIZES[it % len(SIZES)]
        registered = it % 2 == 1
        seed = 0x5EED7000 + 97 * it
        xs = [O.fill("float64", "round", seed + m, n) for m in range(world)]
        want = O.reduce_multi("sum", "float64", xs, rank)
        iface = ops.ShmIface(f"{name}_{it}", world, rank, max_short=256)
        group = ops.Group(iface, 9, world, rank, cmb)
        acc = ctx.alloc(n * 8)
        if registered:
            sbuf = group.mem_alloc(n * 8, device=True)
            ctx_buf = ctx.alloc(n * 8)
            ctx_buf.upload(xs[rank])
            assert ctx.copy_multi([sbuf], [ctx_buf.ptr], n * 8) == 0
            ctx.sync()
            ctx_buf.free()
        else:
            sbuf_b = ctx.alloc(n * 8)
            sbuf_b.upload(xs[rank])
            sbuf = sbuf_b.ptr
        coll = group.allreduce(sbuf, acc, n, DTYPES["float64"], OPS["sum"])
        if coll.status != 0:
            print(f"rank {rank}: FAIL round {it}: create {coll.status}", flush=True)
            rc = 1
            break
        for rep in range(2):
            st = coll.run()
            got = acc.download(np.float64, n)
            if st != 0 or not (O.bits(got) == O.bits(want)).all():
                bad = np.nonzero(O.bits(got) != O.bits(want))[0]
                print(f"rank {rank}: FAIL round {it} start {rep} ({'registered' if registered else 'plain'}"
                      f" send buffer, n={n}): status {st}, {bad.size} elements differ", flush=True)
                rc = 1
        coll.close()
        if registered:
            group.mem_free(sbuf)
        else:
            sbuf_b.free()
        group.close()
        iface.close()
        acc.free()
        if rc:
            break
    cmb.close()
    ctx.close()
    print(f"rank {rank}: {'ok' if rc == 0 else 'FAILED'}", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
