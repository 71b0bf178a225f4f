"""One member of a multi-process allreduce through the builtin operation
engine (libucg_builtin.so) over the shared-memory transport.

    _worker_ops.py <shm-name> <mode: host|dev> <max_short> <iters> [ring_cells]

Every case is checked bit for bit against the oracle's simulation of the
reference's recursive-doubling plan (oracle/combine_ref.c) on this member."""
import os
import sys
import time

import numpy as np

from oracle import oracle as O
from xucg_amd import host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402

CASES = [  # (dtype, op, dist, count)
    ("float32", "sum", "exact", 1024),        # BASELINE config 1: 4 KiB fp32
    ("float32", "sum", "round", 1024),
    ("float32", "sum", "special", 257),
    ("float64", "prod", "round", 999),
    ("int32", "max", "round", 3001),
    ("float16", "sum", "special", 511),
    ("uint8", "bxor", "round", 4099),
    ("bfloat16", "min", "special", 700),
    ("float32", "sum", "round", 1),
    ("int64", "sum", "round", 0),           # empty: completes at start
]


def main():
    name, mode, max_short, iters = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    ring_cells = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    mpi = MockMPI()
    if mode == "dev":
        cfg = host.make_config(dev_enable=2, dev_min_bytes=0, stage_bytes=1 << 16)
    else:
        cfg = host.make_config(dev_enable=0)
    cmb = host.BuiltinCombine(mpi.callbacks(), cfg, op_classifier=op_classifier,
                              dt_classifier=dt_classifier)
    if mode == "dev" and not cmb.has_device:
        print("no device", flush=True)
        sys.exit(2)
    iface = ops.ShmIface(name, world, rank, max_short=max_short, ring_cells=ring_cells)
    group = ops.Group(iface, 7, world, rank, cmb)
    rc = 0
    for dt, op, dist, count in CASES:
        st = O.storage(dt)
        inputs = [O.fill(dt, dist, 500 + r, count) for r in range(world)]
        want = O.reduce_multi(op, dt, inputs, rank)
        for in_place in (False, True):
            sbuf = inputs[rank].copy()
            rbuf = sbuf if in_place else np.zeros_like(sbuf)
            coll = group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op])
            assert coll.status == 0, coll.status
            status = coll.run()
            if status != 0 or not (O.bits(rbuf) == O.bits(want)).all():
                print(f"rank {rank}: MISMATCH {dt} {op} {dist} n={count} "
                      f"in_place={in_place} status={status}", flush=True)
                rc = 1
            coll.close()
    # persistent op reused: C1 latency (4 KiB fp32)
    x = O.fill("float32", "exact", 900 + rank, 1024)
    out = np.zeros_like(x)
    coll = group.allreduce(x, out, 1024, DTYPES["float32"], OPS["sum"])
    for _ in range(5):
        coll.run()
    iface.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        coll.run()
    dt_us = (time.perf_counter() - t0) / max(iters, 1) * 1e6
    want = O.reduce_multi("sum", "float32",
                          [O.fill("float32", "exact", 900 + r, 1024) for r in range(world)],
                          rank)
    if not (O.bits(out) == O.bits(want)).all():
        print(f"rank {rank}: persistent op MISMATCH", flush=True)
        rc = 1
    coll.close()
    # two ops in flight on one group at once (slots coll_id % 16,
    # builtin_ops.h:388): the second finds the step staging busy and combines
    # per fragment; both must still match the plan
    cases2 = [("int32", "sum", "round", 3001), ("float32", "sum", "exact", 2500)]
    colls, sends, outs, wants = [], [], [], []
    for k, (dt, op, dist, count) in enumerate(cases2):
        ins = [O.fill(dt, dist, 1300 + 17 * k + r, count) for r in range(world)]
        wants.append(O.reduce_multi(op, dt, ins, rank))
        sends.append(ins[rank])
        outs.append(np.zeros_like(ins[rank]))
        colls.append(group.allreduce(sends[-1], outs[-1], count, DTYPES[dt], OPS[op]))
    sts = [c.start() for c in colls]
    for c, st in zip(colls, sts):
        if st == 1:   # UCS_INPROGRESS
            st = c.wait()
        if st != 0:
            print(f"rank {rank}: concurrent op status {st}", flush=True)
            rc = 1
    for (dt, op, dist, count), got, want in zip(cases2, outs, wants):
        if not (O.bits(got) == O.bits(want)).all():
            print(f"rank {rank}: concurrent op MISMATCH {dt} {op}", flush=True)
            rc = 1
    for c in colls:
        c.close()
    # with every message on the remote-key steps only small control messages
    # use the ring, and whether 3 cells ever fill depends on the peers' timing:
    # the resend check holds for the data-carrying ring only
    zcopy = os.environ.get("UCX_BUILTIN_SHM_ZCOPY_THRESH", "") == "1"
    if ring_cells <= 4 and not zcopy and group.stats()["resends"] == 0:
        print(f"rank {rank}: expected UCS_ERR_NO_RESOURCE resends with {ring_cells} cells",
              flush=True)
        rc = 1
    if rank == 0:
        print(f"describe:\n{group.allreduce(x, out, 1024, DTYPES['float32'], OPS['sum']).describe()}")
        print(f"latency_us {dt_us:.2f} stats {group.stats()} combine {cmb.stats()}", flush=True)
    group.close()
    iface.close()
    cmb.close()
    if rc == 0:
        print(f"rank {rank}: ok", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
