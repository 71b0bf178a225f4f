"""One member of a multi-process tree collective (MPI_Reduce and the
non-power-of-two MPI_Allreduce) through the builtin operation engine over
the shared-memory transport.

    _worker_tree.py <shm-name> <mode: host|dev> <max_short> [ring_cells]

The root reduces its children's messages in arrival order, so the checks are:
  - integer types, every op: bit-exact vs the oracle's tree simulation (the
    association does not change an integer result);
  - fp32/fp64 SUM of exact integers: bit-exact;
  - fp SUM of rounded values (and any fp16/bf16 SUM): within a per-dtype
    relative tolerance (written in FP_ROUND) of the fp64 sum, and
    (checked by the test across the printed digests) identical bits on every
    member of an allreduce.
Each case prints "digest <case> <sha1 of recv.buffer>" for the cross-member
check."""
import hashlib
import os
import sys

import numpy as np

from oracle import oracle as O
from xucg_amd import host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402

INT_CASES = [  # (dtype, op, count)
    ("int32", "sum", 3001),
    ("int32", "prod", 257),
    ("int64", "max", 999),
    ("uint8", "bxor", 4099),
    ("int16", "min", 700),
    ("uint32", "land", 64),
    ("int8", "lor", 1),
    ("int32", "max", 0),             # empty: completes at start on every member
    ("uint64", "band", 2048),
    ("uint8", "sum", 4099),          # unsigned SUM: the atomic packers with incast
    ("uint16", "sum", 513),
    ("uint32", "sum", 1000),
    ("uint64", "sum", 77),
]
FP_EXACT = [("float32", "sum", 1024), ("float64", "sum", 1500)]
# (dtype, op, count, rtol): fp16/bf16 partial sums of "exact" inputs can round
# too, so the half types are checked by tolerance like rounded values
FP_ROUND = [("float32", "sum", 4096, 1e-5), ("float64", "sum", 777, 1e-13),
            ("float16", "sum", 300, 4e-3), ("bfloat16", "sum", 333, 3e-2)]


def to_float64(dt, a):
    if dt == "float16":
        return a.view(np.float16).astype(np.float64)
    if dt == "bfloat16":
        return (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return a.astype(np.float64)


def digest(a):
    return hashlib.sha1(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()[:16]


def main():
    name, mode, max_short = sys.argv[1], sys.argv[2], int(sys.argv[3])
    ring_cells = int(sys.argv[4]) if len(sys.argv) > 4 else 64
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
    group = ops.Group(iface, 9, world, rank, cmb)
    rc = 0

    def fail(msg):
        nonlocal rc
        print(f"rank {rank}: MISMATCH {msg}", flush=True)
        rc = 1

    roots = sorted({0, world - 1, world // 2})
    for case_i, (dt, op, count) in enumerate(INT_CASES + [c[:3] for c in FP_EXACT]):
        dist = "exact" if dt.startswith(("float", "bfloat")) else "round"
        inputs = [O.fill(dt, dist, 700 + 13 * case_i + r, count) for r in range(world)]
        # allreduce (tree when world is not a power of two)
        for in_place in (False, True):
            want = O.tree_reduce(op, dt, inputs, 0)
            sbuf = inputs[rank].copy()
            rbuf = sbuf if in_place else np.zeros_like(sbuf)
            coll = group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op])
            assert coll.status == 0, coll.status
            st = coll.run()
            if st != 0 or not (O.bits(rbuf) == O.bits(want)).all():
                fail(f"allreduce {dt} {op} n={count} in_place={in_place} status={st}")
            coll.close()
        # reduce to several roots; non-roots pass no recv buffer
        for root in roots:
            want = O.tree_reduce(op, dt, inputs, root)
            sbuf = inputs[rank].copy()
            rbuf = np.zeros_like(sbuf) if rank == root else None
            coll = group.reduce(sbuf, rbuf, count, DTYPES[dt], OPS[op], root)
            assert coll.status == 0, coll.status
            st = coll.run()
            if st != 0:
                fail(f"reduce {dt} {op} root={root} status={st}")
            elif rank == root and not (O.bits(rbuf) == O.bits(want)).all():
                fail(f"reduce {dt} {op} n={count} root={root}")
            if rank != root and not (O.bits(sbuf) == O.bits(inputs[rank])).all():
                fail(f"reduce {dt} {op}: send buffer modified on a child")
            coll.close()

    for case_i, (dt, op, count, rtol) in enumerate(FP_ROUND):
        inputs = [O.fill(dt, "round", 900 + 7 * case_i + r, count) for r in range(world)]
        f64 = [to_float64(dt, x) for x in inputs]
        ref = np.sum(f64, axis=0)
        sbuf = inputs[rank].copy()
        rbuf = np.zeros_like(sbuf)
        coll = group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op])
        st = coll.run()
        scale = np.sum(np.abs(f64), axis=0)
        got = to_float64(dt, rbuf)
        if st != 0 or not (np.abs(got - ref) <= rtol * scale + 1e-30).all():
            fail(f"allreduce {dt} {op} round n={count} status={st}")
        print(f"digest fp{case_i} {digest(rbuf)}", flush=True)
        coll.close()

    x = O.fill("float32", "exact", 1, 1024)
    c = group.allreduce(x, np.zeros_like(x), 1024, DTYPES["float32"], OPS["sum"])
    text = c.describe()
    print("describe:\n" + text, flush=True)
    c.close()
    u = np.zeros(64, np.uint32)
    c = group.allreduce(u, np.zeros_like(u), 64, DTYPES["uint32"], OPS["sum"])
    print("describe uint32 sum:\n" + c.describe(), flush=True)
    c.close()
    if "(tree)" in text:
        up, down = O.tree_intra(rank, world, 0)
        want = (f"receive from {' '.join(map(str, down))}," if not up else
                f"send send.buffer to {up[0]},")
        if want not in text:
            fail(f"plan differs from the oracle's tree: expected '{want}'")
    print(f"stats {group.stats()} combine {cmb.stats()}", flush=True)
    if ring_cells <= 2 and group.stats()["resends"] == 0 and rank == 0:
        fail(f"expected UCS_ERR_NO_RESOURCE resends at the root with {ring_cells} cells")
    group.close()
    iface.close()
    cmb.close()
    if rc == 0:
        print(f"rank {rank}: ok", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
