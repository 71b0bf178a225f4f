"""One member of a randomized engine run: a seeded sequence of allreduce and
reduce ops (random dtype, op, count, root, in-place) on one group, each
checked bit for bit against the oracle (integer types and exact-integer
floats, so the tree's arrival order cannot change a result).

    _worker_fuzz.py <shm-name> <seed> <max_short> <ring_cells> [ppn:socket:radix:factor:thresh]

With a placement (hosts of ppn, sockets of `socket`, 0 = none) the expected
results come from the oracle's simulation of every member's plan
(oracle/plans.py); the inputs keep the association irrelevant.

FUZZ_BUFFERS picks where the op's buffers live: host (default), shm (host
buffers on the shared-memory remote-key steps), device (GPU memory: the
device remote-key steps), and shm-reg / device-reg (send buffers from the
group's registered memory, exposed in place)."""
import ctypes
import os
import sys

import numpy as np

from oracle import oracle as O
from oracle import plans as P
from xucg_amd import host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402

INT_DTS = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "int64", "uint64"]


def main():
    name, seed, max_short, cells = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), \
        int(sys.argv[4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    rng = np.random.default_rng(seed)          # same sequence on every member
    mpi = MockMPI()
    where = os.environ.get("FUZZ_BUFFERS", "host")
    device = where.startswith("device")
    reg = where.endswith("-reg")
    dctx = None
    if where.startswith("shm"):
        os.environ["UCX_BUILTIN_SHM_ZCOPY_THRESH"] = "1"
    if device:
        import xucg_amd
        from xucg_amd import _lib
        ndev = max(1, _lib.dev().ucg_builtin_dev_device_count())
        dctx = xucg_amd.DevContext(device=rank % ndev)
        cfg = host.make_config(device=rank % ndev)
    else:
        cfg = host.make_config(dev_enable=0)
    cmb = host.BuiltinCombine(mpi.callbacks(), cfg, op_classifier=op_classifier,
                              dt_classifier=dt_classifier)
    iface = ops.ShmIface(name, world, rank, max_short=max_short, ring_cells=cells)
    place = None
    if len(sys.argv) > 5:
        ppn, sock, radix, factor, thresh = map(int, sys.argv[5].split(":"))
        place = dict(ppn=ppn, socket=sock or None, radix=radix, factor=factor,
                     sock_thresh=thresh)
        group = ops.Group(iface, 5, world, rank, cmb,
                          distance=ops.layout_distances(world, rank, ppn, sock or None),
                          radix=radix, sock_thresh=thresh, factor=factor)
    else:
        group = ops.Group(iface, 5, world, rank, cmb)
    pow2 = (world & (world - 1)) == 0
    rc = 0

    def put(a, send):
        """the op's buffer for array a: itself, a device copy, or registered
        group memory for a send buffer"""
        nb = max(a.nbytes, 1)
        if reg and send:
            p = group.mem_alloc(nb, device=device)
            if device:
                _lib.dev().ucg_builtin_dev_memcpy(dctx.handle, p, a.ctypes.data, a.nbytes)
            else:
                ctypes.memmove(p, a.ctypes.data, a.nbytes)
            return p
        if device:
            b = dctx.alloc(nb)
            b.upload(a)
            return b
        return a

    def get(b, like):
        if isinstance(b, int):
            out = np.empty_like(like)
            if device:
                _lib.dev().ucg_builtin_dev_memcpy(dctx.handle, out.ctypes.data, b, out.nbytes)
            else:
                ctypes.memmove(out.ctypes.data, b, out.nbytes)
            return out
        return b.download(like.dtype, like.size) if device else b

    def drop(b):
        if isinstance(b, int):
            group.mem_free(b)
        elif device and b is not None:
            b.free()
    for k in range(40):
        if rng.random() < 0.75:
            dt = INT_DTS[rng.integers(len(INT_DTS))]
            op = ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor",
                  "bxor"][rng.integers(10)]
            dist = "round"
        else:
            dt, op, dist = ["float32", "float64"][rng.integers(2)], "sum", "exact"
        count = int(rng.choice([0, 1, 3, 100, 1000, int(rng.integers(1, 6000))]))
        kind = "reduce" if rng.random() < 0.35 else "allreduce"
        root = int(rng.integers(world))
        in_place = bool(rng.random() < 0.3)
        inputs = [O.fill(dt, dist, seed * 1000 + 10 * k + r, count) for r in range(world)]
        zeros = np.zeros_like(inputs[rank])
        sbuf = put(inputs[rank].copy(), True)
        has_recv = kind == "allreduce" or rank == root
        rbuf = (sbuf if in_place else put(zeros, False)) if has_recv else None
        if place and kind == "allreduce":
            want = P.simulate(kind, op, dt, inputs, **place)[rank]
            coll = group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op])
        elif place:
            want = P.simulate(kind, op, dt, inputs, root=root, **place)[root]
            coll = group.reduce(sbuf, rbuf, count, DTYPES[dt], OPS[op], root)
        elif kind == "allreduce":
            want = O.reduce_multi(op, dt, inputs, rank) if pow2 else \
                O.tree_reduce(op, dt, inputs, 0)
            coll = group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op])
        else:
            want = O.tree_reduce(op, dt, inputs, root)
            coll = group.reduce(sbuf, rbuf, count, DTYPES[dt], OPS[op], root)
        assert coll.status == 0, coll.status
        st = coll.run()
        got = get(rbuf, zeros) if rbuf is not None else None
        ok = st == 0 and (got is None or (O.bits(got) == O.bits(want)).all())
        if not ok:
            print(f"rank {rank}: MISMATCH seed {seed} op#{k} {kind} {dt} {op} n={count} "
                  f"root={root} in_place={in_place} status={st}", flush=True)
            rc = 1
        coll.close()
        drop(sbuf)
        if rbuf is not None and rbuf is not sbuf:
            drop(rbuf)
    group.close()
    iface.close()
    cmb.close()
    if dctx is not None:
        dctx.close()
    if rc == 0:
        print(f"rank {rank}: ok", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
