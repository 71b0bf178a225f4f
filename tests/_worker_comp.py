"""One member of a completion-callback test (ucg_params_t.completion,
api/ucg.h:162-171): an allreduce started without waiting, completed by
progress alone, reported once through coll_comp_cb_f and once through the
flag/status words written into a request; the result checked against the
oracle's simulation.   _worker_comp.py <shm-name>"""
import ctypes
import os
import sys

import numpy as np

from oracle import oracle as O
from oracle import plans as P
from xucg_amd import host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES  # noqa: E402


def main():
    name = sys.argv[1]
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    iface = ops.ShmIface(name, n, rank, max_short=256)
    group = ops.Group(iface, 3, n, rank, cmb)
    count = 5000
    xs = [O.fill("int32", "round", 900 + m, count) for m in range(n)]
    want = P.simulate("allreduce", "sum", "int32", xs)[rank]
    sbuf, rbuf = xs[rank].copy(), np.zeros(count, np.int32)
    coll = group.allreduce(sbuf, rbuf, count, DTYPES["int32"], OPS["sum"])
    assert coll.status == 0
    seen = []
    assert coll.set_completion(lambda req, st: seen.append((req, st)), req=0x1234) == 0
    st = coll.start()
    while not seen:
        group.progress()
    assert seen == [(0x1234, 0)], seen
    assert st in (0, 1) and (rbuf == want).all()
    # flag and status words in a request of the caller's
    req = (ctypes.c_uint8 * 64)()
    ctypes.memset(req, 0xEE, 64)
    rbuf[:] = 0
    assert coll.set_completion(None, ctypes.addressof(req), 3, 8) == 0
    coll.start()
    while req[3] != 1:
        group.progress()
    status = ctypes.c_int.from_address(ctypes.addressof(req) + 8).value
    assert status == 0 and (rbuf == want).all(), status
    assert len(seen) == 1
    coll.close()
    group.close()
    iface.close()
    cmb.close()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
