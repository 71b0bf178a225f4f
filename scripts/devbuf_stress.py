"""Stress of the engine on device buffers in the pattern of the two unexplained
mismatches: every op allocates its send and receive buffers,
uploads, runs an allreduce or a reduce to a rotating root, checks the result
and that the send buffer is unchanged, then frees both. One process per
member, started by scripts/devbuf_stress.sh.

    RANK=r WORLD_SIZE=n python scripts/devbuf_stress.py <shm-name> <ops> <n:ppn:socket:radix:factor:thresh>

STRESS_COMPLETION=signal|sync picks how the engine waits for its kernels
(the pinned completion word, or hipStreamSynchronize); STRESS_ALLOC=op|once
allocates the buffers per op or once. Prints one JSON line per member."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import xucg_amd  # noqa: E402
from xucg_amd import _lib, host, ops  # noqa: E402
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402


def inputs(i, m, count):
    rng = np.random.default_rng(1000003 * i + m)
    return rng.integers(-1 << 20, 1 << 20, count, dtype=np.int32)


def main():
    name, nops = sys.argv[1], int(sys.argv[2])
    n, ppn, socket, radix, factor, thresh = map(int, sys.argv[3].split(":"))
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert world == n
    completion = os.environ.get("STRESS_COMPLETION", "signal")
    per_op = os.environ.get("STRESS_ALLOC", "op") == "op"
    ndev = max(1, _lib.dev().ucg_builtin_dev_device_count())
    dctx = xucg_amd.DevContext(device=rank % ndev)
    cmb = host.BuiltinCombine(MockMPI().callbacks(),
                              host.make_config(device=rank % ndev, completion=completion),
                              op_classifier=op_classifier, dt_classifier=dt_classifier)
    iface = ops.ShmIface(name, n, rank, max_short=256, ring_cells=16)
    group = ops.Group(iface, 5, n, rank, cmb,
                      distance=ops.layout_distances(n, rank, ppn, socket or None),
                      radix=radix, sock_thresh=thresh, factor=factor)
    cap = 20000 * 4
    keep = (dctx.alloc(cap), dctx.alloc(cap)) if not per_op else None
    bad, t0 = [], time.perf_counter()
    for i in range(nops):
        count = 257 + (i * 7919) % 19000
        root = i % n                       # n - 1 reduces to each root, then an allreduce
        kind = "allreduce" if i % (n + 1) == n else "reduce"
        xs = [inputs(i, m, count) for m in range(n)]
        want = np.sum(np.stack(xs).astype(np.int64), axis=0).astype(np.int32)
        sbuf, rbuf = (dctx.alloc(count * 4), dctx.alloc(count * 4)) if per_op else keep
        sbuf.upload(xs[rank])
        rbuf.upload(np.zeros(count, np.int32))
        if kind == "allreduce":
            c = group.allreduce(sbuf, rbuf, count, DTYPES["int32"], OPS["sum"])
        else:
            c = group.reduce(sbuf, rbuf, count, DTYPES["int32"], OPS["sum"], root)
        st = c.run()
        if st != 0:
            bad.append({"op": i, "kind": kind, "root": root, "status": st})
        elif kind == "allreduce" or rank == root:
            got = rbuf.download(np.int32, count)
            d = np.nonzero(got != want)[0]
            if d.size:
                bad.append({"op": i, "kind": kind, "root": root, "count": count,
                            "result_differs": int(d.size), "first": int(d[0]),
                            "last": int(d[-1])})
        s = sbuf.download(np.int32, count)
        d = np.nonzero(s != xs[rank])[0]
        if d.size:
            # what the send buffer holds instead: another member's input of
            # this op, the result, zeros?
            cand = {f"input{m}": xs[m] for m in range(n)}
            cand.update({f"prev_input{m}": inputs(i - 1, m, count) for m in range(n)})
            cand.update(result=want, zeros=np.zeros(count, np.int32))
            match = {k: round(float((v[d] == s[d]).mean()), 3) for k, v in cand.items()}
            bad.append({"op": i, "kind": kind, "root": root, "count": count,
                        "sbuf_differs": int(d.size), "first": int(d[0]), "last": int(d[-1]),
                        "matches": {k: v for k, v in match.items() if v > 0}})
        c.close()
        if per_op:
            sbuf.free()
            rbuf.free()
    print(json.dumps({"rank": rank, "ops": nops, "completion": completion,
                      "alloc": "op" if per_op else "once", "mismatches": len(bad),
                      "s": round(time.perf_counter() - t0, 1), "first": bad[:3]}), flush=True)
    group.close()
    iface.close()
    cmb.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
