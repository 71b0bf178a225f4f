"""One member of a multi-process collective on a placement (hosts, sockets)
through the builtin operation engine: the plan the engine builds is checked
against the oracle's restatement (oracle/plans.py), then allreduce and
reduce to several roots run and are checked against the oracle's simulation
of every member's plan.

    _worker_topo.py <shm-name> <mode: host|dev|rma|shm> <max_short> <n:ppn:socket:radix:factor:thresh>

socket = 0 means no socket level. Mode dev stages every REDUCE step of host
buffers on the GPU; mode rma gives the engine device buffers (GPU memory on
device rank % device count), which it runs as remote-key steps: keys once per
op, READY / DONE over the transport, every receive one kernel reading the
senders' buffers. Mode shm runs host buffers through the same steps with
POSIX shared memory segments as the exposed buffers
(UCX_BUILTIN_SHM_ZCOPY_THRESH=1). The transport is the shared-memory one
for every member: a NET distance changes the plan, not the wire.

Checks:
  - the plan: every step's method, step index, send and receive peers (in
    order) equal the oracle's; a layout the oracle rejects is
    UCS_ERR_UNSUPPORTED at create;
  - integer types, every op, and fp SUM of exact integers: bit-exact against
    the oracle's simulation (arrival order does not change these results);
  - fp SUM of rounded values: within the SURVEY 8c-style relative bound of
    the fp64 sum, and "digest" lines so the test can check that every member
    of an allreduce holds identical bits."""
import ctypes
import hashlib
import os
import re
import sys

import numpy as np

from oracle import oracle as O
from oracle import plans as P
from xucg_amd import host, ops

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mock_mpi import MockMPI, OPS, DTYPES, op_classifier, dt_classifier  # noqa: E402

UCS_ERR_UNSUPPORTED = -22
CASES = [("int32", "sum", 3001), ("uint8", "bxor", 777), ("int64", "max", 257),
         ("float64", "sum", 1500), ("uint32", "sum", 64), ("int16", "prod", 33),
         ("float16", "max", 513), ("bfloat16", "min", 300)]
STEP_RE = re.compile(r"Step #\d+ \(step_idx (\d+)\): (\w+)"
                     r"(?:, send (?:send|recv)\.buffer to ([\d ]+))?"
                     r"(?:, receive from ([\d ]+))?"
                     r"(?:, then send recv\.buffer to ([\d ]+))?")


def parse(text):
    out = []
    for m in STEP_RE.finditer(text):
        step, method, s1, r, s2 = m.groups()
        send = s1 or s2 or ""
        out.append((method, int(step), [int(x) for x in send.split()],
                    [int(x) for x in (r or "").split()]))
    return out


def digest(a):
    return hashlib.sha1(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()[:16]


def identify(bad, good, candidates):
    """Where the bytes of a corrupted buffer differ from what it should hold:
    the byte range, and which recently seen arrays (candidates: name -> array)
    hold the corrupted bytes at the same offsets - a diagnosis, not a check."""
    b, g = np.ascontiguousarray(bad).view(np.uint8), np.ascontiguousarray(good).view(np.uint8)
    pos = np.nonzero(b != g)[0]
    if pos.size == 0:
        return "no byte differs"
    out = [f"{pos.size} bytes differ in [{pos[0]}, {pos[-1]}] "
           f"(128-B lines {pos[0] // 128}..{pos[-1] // 128})"]
    scores = []
    for nm, arr in candidates.items():
        c = np.ascontiguousarray(arr).view(np.uint8)
        inr = pos[pos < c.size]
        if inr.size:
            scores.append((float((c[inr] == b[inr]).mean()) * inr.size / pos.size, nm))
    scores.sort(reverse=True)
    out.append("best matches: " + ", ".join(f"{nm} {sc:.2f}" for sc, nm in scores[:4]))
    return "; ".join(out)


GUARD = 4096          # guard zone before and after every per-case device buffer
GUARD_BYTE = 0xA5


class RawHip:
    """Device memory straight from hipMalloc / hipFree of the process's HIP
    runtime (the one torch loaded: same soname), outside the shim: the user
    buffers of a GPU-aware MPI. Uploads and downloads go through the shim's
    memcpy, as DevBuffer's."""
    _hip = None

    def __init__(self, dctx, nbytes):
        from xucg_amd import _lib
        if RawHip._hip is None:
            _lib.dev()                          # loads the process's HIP runtime first
            RawHip._hip = ctypes.CDLL("libamdhip64.so.7")
            RawHip._hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
            RawHip._hip.hipFree.argtypes = [ctypes.c_void_p]
        self.dctx, self.nbytes = dctx, nbytes
        p = ctypes.c_void_p()
        rc = RawHip._hip.hipMalloc(ctypes.byref(p), nbytes)
        if rc != 0 or not p.value:
            raise MemoryError(f"hipMalloc({nbytes}) failed: {rc}")
        self.ptr = p.value

    def upload(self, arr, offset=0):
        from xucg_amd import _lib
        arr = np.ascontiguousarray(arr)
        _lib.check(_lib.dev().ucg_builtin_dev_memcpy(self.dctx.handle, self.ptr + offset,
                                                     arr.ctypes.data, arr.nbytes), "memcpy H2D")

    def download(self, dtype, count, offset=0):
        from xucg_amd import _lib
        out = np.empty(count, dtype=dtype)
        _lib.check(_lib.dev().ucg_builtin_dev_memcpy(self.dctx.handle, out.ctypes.data,
                                                     self.ptr + offset, out.nbytes), "memcpy D2H")
        return out

    def free(self):
        if self.ptr:
            self.dctx.sync()
            RawHip._hip.hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = None


class Guarded:
    """A device buffer between two guard zones of a known pattern: a write
    past either end of the buffer is found when it is freed. By default the
    shim's plain allocator (hipMalloc behind its reuse cache). Round 4 took
    shareable memory here, at addresses never used before; round 5 measured
    that a virtual-memory allocation makes the HIP runtime create one more
    hardware queue per process, after which every process on the GPU is
    time-sliced, and that DMA into a process's own recycled
    hipMalloc memory reads right. XUCG_TOPO_PLAIN=0: shareable
    memory; XUCG_TOPO_PLAIN=raw: hipMalloc / hipFree called here, as a
    GPU-aware MPI does, so the runtime recycles the addresses case after case
    (VERDICT r04 #3)."""

    def __init__(self, dctx, nbytes):
        plain = os.environ.get("XUCG_TOPO_PLAIN", "1")
        if plain == "raw":
            self.raw = RawHip(dctx, nbytes + 2 * GUARD)
        else:
            self.raw = dctx.alloc(nbytes + 2 * GUARD, shareable=plain == "0")
        self.nbytes = nbytes
        self.ptr = self.raw.ptr + GUARD
        pat = np.full(GUARD, GUARD_BYTE, np.uint8)
        self.raw.upload(pat, 0)
        self.raw.upload(pat, GUARD + nbytes)

    def upload(self, a):
        self.raw.upload(a, GUARD)

    def download(self, dtype, count):
        return self.raw.download(dtype, count, GUARD)

    def guards_damaged(self):
        out = []
        for name, off in (("head", 0), ("tail", GUARD + self.nbytes)):
            g = self.raw.download(np.uint8, GUARD, off)
            bad = np.nonzero(g != GUARD_BYTE)[0]
            if bad.size:
                out.append(f"{name} guard: {bad.size} bytes in [{bad[0]}, {bad[-1]}]")
        return "; ".join(out)

    def free(self):
        self.raw.free()


def main():
    name, mode, max_short = sys.argv[1], sys.argv[2], int(sys.argv[3])
    n, ppn, socket, radix, factor, thresh = map(int, sys.argv[4].split(":"))
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    assert world == n
    mpi = MockMPI()
    dctx = None
    if mode == "rma":
        import xucg_amd
        from xucg_amd import _lib
        ndev = max(1, _lib.dev().ucg_builtin_dev_device_count())
        dctx = xucg_amd.DevContext(device=rank % ndev)
        cfg = host.make_config(device=rank % ndev)
    elif mode == "shm":
        os.environ["UCX_BUILTIN_SHM_ZCOPY_THRESH"] = "1"
        cfg = host.make_config(dev_enable=0)
    elif mode == "dev":
        cfg = host.make_config(dev_enable=2, dev_min_bytes=0, stage_bytes=1 << 16)
    else:
        cfg = host.make_config(dev_enable=0)
    cmb = host.BuiltinCombine(mpi.callbacks(), cfg, op_classifier=op_classifier,
                              dt_classifier=dt_classifier)
    if mode in ("dev", "rma") and not cmb.has_device:
        print("no device", flush=True)
        sys.exit(2)

    def buf(a, what="buf"):
        """the op's buffer: the array itself, or a device copy of it between
        guard zones, read back right after the upload"""
        if dctx is None:
            return a
        b = Guarded(dctx, a.nbytes)
        b.upload(a)
        chk = b.download(a.dtype, a.size)
        if not (O.bits(chk) == O.bits(a)).all():
            fail(f"UPLOAD LOST before any engine call: {what} at 0x{b.ptr:x}; "
                 f"{identify(chk, a, {'zeros': np.zeros_like(a)})}")
            diag(b, what)
        return b

    def back(b, like):
        if isinstance(b, int):             # registered group memory
            return read_reg(b, like)
        return b if dctx is None else b.download(like.dtype, like.size)

    def ptr(b):
        return b.ptr if isinstance(b, Guarded) else b

    # TOPO_REGISTERED=1: send buffers from the group's registered memory
    # (ucg_builtin_lgroup_mem_alloc), exposed in place by remote-key steps
    registered = os.environ.get("TOPO_REGISTERED") == "1" and mode in ("rma", "shm")

    def read_reg(ptr, like):
        out = np.empty_like(like)
        if mode == "rma":
            _lib.dev().ucg_builtin_dev_memcpy(dctx.handle, out.ctypes.data, ptr, out.nbytes)
        else:
            ctypes.memmove(out.ctypes.data, ptr, out.nbytes)
        return out

    def send_buf(a):
        if not registered:
            return buf(a)
        p = group.mem_alloc(max(a.nbytes, 1), device=(mode == "rma"))
        if mode == "rma":
            _lib.dev().ucg_builtin_dev_memcpy(dctx.handle, p, a.ctypes.data, a.nbytes)
        else:
            ctypes.memmove(p, a.ctypes.data, a.nbytes)
        return p

    def free_buf(b, what):
        if isinstance(b, int):
            group.mem_free(b)
        elif dctx is not None and b is not None:
            bad = b.guards_damaged()
            if bad:
                fail(f"guard zone of {what} at 0x{b.ptr:x} written: {bad}")
                diag(b, what)
            b.free()

    iface = ops.ShmIface(name, n, rank, max_short=max_short, ring_cells=16)
    dist = ops.layout_distances(n, rank, ppn, socket or None)
    assert dist == P.layout(n, rank, ppn, socket or None)
    group = ops.Group(iface, 5, n, rank, cmb, distance=dist, radix=radix,
                      sock_thresh=thresh, factor=factor)
    cfgkw = dict(ppn=ppn, socket=socket or None, radix=radix, factor=factor,
                 sock_thresh=thresh)
    rc = 0

    def fail(msg):
        nonlocal rc
        print(f"rank {rank}: MISMATCH {msg}", flush=True)
        rc = 1

    def diag(b, what):
        """after a corrupted buffer: what the runtime and the device shim know
        about its allocation, the process's memory events near it, and whether
        it still reads the same 50 ms later (corruption analysis)"""
        if not isinstance(b, Guarded):
            return
        import time
        g0 = b.raw.download(np.uint8, GUARD, 0)
        time.sleep(0.05)
        g1 = b.raw.download(np.uint8, GUARD, 0)
        print(f"rank {rank}: DIAG {what} allocation 0x{b.raw.ptr:x} (+{b.raw.nbytes} B): head "
              f"guard zero bytes {int((g0 == 0).sum())} -> {int((g1 == 0).sum())} after 50 ms\n"
              + dctx.debug_ptr(b.raw.ptr), flush=True)

    kinds = [("allreduce", 0)] + [("reduce", r) for r in sorted({0, n - 1, n // 2})]
    seen = {}          # recent arrays, for identify() on a mismatch
    # TOPO_REPEAT=k runs the case list k times (a stress knob for races)
    for ci, (dt, op, count) in enumerate(CASES * int(os.environ.get("TOPO_REPEAT", "1"))):
        dist_kind = "exact" if dt.startswith("float") else "round"
        inputs = [O.fill(dt, dist_kind, 5000 + 31 * ci + m, count) for m in range(n)]
        seen = {k: v for k, v in seen.items() if k.startswith(f"c{ci - 1} ")}
        seen.update({f"c{ci} input{m}": x for m, x in enumerate(inputs)})
        for kind, root in kinds:
            try:
                want = P.simulate(kind, op, dt, inputs, root=root, **cfgkw)
                oplan = P.plan(kind, n, rank, root=root, **cfgkw)
            except P.Unsupported:
                want = oplan = None
            if want is not None:
                seen.update({f"c{ci} {kind}{root} want{m}": w for m, w in enumerate(want)
                             if w is not None})
            sbuf = send_buf(inputs[rank].copy())
            rbuf = buf(np.zeros_like(inputs[rank]), "recv buffer") if (
                kind == "allreduce" or rank == root) else None
            if dctx is not None:
                # every user buffer's address, so that a corrupted range can be
                # matched against the engine's launches (XUCG_RMA_TRACE)
                print(f"case c{ci} {kind}{root} {dt} {op}: sbuf 0x{ptr(sbuf):x} rbuf "
                      f"{'-' if rbuf is None else hex(ptr(rbuf))}", flush=True)
            coll = (group.allreduce(sbuf, rbuf, count, DTYPES[dt], OPS[op]) if kind == "allreduce"
                    else group.reduce(sbuf, rbuf, count, DTYPES[dt], OPS[op], root))
            if oplan is None:
                if coll.status != UCS_ERR_UNSUPPORTED:
                    fail(f"{kind} root={root}: oracle rejects the layout, create gave "
                         f"{coll.status}")
                coll.close()
                continue
            if coll.status != 0:
                fail(f"{kind} root={root}: create failed {coll.status}")
                continue
            if ci == 0:
                text = coll.describe()
                got = parse(text)
                exp = [(p["method"], p["step"], p["send"], p["recv"]) for p in oplan[2]]
                if got != exp:
                    fail(f"{kind} root={root} plan\n engine {got}\n oracle {exp}\n{text}")
                if kind == "allreduce" or root == n - 1:
                    print(f"describe {kind} root={root}:\n{text}", flush=True)
                if (mode == "rma") != ("Buffers: device memory" in text) or \
                        (mode == "shm") != ("Buffers: shared memory" in text):
                    fail(f"{kind} root={root}: buffers not described\n{text}")
            # persistent: a second start reuses the keys of the first
            for rep in range(2 if mode in ("rma", "shm") and ci < 2 else 1):
                if dctx is not None and not isinstance(sbuf, int):
                    pre = back(sbuf, inputs[rank])
                    if not (O.bits(pre) == O.bits(inputs[rank])).all():
                        fail(f"{kind} {dt} {op}: send buffer changed before start {rep} "
                             f"(no engine call has touched it): "
                             f"{identify(pre, inputs[rank], {'zeros': np.zeros_like(pre)})}")
                        diag(sbuf, "send buffer")
                st = coll.run()
                got = back(rbuf, inputs[rank]) if rbuf is not None else None
                if st != 0:
                    why = ""
                    if dctx is not None:
                        from xucg_amd import _lib
                        why = f" (device shim: {_lib.last_error()})"
                    fail(f"{kind} {dt} {op} root={root} start {rep} status={st}{why}")
                elif got is not None and not (O.bits(got) == O.bits(want[rank])).all():
                    bad = np.nonzero(O.bits(got) != O.bits(want[rank]))[0]
                    fail(f"{kind} {dt} {op} n={count} root={root} start {rep}: "
                         f"{bad.size} elements differ, first {bad[:6].tolist()}: got "
                         f"{got[bad[:3]].tolist()} want {want[rank][bad[:3]].tolist()}; "
                         f"{identify(got, want[rank], dict(seen, zeros=np.zeros_like(got)))}")
            sgot = back(sbuf, inputs[rank])
            if not (O.bits(sgot) == O.bits(inputs[rank])).all():
                fail(f"{kind} {dt} {op}: send buffer modified; "
                     f"{identify(sgot, inputs[rank], dict(seen, zeros=np.zeros_like(sgot)))}")
            if registered and ci == 0 and "Send buffer: registered" not in coll.describe():
                fail(f"{kind} root={root}: registered send buffer not exposed in place")
            coll.close()
            free_buf(sbuf, "send buffer")
            free_buf(rbuf, "recv buffer")

    # the last cases and the teardown take a second: a member that stalls in
    # them names its step (the Python stack on stderr after 60 s; the peers'
    # last barrier gives up after 90)
    import faulthandler
    faulthandler.dump_traceback_later(60, exit=False)
    # rounded fp32: tolerance against the fp64 sum, digests for identity
    for ci, count in enumerate((4096, 1000)):
        xs = [O.fill("float32", "round", 7000 + 11 * ci + m, count) for m in range(n)]
        f64 = np.sum([x.astype(np.float64) for x in xs], axis=0)
        scale = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
        rbuf_d = buf(np.zeros(count, np.float32))
        sbuf = buf(xs[rank].copy())      # the op keeps the address: keep it alive
        coll = group.allreduce(sbuf, rbuf_d, count, DTYPES["float32"], OPS["sum"])
        if coll.status == UCS_ERR_UNSUPPORTED:
            coll.close()
            continue
        st = coll.run()
        rbuf = back(rbuf_d, np.zeros(count, np.float32))
        tol = 2 * (n - 1) * 2.0 ** -24 * scale + 1e-30
        err = np.abs(rbuf.astype(np.float64) - f64)
        if st != 0 or not (err <= tol).all():
            i = int(np.argmax(err / tol))
            fail(f"allreduce float32 round n={count} status={st}: element {i} "
                 f"{rbuf[i]!r} vs {f64[i]!r} (error {err[i] / tol[i]:.3g} x the bound)")
        print(f"digest r{ci} {digest(rbuf)}", flush=True)
        coll.close()
    if rank == 0:
        print(f"stats {group.stats()} combine {cmb.stats()}", flush=True)
    group.close()
    iface.close()
    cmb.close()
    faulthandler.cancel_dump_traceback_later()
    if dctx is not None:
        dctx.close()
    if rc == 0:
        print(f"rank {rank}: ok", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
