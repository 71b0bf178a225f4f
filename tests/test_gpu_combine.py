"""GPU parity: the HIP combine path (through the C-ABI) against the oracle and
the golden vectors. Bit-exact for every dtype and op."""
import os

import numpy as np
import pytest

import xucg_amd
from xucg_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def bits(a):
    return O.bits(a)


def run_reduce(ctx, op, dt, src, dst, src_off=0, dst_off=0):
    """Upload, combine on the device, download. Offsets in bytes."""
    st = O.storage(dt)
    n = src.size
    nb = n * np.dtype(st).itemsize
    bs = ctx.alloc(nb + 64)
    bd = ctx.alloc(nb + 64)
    bs.upload(src, src_off)
    bd.upload(dst, dst_off)
    rc = ctx.reduce(op, dt, bd.ptr + dst_off, bs.ptr + src_off, n)
    assert rc == 0, _lib.last_error()
    ctx.sync()
    return bd.download(st, n, dst_off)


@pytest.mark.parametrize("dt", O.DTYPES)
def test_golden_vectors_on_gpu(dev_ctx, dt):
    z = np.load(os.path.join(GOLDEN, f"golden_{dt}.npz"))
    sz = np.dtype(O.storage(dt)).itemsize
    for k, op in enumerate(O.OPS):
        if not z["supported"][k]:
            assert dev_ctx.reduce(op, dt, 0, 0, 4) == xucg_amd.UCS_ERR_UNSUPPORTED
            continue
        # aligned, dst-misaligned-with-src (same phase) and relative-misaligned
        for so, do in ((0, 0), (sz, sz), (0, sz), (3 * sz, 5 * sz)):
            got = run_reduce(dev_ctx, op, dt, z["src"], z["dst"], so, do)
            bad = np.nonzero(bits(got) != bits(z["out"][k]))[0]
            assert bad.size == 0, (op, so, do, [
                (hex(int(bits(z["src"])[i])), hex(int(bits(z["dst"])[i])),
                 hex(int(bits(got)[i])), hex(int(bits(z["out"][k])[i]))) for i in bad[:4]])


@pytest.mark.parametrize("dt", O.DTYPES)
def test_fill_matches_oracle(dev_ctx, dt):
    n = 10007
    buf = dev_ctx.alloc(n * 8)
    for dist in O.DISTS:
        dev_ctx.fill(dt, dist, 0xC0FFEE, buf, n)
        dev_ctx.sync()
        got = buf.download(O.storage(dt), n)
        want = O.fill(dt, dist, 0xC0FFEE, n)
        assert (bits(got) == bits(want)).all(), dist


SIZES = [1, 2, 3, 7, 15, 16, 17, 31, 33, 255, 256, 257, 1000, 4099, 65537,
         (1 << 20) + 3]


@pytest.mark.parametrize("dt", O.DTYPES)
def test_ragged_sizes_vs_oracle(dev_ctx, dt):
    rng = np.random.default_rng(O.dt_index(dt))
    st = O.storage(dt)
    for n in SIZES:
        for dist in ("round", "special"):
            src = O.fill(dt, dist, 11 + n, n)
            dst = O.fill(dt, dist, 12 + n, n)
            ops = [op for op in O.OPS if O.is_supported(dt, op)]
            op = ops[int(rng.integers(len(ops)))] if n > 4099 else None
            for o in ([op] if op else ops):
                off = int(rng.integers(0, 4)) * np.dtype(st).itemsize
                got = run_reduce(dev_ctx, o, dt, src, dst, off, off)
                want = O.reduce(o, dt, src, dst)
                assert (bits(got) == bits(want)).all(), (o, n, dist)


def test_zero_count_is_noop(dev_ctx):
    assert dev_ctx.reduce("sum", "float32", 0, 0, 0) == 0


def test_self_combine(dev_ctx):
    n = 12345
    x = O.fill("float32", "round", 3, n)
    b = dev_ctx.alloc(n * 4)
    b.upload(x)
    assert dev_ctx.reduce("sum", "float32", b, b, n) == 0
    dev_ctx.sync()
    assert (bits(b.download(np.float32, n)) == bits(O.reduce("sum", "float32", x, x))).all()


def test_debug_ptr_memory_events(dev_ctx):
    """ucg_builtin_dev_debug_ptr: the runtime's view of a live allocation, and
    the malloc / free events of its address in the shim's event log (the
    diagnostics the device-buffer placement worker prints on a corrupted
    buffer). M: a new hipMalloc; R: a freed allocation of the same size taken
    from the shim's reuse cache (dev_mem.hip, g_plain_cache)."""
    b = dev_ctx.alloc(3 << 20)
    p = b.ptr
    live = dev_ctx.debug_ptr(p + 100)
    assert "runtime range ok" in live and "own allocation" in live, live
    assert f" M ptr 0x{p:x}" in live or f" R ptr 0x{p:x}" in live, live
    b.free()
    gone = dev_ctx.debug_ptr(p)
    assert f" F ptr 0x{p:x}" in gone and "rc 0" in gone, gone
    assert "own allocation" not in gone, gone


def test_argument_errors(dev_ctx):
    b = dev_ctx.alloc(4096)
    # partial overlap
    assert dev_ctx.reduce("sum", "float32", b.ptr, b.ptr + 4, 100) == xucg_amd.UCS_ERR_INVALID_PARAM
    # not element-aligned
    assert dev_ctx.reduce("sum", "float32", b.ptr + 2, b.ptr + 2050, 10) == xucg_amd.UCS_ERR_INVALID_PARAM
    # float bitwise
    assert dev_ctx.reduce("bxor", "float64", b.ptr, b.ptr + 2048, 10) == xucg_amd.UCS_ERR_UNSUPPORTED
    # multi: non power of two
    assert dev_ctx.reduce_multi("sum", "int32", b, [b, b, b], 0, 10) == xucg_amd.UCS_ERR_INVALID_PARAM
    # fragment outside a staged step
    assert dev_ctx.combine("sum", "int32", 0, np.zeros(4, np.int32), 4) == xucg_amd.UCS_ERR_OUT_OF_RANGE


def test_c2_full_size_fp32_sum(dev_ctx):
    """BASELINE config 2 at full size: 2 x 256 MiB fp32, device-resident,
    bit-exact against the oracle over all 2^26 elements."""
    n = 1 << 26
    bs, bd = dev_ctx.alloc(n * 4), dev_ctx.alloc(n * 4)
    dev_ctx.fill("float32", "round", 0x5EED0000, bs, n)
    dev_ctx.fill("float32", "round", 0x5EED0001, bd, n)
    assert dev_ctx.reduce("sum", "float32", bd, bs, n) == 0
    dev_ctx.sync()
    got = bd.download(np.float32, n)
    want = O.reduce("sum", "float32", O.fill("float32", "round", 0x5EED0000, n),
                    O.fill("float32", "round", 0x5EED0001, n))
    assert (bits(got) == bits(want)).all()


@pytest.mark.parametrize("dt,op", [("float32", "sum"), ("float32", "prod"),
                                   ("float64", "sum"), ("int32", "sum"),
                                   ("float16", "sum"), ("bfloat16", "max"),
                                   ("uint8", "bxor")])
@pytest.mark.parametrize("nsrc", [1, 2, 4, 8, 16])
def test_reduce_multi_recursive_doubling(dev_ctx, dt, op, nsrc):
    n = 5003
    st = O.storage(dt)
    sz = np.dtype(st).itemsize
    dist = "special" if dt.startswith("float") else "round"
    xs = [O.fill(dt, dist, 900 + r, n) for r in range(nsrc)]
    bufs = []
    for r, x in enumerate(xs):
        b = dev_ctx.alloc(n * sz + 64)
        b.upload(x)
        bufs.append(b)
    out = dev_ctx.alloc(n * sz + 64)
    for self_index in sorted({0, nsrc - 1, nsrc // 2}):
        for off in (0, sz):  # aligned and shifted by one element (all agree)
            for b, x in zip(bufs, xs):
                b.upload(x, off)
            srcs = [b.ptr + off for b in bufs]
            rc = dev_ctx.reduce_multi(op, dt, out.ptr + off, srcs, self_index, n)
            assert rc == 0, _lib.last_error()
            dev_ctx.sync()
            got = out.download(st, n, off)
            want = O.reduce_multi(op, dt, xs, self_index)
            assert (bits(got) == bits(want)).all(), (self_index, off)
    # sources disagreeing mod 16 B -> scalar path
    if nsrc > 1:
        for b, x in zip(bufs, xs):
            b.upload(x)
        bufs[0].upload(xs[0], sz)
        srcs = [bufs[0].ptr + sz] + [b.ptr for b in bufs[1:]]
        assert dev_ctx.reduce_multi(op, dt, out.ptr, srcs, 0, n) == 0
        dev_ctx.sync()
        assert (bits(out.download(st, n)) == bits(O.reduce_multi(op, dt, xs, 0))).all()


@pytest.mark.parametrize("pinned", [True, False])
def test_combine_host_pipeline(pinned):
    """Host-resident whole-buffer combine: H2D -> kernel -> D2H in 1 MiB chunks."""
    n = (3 << 20) + 5  # crosses many ring slots, ragged tail
    ctx = xucg_amd.DevContext(device=0, stage_bytes=1 << 20, stage_slots=3)
    try:
        src = O.fill("float32", "round", 41, n)
        dst = O.fill("float32", "round", 42, n)
        want = O.reduce("sum", "float32", src, dst)
        if pinned:
            hs, hd = xucg_amd.HostBuffer(n * 4), xucg_amd.HostBuffer(n * 4)
            vs, vd = hs.view(np.float32, n), hd.view(np.float32, n)
            vs[:] = src
            vd[:] = dst
            assert ctx.combine_host("sum", "float32", hd.ptr, hs.ptr, n) == 0, _lib.last_error()
            got = vd.copy()
        else:
            d = dst.copy()
            assert ctx.combine_host("sum", "float32", d, src, n) == 0, _lib.last_error()
            got = d
        assert (bits(got) == bits(want)).all()
        c = ctx.counters()
        assert c["h2d_bytes"] == 2 * n * 4 and c["d2h_bytes"] == n * 4
    finally:
        ctx.close()


@pytest.mark.parametrize("dt,op", [("float32", "sum"), ("float64", "prod"),
                                   ("int32", "max"), ("float16", "sum")])
def test_staged_fragments_like_the_am_handler(dt, op):
    """Per-step staging: fragments of the reference's AM-short size arrive
    from two peers in interleaved order (a tree fan-in with ep_cnt = 2) and
    are combined in arrival order, exactly like ucg_builtin_step_recv_cb()."""
    ctx = xucg_amd.DevContext(device=0, stage_bytes=64 << 10, stage_slots=4)
    try:
        st = O.storage(dt)
        sz = np.dtype(st).itemsize
        n = 40_000 + 3
        acc = O.fill(dt, "round", 7, n)
        peers = [O.fill(dt, "round", 8 + p, n) for p in range(2)]
        frag = O.frag_length(256, sz)            # (max_short - 8) rounded
        want = acc.copy()
        host = acc.copy()
        assert ctx.stage_begin(host, host.nbytes) == 0
        order = []
        for off in range(0, n * sz, frag):
            for p in range(2):
                order.append((p, off))
        for p, off in order:
            cnt = min(frag, n * sz - off) // sz
            i0 = off // sz
            piece = np.ascontiguousarray(peers[p][i0:i0 + cnt])
            assert ctx.combine(op, dt, off, piece, cnt) == 0, _lib.last_error()
            want[i0:i0 + cnt] = O.reduce(op, dt, piece, want[i0:i0 + cnt])
        assert ctx.stage_end() == 0, _lib.last_error()
        assert (bits(host) == bits(want)).all()
        c = ctx.counters()
        # aggregation: far fewer launches than fragments
        assert c["launches"] < len(order) / 4
    finally:
        ctx.close()


@pytest.mark.parametrize("zcopy", [0, None, 1 << 20])
def test_staged_runs_zero_copy_and_dma_counters(zcopy):
    """Both flush paths of the fragment aggregator give the same bits, and the
    counters tell them apart: runs of at most the zero-copy threshold are read
    by the kernel from the pinned slot (counter 4, no DMA), larger ones are
    copied H2D (counter 2, which also holds stage_begin's mirror copy).
    zcopy: 0 = default 64 KiB, None = never, 1 MiB = every run."""
    ctx = xucg_amd.DevContext(device=0, stage_bytes=64 << 10, stage_slots=3,
                              zcopy_bytes=zcopy)
    try:
        n = 50_000 + 1          # 200 KiB: four 64 KiB slots, the last ragged
        acc = O.fill("float32", "round", 5, n)
        src = O.fill("float32", "round", 6, n)
        host = acc.copy()
        assert ctx.stage_begin(host, host.nbytes) == 0
        frag = O.frag_length(256, 4)
        for off in range(0, n * 4, frag):
            cnt = min(frag, n * 4 - off) // 4
            assert ctx.combine("sum", "float32", off, src[off // 4: off // 4 + cnt],
                               cnt) == 0, _lib.last_error()
        assert ctx.stage_end() == 0, _lib.last_error()
        assert (bits(host) == bits(O.reduce("sum", "float32", src, acc))).all()
        c = ctx.counters()
        if zcopy is None:
            assert c["zcopy_bytes"] == 0 and c["h2d_bytes"] == 2 * n * 4
        else:
            assert c["zcopy_bytes"] == n * 4 and c["h2d_bytes"] == n * 4
        assert c["d2h_bytes"] == n * 4
    finally:
        ctx.close()


@pytest.mark.parametrize("completion", ["signal", "sync"])
@pytest.mark.parametrize("recv", ["device", "pinned", "pageable"])
def test_stage_end_completion_word(completion, recv):
    """stage_end's two completion waits give the same bits for every recv
    buffer kind. With "signal" a device or pinned result is waited for on the
    pinned completion word (counter 5 counts the waits); a pageable result is
    always waited for by the runtime (its D2H may end in a host-side copy).
    Steps of one fragment (the small-step floor) and of many, 3 steps each so
    the sequence number advances and a stale word never passes for a new one."""
    ctx = xucg_amd.DevContext(device=0, stage_bytes=64 << 10, stage_slots=3,
                              completion=completion)
    try:
        for n in (64, 30_001):
            acc = O.fill("float64", "round", 21, n)
            srcs = [O.fill("float64", "round", 22 + k, n) for k in range(3)]
            want = acc.copy()
            hb = db = None
            if recv == "device":
                db = ctx.alloc(n * 8)
                db.upload(acc)
                target = db.ptr
            elif recv == "pinned":
                hb = xucg_amd.HostBuffer(n * 8)
                hv = hb.view(np.float64, n)
                hv[:] = acc
                target = hb.ptr
            else:
                hv = acc.copy()
                target = hv
            before = ctx.counters()["signal_waits"]
            frag = O.frag_length(8192, 8)
            for src in srcs:
                assert ctx.stage_begin(target, n * 8) == 0, _lib.last_error()
                for off in range(0, n * 8, frag):
                    cnt = min(frag, n * 8 - off) // 8
                    piece = np.ascontiguousarray(src[off // 8: off // 8 + cnt])
                    assert ctx.combine("sum", "float64", off, piece, cnt) == 0
                assert ctx.stage_end() == 0, _lib.last_error()
                want = O.reduce("sum", "float64", src, want)
                got = db.download(np.float64, n) if db else hv.copy()
                assert (bits(got) == bits(want)).all(), (n, recv, completion)
            waits = ctx.counters()["signal_waits"] - before
            expect = 3 if completion == "signal" and recv != "pageable" else 0
            assert waits == expect, (waits, expect)
            if hb:
                hb.free()
            if db:
                db.free()
    finally:
        ctx.close()


@pytest.mark.parametrize("completion", ["signal", "sync"])
def test_whole_buffer_combine_inside_a_staged_step(completion):
    """Another op of the group combines a whole host buffer (the per-fragment
    path of a step that found the staging busy, builtin_ops.c) while a staged
    step holds a pending run in a ring slot. The whole-buffer combine takes
    ring slots and frees them all at its end; the staged run must have been
    flushed first, or the step's next run lands in its slot and overwrites it."""
    ctx = xucg_amd.DevContext(device=0, stage_bytes=4096, stage_slots=3,
                              completion=completion)
    try:
        n = 2048
        acc = O.fill("float32", "round", 31, n)
        a = O.fill("float32", "round", 32, 256)
        b = O.fill("float32", "round", 33, 256)
        host = acc.copy()
        assert ctx.stage_begin(host, host.nbytes) == 0
        assert ctx.combine("sum", "float32", 0, a, 256) == 0          # run in slot 0
        hs, hd0 = O.fill("float32", "round", 34, n), O.fill("float32", "round", 35, n)
        hd = hd0.copy()
        assert ctx.combine_host("sum", "float32", hd, hs, n) == 0, _lib.last_error()
        assert ctx.combine("sum", "float32", 4096, b, 256) == 0       # a new run
        assert ctx.stage_end() == 0, _lib.last_error()
        want = acc.copy()
        want[:256] = O.reduce("sum", "float32", a, want[:256])
        want[1024:1280] = O.reduce("sum", "float32", b, want[1024:1280])
        assert (bits(host) == bits(want)).all()
        assert (bits(hd) == bits(O.reduce("sum", "float32", hs, hd0))).all()
    finally:
        ctx.close()


def test_empty_staged_step_waits_for_nothing(dev_ctx):
    """A step with no fragment queues nothing, and its stage_end returns at
    once in either completion mode (no signal launch)."""
    b = dev_ctx.alloc(4096)
    before = dev_ctx.counters()["signal_waits"]
    for _ in range(3):
        assert dev_ctx.stage_begin(b, 4096) == 0
        assert dev_ctx.stage_end() == 0
    assert dev_ctx.counters()["signal_waits"] == before


def test_completion_mode_rejects_unknown():
    p = _lib.DevCtxParams(0, None, 0, 0, 0, 7)
    import ctypes
    h = ctypes.c_void_p()
    assert _lib.dev().ucg_builtin_dev_ctx_create(ctypes.byref(p), ctypes.byref(h)) == \
        xucg_amd.UCS_ERR_INVALID_PARAM


def test_staged_contiguous_fragments_one_launch_per_slot():
    ctx = xucg_amd.DevContext(device=0, stage_bytes=1 << 20, stage_slots=2)
    try:
        n = 1 << 20  # 4 MiB of fp32 = 4 slots
        acc = O.fill("float32", "exact", 1, n)
        src = O.fill("float32", "exact", 2, n)
        host = acc.copy()
        assert ctx.stage_begin(host, host.nbytes) == 0
        frag = O.frag_length(8192, 4)
        for off in range(0, n * 4, frag):
            cnt = min(frag, n * 4 - off) // 4
            assert ctx.combine("sum", "float32", off, src[off // 4: off // 4 + cnt], cnt) == 0
        assert ctx.stage_end() == 0
        assert (bits(host) == bits(O.reduce("sum", "float32", src, acc))).all()
        assert ctx.counters()["launches"] == 4
    finally:
        ctx.close()


def test_profile_hook_and_counters(dev_ctx):
    n = 1 << 22
    bs, bd = dev_ctx.alloc(n * 4), dev_ctx.alloc(n * 4)
    dev_ctx.fill("float32", "exact", 1, bs, n)
    dev_ctx.fill("float32", "exact", 2, bd, n)
    before = dev_ctx.counters()
    us = dev_ctx.profile_reduce("sum", "float32", bd, bs, n, 10)
    after = dev_ctx.counters()
    assert 0 < us < 10_000
    assert after["launches"] - before["launches"] == 10
    assert after["combined_bytes"] - before["combined_bytes"] == 10 * 3 * n * 4


@pytest.mark.gpu
@pytest.mark.parametrize("shareable", [True, False])
def test_ipc_keys_name_allocations_and_retire_on_free(dev_ctx, shareable):
    """A key names the allocation, not the address (round 4):
    exporting one allocation twice gives one key; importing it in the
    exporting process maps the allocation itself; freeing the allocation
    retires the key, so importing it afterwards is refused with
    UCS_ERR_NO_RESOURCE ("stale key") even when a new allocation of the same
    size sits at the same address - and that one has a key of its own."""
    from xucg_amd import _lib
    nbytes = 6 << 20
    a = dev_ctx.alloc(nbytes, shareable=shareable)
    assert bool(_lib.dev().ucg_builtin_dev_is_shareable(a.ptr)) == shareable
    a.upload(np.arange(16, dtype=np.int64))
    key = dev_ctx.ipc_export(a.ptr + 4096)
    assert dev_ctx.ipc_export(a.ptr + 4096) == key
    p = dev_ctx.ipc_import(key)
    assert p == a.ptr + 4096
    dev_ctx.ipc_release(p)
    pa = a.ptr
    a.free()
    with pytest.raises(xucg_amd.UcsError) as e:
        dev_ctx.ipc_import(key)
    assert e.value.status == -2 and "stale key" in str(e.value)
    b = dev_ctx.alloc(nbytes, shareable=shareable)
    try:
        key_b = dev_ctx.ipc_export(b.ptr + 4096)
        assert key_b != key, (hex(pa), hex(b.ptr))
        with pytest.raises(xucg_amd.UcsError):
            dev_ctx.ipc_import(key)                   # still stale
        q = dev_ctx.ipc_import(key_b)
        assert q == b.ptr + 4096
        dev_ctx.ipc_release(q)
    finally:
        b.free()


@pytest.mark.gpu
def test_shareable_allocations_never_reuse_an_address(dev_ctx):
    """Round 4: an address mapped again to other physical memory
    took DMA writes into the previous allocation's pages in 98 of 200 rounds
    (tools/va_reuse_probe). The shim's shareable allocations never reuse an
    address: 60 rounds of allocate, DMA upload, kernel read-back (copy_multi
    into a second buffer), free - every address new, every read right."""
    seen = set()
    n = (6 << 20) // 4
    out = dev_ctx.alloc(n * 4, shareable=True)
    try:
        for r in range(60):
            b = dev_ctx.alloc(n * 4, shareable=True)
            assert b.ptr not in seen, r
            seen.add(b.ptr)
            b.upload(np.full(n, r + 1, np.uint32))                 # DMA write
            assert dev_ctx.copy_multi([out.ptr], [b.ptr], n * 4) == 0   # kernel read
            dev_ctx.sync()
            got = out.download(np.uint32, n)
            assert (got == r + 1).all(), (r, int((got != r + 1).sum()))
            b.free()
    finally:
        out.free()


@pytest.mark.gpu
def test_retired_address_ranges_are_counted_and_capped(dev_ctx):
    """the ranges that freed shareable allocations leave
    behind are counted (ucg_builtin_dev_mem_stats) and bounded. Every churned
    6 MiB allocation retires exactly its bytes; with the cap set just past the
    current total, the allocation that would cross it fails with
    UCS_ERR_EXCEEDS_LIMIT and an error that names the knob, and nothing is
    retired by the failure."""
    from xucg_amd import _lib
    nbytes = 6 << 20
    s0 = _lib.mem_stats()
    assert s0["va_retired_max"] == 64 << 40            # the default cap, 64 TiB
    for r in range(5):
        b = dev_ctx.alloc(nbytes, shareable=True)
        assert _lib.mem_stats()["shareable_live_bytes"] >= nbytes
        b.free()
        s = _lib.mem_stats()
        assert s["va_retired_bytes"] == s0["va_retired_bytes"] + (r + 1) * nbytes, (r, s)
        assert s["va_retired_ranges"] == s0["va_retired_ranges"] + r + 1
    assert dev_ctx.counters()["va_retired_bytes"] == s["va_retired_bytes"]
    _lib.dev().ucg_builtin_dev_set_va_retired_max(s["va_retired_bytes"] + 2 * nbytes)
    try:
        for _ in range(2):                             # two more fit under the cap
            dev_ctx.alloc(nbytes, shareable=True).free()
        with pytest.raises(MemoryError) as e:
            dev_ctx.alloc(nbytes, shareable=True)
        assert "UCX_BUILTIN_DEV_VA_RETIRED_MAX" in str(e.value), str(e.value)
        assert _lib.mem_stats()["va_retired_bytes"] == s["va_retired_bytes"] + 2 * nbytes
    finally:
        _lib.dev().ucg_builtin_dev_set_va_retired_max(0)
    assert _lib.mem_stats()["va_retired_max"] == 64 << 40
    dev_ctx.alloc(nbytes, shareable=True).free()      # room again under the default


@pytest.mark.gpu
def test_parked_memory_is_never_handed_out_again(dev_ctx):
    """an exported buffer a peer may still read (an op that ended
    before every peer was done) is parked, not freed: its key is refused from
    then on, and its memory is never handed out again - not by the reuse
    cache, which takes every other freed allocation (exported or not: the
    same memory at the same address keeps the runtime's hipIpc mappings of
    it right)."""
    from xucg_amd import _lib
    nbytes = 6 << 20
    a = dev_ctx.alloc(nbytes)
    key = dev_ctx.ipc_export(a.ptr)
    pa = a.ptr
    p0 = _lib.mem_stats()["parked_bytes"]
    _lib.dev().ucg_builtin_dev_park(dev_ctx.handle, pa)
    a.ptr = None                                      # parked: not ours to free
    assert _lib.mem_stats()["parked_bytes"] == p0 + nbytes
    with pytest.raises(xucg_amd.UcsError) as e:
        dev_ctx.ipc_import(key)
    assert e.value.status == -2
    got = [dev_ctx.alloc(nbytes) for _ in range(3)]
    assert pa not in [b.ptr for b in got]
    for b in got:
        b.free()
    # an exported allocation freed the normal way is reused whole
    b = dev_ctx.alloc(nbytes)
    dev_ctx.ipc_export(b.ptr)
    bp = b.ptr
    c1 = _lib.mem_stats()["plain_cache_bytes"]
    b.free()
    assert _lib.mem_stats()["plain_cache_bytes"] == c1 + nbytes
    c = dev_ctx.alloc(nbytes)
    assert c.ptr == bp and _lib.mem_stats()["plain_cache_bytes"] == c1
    c.free()


@pytest.mark.gpu
def test_exported_allocations_kept_past_the_cache_bound():
    """With the reuse cache's bound at 0 (UCX_BUILTIN_DEV_CACHE_BYTES=0, read
    once per process: a child process), a never-exported allocation is freed
    at once, and one that was ever exported is kept all the same - given back
    to the runtime, its address could come back with other memory and peers'
    fresh hipIpc imports of it map another process's buffer.
    The oom drain gives back only the never-exported ones. A smaller request,
    at least half the size, takes the kept allocation whole, so a caller whose
    sizes vary does not add one kept allocation per size."""
    import subprocess
    import sys
    code = r"""
import xucg_amd
from xucg_amd import _lib
ctx = xucg_amd.DevContext(device=0)
n = 6 << 20
a = ctx.alloc(n); a.free()
assert _lib.mem_stats()["plain_cache_bytes"] == 0, _lib.mem_stats()
b = ctx.alloc(n); ctx.ipc_export(b.ptr); pb = b.ptr; b.free()
assert _lib.mem_stats()["plain_cache_bytes"] == n, _lib.mem_stats()
c = ctx.alloc(n)
assert c.ptr == pb and _lib.mem_stats()["plain_cache_bytes"] == 0
c.free()                        # still the ever-exported allocation: kept again
assert _lib.mem_stats()["plain_cache_bytes"] == n, _lib.mem_stats()
d = ctx.alloc(4 << 20)          # smaller, at least half its size: the same memory
assert d.ptr == pb and _lib.mem_stats()["plain_cache_bytes"] == 0, _lib.mem_stats()
d.free()                        # back whole, at its own size
assert _lib.mem_stats()["plain_cache_bytes"] == n, _lib.mem_stats()
e = ctx.alloc(2 << 20)          # under half: a new allocation, freed at once
assert e.ptr != pb and _lib.mem_stats()["plain_cache_bytes"] == n, _lib.mem_stats()
e.free()
assert _lib.mem_stats()["plain_cache_bytes"] == n, _lib.mem_stats()
ctx.close()
print("OK")
"""
    env = dict(os.environ, UCX_BUILTIN_DEV_CACHE_BYTES="0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]


@pytest.mark.gpu
def test_kept_memory_is_capped_and_slack_counted():
    """memory the shim keeps for the life of the process
    (ever-exported allocations, live or cached, and parked ones) is bounded by
    UCX_BUILTIN_DEV_KEEP_MAX: the export that would cross it fails with
    UCS_ERR_EXCEEDS_LIMIT naming the knob, a warning is printed once past
    half, and nothing is counted for the refused export. A cached exported
    allocation handed out for a smaller request counts its extra bytes as
    slack until it is freed. Only never-exported bytes count against
    UCX_BUILTIN_DEV_CACHE_BYTES."""
    import subprocess
    import sys
    code = r"""
import xucg_amd
from xucg_amd import _lib
ctx = xucg_amd.DevContext(device=0)
n = 6 << 20
s0 = _lib.mem_stats()
assert s0["keep_max"] == 20 << 20 and s0["kept_bytes"] == 0, s0
bufs = [ctx.alloc(n) for _ in range(4)]
for b in bufs[:3]:
    ctx.ipc_export(b.ptr)
s = _lib.mem_stats()
assert s["kept_bytes"] == 3 * n, s
try:
    ctx.ipc_export(bufs[3].ptr)
    raise SystemExit("export past the keep cap succeeded")
except xucg_amd.UcsError as e:
    assert e.status == -21 and "UCX_BUILTIN_DEV_KEEP_MAX" in str(e), str(e)
assert _lib.mem_stats()["kept_bytes"] == 3 * n
bufs[3].free()                          # never exported: bounded cache (0 here): freed
s = _lib.mem_stats()
assert s["plain_cache_bytes"] == 0 and s["plain_cache_exported_bytes"] == 0, s
bufs[0].free()                          # exported: kept whatever the cache bound
s = _lib.mem_stats()
assert s["plain_cache_exported_bytes"] == n and s["plain_cache_bytes"] == n, s
assert s["kept_bytes"] == 3 * n, s
small = ctx.alloc(4 << 20)              # takes the kept 6 MiB one: 2 MiB slack
s = _lib.mem_stats()
assert s["slack_bytes"] == 2 << 20 and s["plain_cache_exported_bytes"] == 0, s
small.free()
assert _lib.mem_stats()["slack_bytes"] == 0
for b in bufs[1:3]:
    b.free()
assert _lib.mem_stats()["kept_bytes"] == 3 * n
ctx.close()
print("OK")
"""
    env = dict(os.environ, UCX_BUILTIN_DEV_KEEP_MAX="20m", UCX_BUILTIN_DEV_CACHE_BYTES="0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    assert p.stderr.count("past half of UCX_BUILTIN_DEV_KEEP_MAX") == 1, p.stderr[-2000:]


@pytest.mark.gpu
def test_free_waits_for_the_shims_streams_not_the_device():
    """ucg_builtin_dev_free (plain and shareable memory)
    waits for the work queued on the streams of the shim's contexts, not for
    the whole device: with a 1.5-second kernel running on an unrelated torch
    stream, a free returns in milliseconds (round 5's hipDeviceSynchronize
    waited for it). Work of the shim's own stream on the buffer is still
    waited for: a combine queued just before the free has completed, with
    the right result, before the same memory is handed out again."""
    import subprocess
    import sys
    code = r"""
import time
import numpy as np
import torch
import xucg_amd
torch.cuda.init()
ctx = xucg_amd.DevContext(device=0)
n = 6 << 20
side = torch.cuda.Stream()
with torch.cuda.stream(side):
    torch.cuda._sleep(int(1.5 * 2.4e9))          # ~1.5 s of one wave spinning
t_long = time.perf_counter()
out = {}
for kind in ("plain", "shareable"):
    b = ctx.alloc(n, shareable=(kind == "shareable"))
    t0 = time.perf_counter()
    b.free()
    out[kind] = time.perf_counter() - t0
assert not side.query(), "the side kernel ended before the frees were timed"
# the shim's own work on a buffer is waited for before its memory is reused
cnt = 1 << 20
a, d = ctx.alloc(cnt * 4), ctx.alloc(cnt * 4)
ctx.fill("float32", "exact", 7, a.ptr, cnt)
ctx.fill("float32", "exact", 8, d.ptr, cnt)
want = a.download(np.float32, cnt).astype(np.float64) + d.download(np.float32, cnt)
pd = d.ptr
assert ctx.reduce("sum", "float32", d.ptr, a.ptr, cnt) == 0
d.free()
e = ctx.alloc(cnt * 4)
assert e.ptr == pd                                # the same memory, reused
got = e.download(np.float32, cnt)
assert np.array_equal(got.astype(np.float64), want)
side.synchronize()
print("FREE_S", out, "side kernel", round(time.perf_counter() - t_long, 3))
assert max(out.values()) < 0.5, out
ctx.close()
print("OK")
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=180, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]


@pytest.mark.gpu
def test_plain_allocations_reused_whole(dev_ctx):
    """Round 4: a freed ucg_builtin_dev_malloc allocation is
    kept and handed out again, whole, for the next allocation of its size - the
    same address on the same memory, never a remap - and its old key is
    refused. 60 rounds of allocate, DMA upload, kernel read-back, free: one
    address throughout, every read right. Round 5: exported allocations
    included - given back to the runtime, the address would return with other
    memory, and peers' new imports of it could map the old memory
    (tools/va_reuse_probe ipc)."""
    n = (6 << 20) // 4
    out = dev_ctx.alloc(n * 4)
    first = None
    try:
        for r in range(60):
            b = dev_ctx.alloc(n * 4)
            if first is None:
                first = b.ptr
                key = dev_ctx.ipc_export(b.ptr)
            assert b.ptr == first, (r, hex(b.ptr), hex(first))
            assert " R ptr" in dev_ctx.debug_ptr(b.ptr) or r == 0
            b.upload(np.full(n, r + 1, np.uint32))                 # DMA write
            assert dev_ctx.copy_multi([out.ptr], [b.ptr], n * 4) == 0   # kernel read
            dev_ctx.sync()
            got = out.download(np.uint32, n)
            assert (got == r + 1).all(), (r, int((got != r + 1).sum()))
            b.free()
        with pytest.raises(xucg_amd.UcsError) as e:
            dev_ctx.ipc_import(key)
        assert e.value.status == -2
    finally:
        out.free()


@pytest.mark.gpu
def test_ipc_import_rejects_foreign_and_dead_keys(dev_ctx):
    """A blob that is no key, and a key whose exporter's key server is gone,
    fail loudly at import."""
    with pytest.raises(xucg_amd.UcsError) as e:
        dev_ctx.ipc_import(bytes(96))
    assert e.value.status == -5
    a = dev_ctx.alloc(2 << 20, shareable=True)
    try:
        key = bytearray(dev_ctx.ipc_export(a.ptr))
        key[12:16] = (0x7ffffffe).to_bytes(4, "little")     # another (absent) pid
        with pytest.raises(xucg_amd.UcsError) as e:
            dev_ctx.ipc_import(bytes(key))
        assert "key server is gone" in str(e.value)
    finally:
        a.free()


@pytest.mark.gpu
def test_mem_kind(dev_ctx):
    """ucg_builtin_dev_mem_kind: pageable host 0, pinned host 1, device 2
    (also at an interior offset of a device allocation)."""
    from xucg_amd import _lib
    f = _lib.dev().ucg_builtin_dev_mem_kind
    a = np.zeros(64, np.float32)
    hb = xucg_amd.HostBuffer(4096)
    db = dev_ctx.alloc(4096)
    sb = dev_ctx.alloc(4096, shareable=True)     # HIP virtual memory
    try:
        assert f(a.ctypes.data) == 0
        assert f(hb.ptr) == 1
        assert f(db.ptr) == 2 and f(db.ptr + 1000) == 2
        assert f(sb.ptr) == 2 and f(sb.ptr + 1000) == 2
    finally:
        hb.free()
        db.free()
        sb.free()


@pytest.mark.gpu
@pytest.mark.parametrize("dt,count,multi", [
    ("uint8", (1 << 32) + 4099, False),     # past 4 GiB per operand
    ("float32", (1 << 32) + 5, False),      # past 2^32 elements (16 GiB per operand)
    ("uint8", (1 << 36) + 4099, False),     # past 2^32 16-B vectors: several dispatches
    ("uint8", (1 << 35) + 4099, True)])     # the multi-operand kernel (2 operands)
def test_max_size_operands(dev_ctx, dt, count, multi):
    """Maximum sizes on a 288 GB device: 64-bit indexing and the chunking of
    launches whose work-item count would not fit a dispatch packet. Windows
    around every boundary (4 GiB, 2^32 elements, each 2^31-vector chunk) and
    the ragged end are checked bit for bit against the oracle."""
    st = O.storage(dt)
    sz = np.dtype(st).itemsize
    nbytes = count * sz
    src, dst = dev_ctx.alloc(nbytes), dev_ctx.alloc(nbytes)
    try:
        dev_ctx.fill(dt, "round", 31, src, count)
        dev_ctx.fill(dt, "round", 32, dst, count)
        dev_ctx.sync()
        chunk = (1 << 31) * (16 // sz)
        bounds = sorted({(1 << 32) // sz, 1 << 32, chunk, 2 * chunk, count})
        starts = [0] + [max(0, b - 2048) for b in bounds if b <= count]
        wins = [(a, min(count, a + 4096)) for a in starts]
        before = [(src.download(st, b - a, a * sz), dst.download(st, b - a, a * sz))
                  for a, b in wins]
        if multi:
            assert dev_ctx.reduce_multi("sum", dt, dst, [src, dst], 1, count) == 0, \
                _lib.last_error()
        else:
            dev_ctx.reduce_checked("sum", dt, dst, src, count)
        dev_ctx.sync()
        for (a, b), (s, d) in zip(wins, before):
            got = dst.download(st, b - a, a * sz)
            # reduce_multi with self = 1: V(1, 1) = x0 (op) x1, src = member 0
            want = O.reduce("sum", dt, s, d)
            assert (O.bits(got) == O.bits(want)).all(), (dt, count, a)
    finally:
        src.free()
        dst.free()


@pytest.mark.gpu
@pytest.mark.parametrize("nsrc,shard,offset", [(1, 4096, 0), (4, 1 << 20, 0), (8, 100_000, 0),
                                               (16, 4099, 0), (3, 65536, 4), (8, 33, 1),
                                               (1, 4099, 0), (1, 7, 0), (1, (1 << 20) + 9, 0)])
def test_gather_multi(dev_ctx, nsrc, shard, offset):
    """One-shot all-gather copy: dst[r * shard:] = srcs[r][:shard] (vector path
    when every row starts on 16 B, whatever its length, byte path otherwise); then again with one row's
    source NULL (a member's own shard), which must stay untouched."""
    srcs = [np.frombuffer(np.random.default_rng(r).bytes(shard), np.uint8) for r in range(nsrc)]
    bufs = [dev_ctx.alloc(shard + 16) for _ in range(nsrc)]
    out = dev_ctx.alloc(nsrc * shard + 16)
    try:
        for b, s in zip(bufs, srcs):
            b.upload(s, offset)
        rc = dev_ctx.gather_multi(out.ptr + offset, [b.ptr + offset for b in bufs], shard)
        assert rc == 0, _lib.last_error()
        dev_ctx.sync()
        got = out.download(np.uint8, nsrc * shard, offset)
        assert (got == np.concatenate(srcs)).all()
        if nsrc > 1:
            skip = nsrc // 2
            out.upload(np.full(nsrc * shard, 0xA5, np.uint8), offset)
            ptrs = [None if r == skip else b.ptr + offset for r, b in enumerate(bufs)]
            assert dev_ctx.gather_multi(out.ptr + offset, ptrs, shard) == 0, _lib.last_error()
            dev_ctx.sync()
            got = out.download(np.uint8, nsrc * shard, offset).reshape(nsrc, shard)
            for r in range(nsrc):
                if r == skip:
                    assert (got[r] == 0xA5).all(), "NULL row overwritten"
                else:
                    assert (got[r] == srcs[r]).all(), r
        assert dev_ctx.gather_multi(out.ptr, [None] * nsrc, shard) == \
            xucg_amd.UCS_ERR_INVALID_PARAM
    finally:
        for b in bufs:
            b.free()
        out.free()


@pytest.mark.gpu
@pytest.mark.parametrize("nsrc,shard,offset", [(2, 4099, 0), (8, 33, 5), (5, (1 << 20) + 3, 12),
                                               (16, 100_003, 7), (3, 15, 9)])
def test_gather_multi_phase_matched_rows(dev_ctx, nsrc, shard, offset):
    """Rows of a ragged length, each source placed in its destination row's
    16-B phase (the one-shot all-gather over buffers at one common offset):
    the vector kernel with per-row byte heads and tails. Guard bytes on both
    sides of the output must stay untouched."""
    srcs = [np.frombuffer(np.random.default_rng(40 + r).bytes(shard), np.uint8)
            for r in range(nsrc)]
    phase = [(offset + r * shard) % 16 for r in range(nsrc)]
    bufs = [dev_ctx.alloc(shard + 32) for _ in range(nsrc)]
    out = dev_ctx.alloc(nsrc * shard + 64)
    try:
        for b, s_, ph in zip(bufs, srcs, phase):
            b.upload(s_, ph)
        out.upload(np.full(nsrc * shard + 64, 0x5A, np.uint8))
        rc = dev_ctx.gather_multi(out.ptr + 16 + offset,
                                  [b.ptr + ph for b, ph in zip(bufs, phase)], shard)
        assert rc == 0, _lib.last_error()
        dev_ctx.sync()
        raw = out.download(np.uint8, nsrc * shard + 64)
        got = raw[16 + offset:16 + offset + nsrc * shard]
        assert (got == np.concatenate(srcs)).all()
        assert (raw[:16 + offset] == 0x5A).all() and (raw[16 + offset + nsrc * shard:] == 0x5A).all()
    finally:
        for b in bufs:
            b.free()
        out.free()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["int8", "float16", "float32", "float64"])
def test_line_heads(dev_ctx, dt):
    """The ragged head runs to dst's next 128-B line (up to 127 B: more
    lanes than one wave for int8). dst at every element offset within a
    line, src in phase, 16-B-in-phase but not line-in-phase (the XCD-aware
    map), and out of phase; counts shorter and longer than the head. Guard
    bytes around dst stay untouched. Then the multi-operand and tree kernels
    with dst off a line."""
    st = O.storage(dt)
    sz = np.dtype(st).itemsize
    counts = [1, 63, 64, 65, 127, 128 // sz + 3, 1000, 64 * 64 + 17]
    cap = max(counts) * sz + 512
    bs, bd = dev_ctx.alloc(cap), dev_ctx.alloc(cap + 256)
    try:
        for count in counts:
            nb = count * sz
            src = O.fill(dt, "round", 500 + count, count)
            dst = O.fill(dt, "round", 600 + count, count)
            want = O.reduce("sum", dt, src, dst)
            for doff in range(0, 128, sz if sz > 1 else 7):
                for delta in (0, 16, 48, 4 * sz if sz < 4 else sz):
                    soff = (doff + delta) % 128 + 64
                    do = 128 + doff
                    bd.upload(np.full(do + nb + 64, 0x3C, np.uint8))
                    bd.upload(dst, do)
                    bs.upload(src, soff)
                    dev_ctx.reduce_checked("sum", dt, bd.ptr + do, bs.ptr + soff, count)
                    dev_ctx.sync()
                    raw = bd.download(np.uint8, do + nb + 64)
                    got = raw[do:do + nb].view(st)
                    assert (O.bits(got) == O.bits(want)).all(), (count, doff, delta)
                    assert (raw[:do] == 0x3C).all() and (raw[do + nb:] == 0x3C).all(), \
                        (count, doff, delta, "guard bytes overwritten")
    finally:
        bs.free()
        bd.free()
    # multi-operand and tree kernels, dst off a line, sources in its 16-B phase
    count = 64 * 64 * 3 + 5
    xs = [O.fill(dt, "round", 700 + r, count) for r in range(4)]
    bufs = [dev_ctx.alloc(count * sz + 512) for _ in range(5)]
    try:
        for doff in (sz, 48, 64 + sz, 112):
            for r in range(4):
                bufs[r].upload(xs[r], doff + 16 * (r % 2))
            ptrs = [bufs[r].ptr + doff + 16 * (r % 2) for r in range(4)]
            assert dev_ctx.reduce_multi("sum", dt, bufs[4].ptr + doff, ptrs, 1, count) == 0, \
                _lib.last_error()
            dev_ctx.sync()
            got = bufs[4].download(st, count, doff)
            assert (O.bits(got) == O.bits(O.reduce_multi("sum", dt, xs, 1))).all(), ("multi", doff)
            assert dev_ctx.reduce_tree("sum", dt, bufs[4].ptr + doff, ptrs, count) == 0, \
                _lib.last_error()
            dev_ctx.sync()
            got = bufs[4].download(st, count, doff)
            assert (O.bits(got) == O.bits(O.tree_reduce("sum", dt, xs, root=0))).all(), \
                ("tree", doff)
    finally:
        for b in bufs:
            b.free()


@pytest.mark.gpu
def test_row_copy_every_phase_pair(dev_ctx):
    """The row copy behind gather_multi and copy_multi for every (source
    phase, destination phase) pair mod 16 B and lengths around the head,
    tail and wave boundaries: in phase it is the vector path with byte heads
    and tails, out of phase the realigning path (aligned loads, next-lane
    shuffle, funnel shift). Guard bytes around the output stay untouched;
    the source sits flush with the end of its allocation once per case."""
    lens = [1, 15, 16, 17, 1023, 1024 + 5, 64 * 16 * 3 + 7, 100_003]
    cap = max(lens) + 64
    sb, db = dev_ctx.alloc(cap), dev_ctx.alloc(cap + 64)
    rng = np.random.default_rng(77)
    try:
        for nb in lens:
            data = np.frombuffer(rng.bytes(nb), np.uint8)
            for sp in range(16):
                for dp in range(16):
                    for at_end in (False, True):
                        so = ((cap - nb - sp) // 16) * 16 + sp if at_end else sp
                        sb.upload(data, so)
                        db.upload(np.full(cap + 64, 0xC3, np.uint8))
                        do = 16 + dp
                        if (sp + dp + nb) % 2:
                            rc = dev_ctx.gather_multi(db.ptr + do, [sb.ptr + so], nb)
                        else:
                            rc = dev_ctx.copy_multi([db.ptr + do], [sb.ptr + so], nb)
                        assert rc == 0, _lib.last_error()
                        dev_ctx.sync()
                        raw = db.download(np.uint8, cap + 64)
                        assert (raw[do:do + nb] == data).all(), (nb, sp, dp, at_end)
                        assert (raw[:do] == 0xC3).all() and (raw[do + nb:] == 0xC3).all(), \
                            (nb, sp, dp, at_end, "guard bytes overwritten")
    finally:
        sb.free()
        db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("n,nbytes,offset", [(1, 4096, 0), (7, 1 << 20, 0), (16, 100_000, 0),
                                             (5, 4099, 0), (3, 65536, 4), (8, 33, 1),
                                             (4, 15, 0), (2, (1 << 20) + 7, 0), (5, 4099, 7),
                                             (3, 100_001, 13)])
def test_copy_multi(dev_ctx, n, nbytes, offset):
    """n independent copies in one launch; sources repeat (pairs 0 and 1 read
    the same source, as the push all-gather's broadcast does)."""
    srcs = [np.frombuffer(np.random.default_rng(10 + r).bytes(nbytes), np.uint8)
            for r in range(n)]
    sbufs = [dev_ctx.alloc(nbytes + 16) for _ in range(n)]
    dbufs = [dev_ctx.alloc(nbytes + 16) for _ in range(n)]
    try:
        for b, s in zip(sbufs, srcs):
            b.upload(s, offset)
        src_ptrs = [b.ptr + offset for b in sbufs]
        if n > 1:
            src_ptrs[1] = src_ptrs[0]
            srcs[1] = srcs[0]
        rc = dev_ctx.copy_multi([b.ptr + offset for b in dbufs], src_ptrs, nbytes)
        assert rc == 0, _lib.last_error()
        dev_ctx.sync()
        for b, s in zip(dbufs, srcs):
            assert (b.download(np.uint8, nbytes, offset) == s).all()
    finally:
        for b in sbufs + dbufs:
            b.free()


@pytest.mark.gpu
def test_gather_multi_split_dispatch(dev_ctx):
    """16 rows of 2^31 + 48 bytes: past 2^31 / 16 vectors per row, so the
    copy takes two dispatches (work-items are counted in 32 bits). The rows
    alias one source buffer at 64-B steps; windows around the split and the
    ends of every row are compared byte for byte."""
    nsrc, shard = 16, (1 << 31) + 48
    src = dev_ctx.alloc(shard + 64 * nsrc)
    out = dev_ctx.alloc(nsrc * shard)
    try:
        dev_ctx.fill("uint8", "round", 77, src, shard + 64 * nsrc)
        rc = dev_ctx.gather_multi(out, [src.ptr + 64 * r for r in range(nsrc)], shard)
        assert rc == 0, _lib.last_error()
        dev_ctx.sync()
        split = (((1 << 31) // nsrc) // 64 * 64) * 16    # bytes per row, first dispatch
        for r in range(nsrc):
            for a in (0, split - 4096, shard - 4096):
                got = out.download(np.uint8, 4096, r * shard + a)
                want = src.download(np.uint8, 4096, 64 * r + a)
                assert (got == want).all(), (r, a)
    finally:
        src.free()
        out.free()


@pytest.mark.gpu
def test_random_cases_against_oracle(dev_ctx):
    """Fuzz: 300 random (dtype, op, distribution, count, src offset, dst
    offset) cases through ucg_builtin_dev_reduce, each bit-exact against the
    oracle. Offsets are whole elements from 0 to 15, so src and dst are often
    misaligned relative to each other (scalar kernel) or to 16 B (head/tail);
    counts from 0 to 70,000."""
    rng = np.random.default_rng(20261015)
    cap = 70_000 * 8 + 256
    bs, bd = dev_ctx.alloc(cap), dev_ctx.alloc(cap)
    try:
        pairs = [(dt, op) for dt in O.DTYPES for op in O.OPS if O.is_supported(dt, op)]
        for case in range(300):
            dt, op = pairs[rng.integers(len(pairs))]
            dist = ("exact", "round", "special")[rng.integers(3)]
            count = int(rng.choice([0, 1, 2, 3, 7, 15, 16, 17, 255, 4099,
                                    int(rng.integers(1, 70_000))]))
            st = O.storage(dt)
            sz = np.dtype(st).itemsize
            so, do = int(rng.integers(16)) * sz, int(rng.integers(16)) * sz
            src = O.fill(dt, dist, 1000 + case, count)
            dst = O.fill(dt, dist, 5000 + case, count)
            bs.upload(src, so)
            bd.upload(dst, do)
            dev_ctx.reduce_checked(op, dt, bd.ptr + do, bs.ptr + so, count)
            dev_ctx.sync()
            got = bd.download(st, count, do)
            want = O.reduce(op, dt, src, dst)
            assert (O.bits(got) == O.bits(want)).all(), (case, dt, op, dist, count, so, do)
    finally:
        bs.free()
        bd.free()


@pytest.mark.gpu
def test_random_multi_cases_against_oracle(dev_ctx):
    """Fuzz of the one-shot multi-operand kernel: random N in {1,2,4,8,16},
    member `self`, dtype/op, count and per-operand element offsets (vector
    path when all agree mod 16 B, scalar path otherwise), against the oracle's
    simulation of the recursive-doubling plan."""
    rng = np.random.default_rng(7)
    pairs = [(dt, op) for dt in O.DTYPES for op in O.OPS if O.is_supported(dt, op)]
    cap = 20_000 * 8 + 256
    bufs = [dev_ctx.alloc(cap) for _ in range(17)]
    try:
        for case in range(120):
            dt, op = pairs[rng.integers(len(pairs))]
            n = int(rng.choice([1, 2, 4, 8, 16]))
            me = int(rng.integers(n))
            count = int(rng.choice([0, 1, 5, 31, 4099, int(rng.integers(1, 20_000))]))
            st = O.storage(dt)
            sz = np.dtype(st).itemsize
            same_off = rng.random() < 0.5
            base_off = int(rng.integers(16)) * sz
            offs = [base_off if same_off else int(rng.integers(16)) * sz for _ in range(n + 1)]
            xs = [O.fill(dt, "special" if rng.random() < 0.3 else "round", 77 * case + r, count)
                  for r in range(n)]
            for r in range(n):
                bufs[r].upload(xs[r], offs[r])
            rc = dev_ctx.reduce_multi(op, dt, bufs[16].ptr + offs[n],
                                      [bufs[r].ptr + offs[r] for r in range(n)], me, count)
            assert rc == 0, _lib.last_error()
            dev_ctx.sync()
            got = bufs[16].download(st, count, offs[n])
            want = O.reduce_multi(op, dt, xs, me) if count else got
            assert (O.bits(got) == O.bits(want)).all(), (case, dt, op, n, me, count, offs)
    finally:
        for b in bufs:
            b.free()


# vector counts (fp32, 64 vectors per tile) that reach every branch of the
# realigning kernels' XCD-aware tile map (dev_kernels.h xcd_tile, chunks of 64
# tiles per XCD): whole chunk rows only, chunk rows plus a remainder row, a
# ragged last round of < 8 tiles, a ragged last tile, fewer than 8 tiles
XCD_NVECS = [3, 7 * 64 + 5, 512 * 64, 1677 * 64 - 34, (8 * 64 * 5 + 8 * 13 + 3) * 64,
             (8 * 64 * 2) * 64 + 1]


# the same branches for the 2-operand combine's 256-tile chunks (dev_launch.h
# kReduceChunkSmall, below 1 GiB per operand)
XCD256_NVECS = [3, 7 * 64 + 5, 2048 * 64, (8 * 256 * 2) * 64, (8 * 256 * 3 + 8 * 13 + 3) * 64,
                (8 * 256 * 2 + 5) * 64 - 17, 1677 * 64 - 34]


@pytest.mark.gpu
def test_reduce_xcd_chunk_map_every_branch(dev_ctx):
    """The in-phase 2-operand combine on 256-tile XCD chunks (round 6): whole
    chunk rows, chunk rows plus a remainder row, a ragged last round and tile,
    fewer tiles than a round - every element bit-exact against the oracle, src
    and dst in phase with a ragged head and tail."""
    dt, st = "float32", np.float32
    cap = max(XCD256_NVECS) * 16 + 256
    src, dst = dev_ctx.alloc(cap), dev_ctx.alloc(cap)
    try:
        for nvec in XCD256_NVECS:
            count = nvec * 4 + 3 + 2          # 8 B into a vector: head 2, tail 3
            xs = O.fill(dt, "round", 500 + nvec % 991, count)
            ys = O.fill(dt, "round", 700 + nvec % 983, count)
            src.upload(xs, 8)
            dst.upload(ys, 8)
            rc = dev_ctx.reduce("sum", dt, dst.ptr + 8, src.ptr + 8, count)
            assert rc == 0, _lib.last_error()
            dev_ctx.sync()
            got = dst.download(st, count, 8)
            bad = np.flatnonzero(O.bits(got) != O.bits(O.reduce("sum", dt, xs, ys)))
            assert bad.size == 0, (nvec, bad[:8])
    finally:
        src.free()
        dst.free()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["reduce", "multi", "tree"])
def test_realigning_kernels_xcd_tile_map(dev_ctx, kernel):
    """The realigning kernels (k_reduce_shift, k_reduce_multi_shift,
    k_reduce_tree_shift) remap workgroups to tiles so that neighbouring tiles
    share an XCD's L2. The map must be a bijection on the tiles for every grid
    size: each count here is checked element for element against the oracle,
    with the first operand 4 B out of dst's phase and a ragged head and tail."""
    dt, st = "float32", np.float32
    n_ops = {"reduce": 2, "multi": 4, "tree": 5}[kernel]
    cap = max(XCD_NVECS) * 16 + 256
    bufs = [dev_ctx.alloc(cap) for _ in range(n_ops + 1)]
    try:
        for nvec in XCD_NVECS:
            count = nvec * 4 + 3 + 2          # dst 8 B into a vector: head 2, tail 3
            xs = [O.fill(dt, "round", 300 + nvec % 997 + r, count) for r in range(n_ops)]
            offs = [12] + [8] * (n_ops - 1)   # dst at 8: operand 0 out of phase
            for r in range(n_ops):
                bufs[r].upload(xs[r], offs[r])
            out = bufs[n_ops]
            if kernel == "reduce":
                # dst is operand 1, in place
                rc = dev_ctx.reduce("sum", dt, bufs[1].ptr + 8, bufs[0].ptr + 12, count)
                want = O.reduce("sum", dt, xs[0], xs[1])
                where = (bufs[1], 8)
            elif kernel == "multi":
                rc = dev_ctx.reduce_multi("sum", dt, out.ptr + 8,
                                          [b.ptr + o for b, o in zip(bufs, offs)], 2, count)
                want = O.reduce_multi("sum", dt, xs, 2)
                where = (out, 8)
            else:
                rc = dev_ctx.reduce_tree("sum", dt, out.ptr + 8,
                                         [b.ptr + o for b, o in zip(bufs, offs)], count)
                want = O.tree_reduce("sum", dt, xs, root=0)
                where = (out, 8)
            assert rc == 0, _lib.last_error()
            dev_ctx.sync()
            got = where[0].download(st, count, where[1])
            bad = np.flatnonzero(O.bits(got) != O.bits(want))
            assert bad.size == 0, (kernel, nvec, bad[:8])
    finally:
        for b in bufs:
            b.free()


@pytest.mark.gpu
def test_random_tree_cases_against_oracle(dev_ctx):
    """Fuzz of the tree fan-in kernel: random n in 1..16, dtype/op, count and
    per-operand element offsets (vector path when all agree mod 16 B, element
    loop otherwise), against the oracle's tree_reduce (root first, children in
    the given order)."""
    rng = np.random.default_rng(8)
    pairs = [(dt, op) for dt in O.DTYPES for op in O.OPS if O.is_supported(dt, op)]
    cap = 20_000 * 8 + 256
    bufs = [dev_ctx.alloc(cap) for _ in range(17)]
    try:
        for case in range(120):
            dt, op = pairs[rng.integers(len(pairs))]
            n = int(rng.integers(1, 17))
            count = int(rng.choice([0, 1, 5, 31, 4099, int(rng.integers(1, 20_000))]))
            st = O.storage(dt)
            sz = np.dtype(st).itemsize
            same_off = rng.random() < 0.5
            base_off = int(rng.integers(16)) * sz
            offs = [base_off if same_off else int(rng.integers(16)) * sz for _ in range(n + 1)]
            xs = [O.fill(dt, "special" if rng.random() < 0.3 else "round", 91 * case + r, count)
                  for r in range(n)]
            for r in range(n):
                bufs[r].upload(xs[r], offs[r])
            rc = dev_ctx.reduce_tree(op, dt, bufs[16].ptr + offs[n],
                                     [bufs[r].ptr + offs[r] for r in range(n)], count)
            assert rc == 0, _lib.last_error()
            dev_ctx.sync()
            got = bufs[16].download(st, count, offs[n])
            want = O.tree_reduce(op, dt, xs, root=0) if count else got
            assert (O.bits(got) == O.bits(want)).all(), (case, dt, op, n, count, offs)
    finally:
        for b in bufs:
            b.free()


@pytest.mark.gpu
def test_multi_and_tree_either_side_of_the_lines_first_threshold(dev_ctx):
    """Round 6: below 256 MiB per operand the every-operand PF forms issue
    their lines first (dev_launch.h kPfoMaxVecs, PFO), from there the earlier
    forms run (fan-ins of 9 operands and more take the lines-first form at
    every size). k_reduce_multi N = 8 and 16 and the tree fan-in at n = 8 (the
    NMAX form), 12 and 6 (the exact-n kernels), fp32 SUM on rounded inputs
    (the association shows), just under and just past 2^24 vectors per
    operand: sampled windows (head, tile and XCD-chunk edges, tail) of every
    result bit-exact against the oracle's plan over the same windows of the
    device-filled operands (ucg_builtin_dev_fill == the oracle's generator)."""
    dt, op, st = "float32", "sum", np.float32
    counts = [(1 << 26) - 12, (1 << 26) + 20]
    cap = (counts[1] + 64) * 4
    bufs = [dev_ctx.alloc(cap) for _ in range(17)]
    try:
        for count in counts:
            for r in range(16):
                dev_ctx.fill(dt, "round", 4000 + r, bufs[r], count)
            dev_ctx.sync()
            w = 4096
            starts = [0, count - w, (1 << 24) * 4 - 2048, 64 * 64 * 4 * 8 - 100,
                      (count // 3) & ~63, (2 * count // 3) | 5]
            wins = [(a, min(count, a + w)) for a in starts]
            xs = {r: [bufs[r].download(st, b - a, a * 4) for a, b in wins] for r in range(16)}
            for kind, n, me in [("multi", 8, 3), ("multi", 16, 5), ("tree", 8, 0),
                                ("tree", 12, 0), ("tree", 6, 0)]:
                srcs = [bufs[r].ptr for r in range(n)]
                if kind == "multi":
                    rc = dev_ctx.reduce_multi(op, dt, bufs[16].ptr, srcs, me, count)
                else:
                    rc = dev_ctx.reduce_tree(op, dt, bufs[16].ptr, srcs, count)
                assert rc == 0, _lib.last_error()
                dev_ctx.sync()
                for k, (a, b) in enumerate(wins):
                    got = bufs[16].download(st, b - a, a * 4)
                    ops_k = [xs[r][k] for r in range(n)]
                    want = (O.reduce_multi(op, dt, ops_k, me) if kind == "multi"
                            else O.tree_reduce(op, dt, ops_k, root=0))
                    bad = np.flatnonzero(O.bits(got) != O.bits(want))
                    assert bad.size == 0, (kind, n, count, a, bad[:8])
    finally:
        for b in bufs:
            b.free()


@pytest.mark.gpu
def test_shift_kernel_every_dtype_and_op(dev_ctx):
    """Every supported (dtype, op) pair through the realigning kernel: src one
    element out of dst's 16-B phase, a ragged count spanning several waves,
    all three distributions, bit-exact against the oracle."""
    n = 64 * 16 * 3 + 5
    bs, bd = dev_ctx.alloc(n * 8 + 64), dev_ctx.alloc(n * 8 + 64)
    try:
        for dt in O.DTYPES:
            st = O.storage(dt)
            sz = np.dtype(st).itemsize
            for op in O.OPS:
                if not O.is_supported(dt, op):
                    continue
                for dist in O.DISTS:
                    src = O.fill(dt, dist, 31, n)
                    dst = O.fill(dt, dist, 32, n)
                    bs.upload(src, sz)
                    bd.upload(dst, 0)
                    dev_ctx.reduce_checked(op, dt, bd.ptr, bs.ptr + sz, n)
                    dev_ctx.sync()
                    got = bd.download(st, n)
                    want = O.reduce(op, dt, src, dst)
                    assert (bits(got) == bits(want)).all(), (dt, op, dist)
    finally:
        bs.free()
        bd.free()


SHIFT_COUNTS = [1, 5, 16, 17, 63 * 4 + 3, 64 * 16, 64 * 16 + 1, 65 * 16 + 7, 128 * 16, 4099,
                64 * 64 * 16 + 9]


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["int8", "float16", "float32", "float64"])
def test_shift_kernel_every_phase(dev_ctx, dt):
    """k_reduce_shift (src and dst disagree mod 16 B): every (src, dst)
    phase pair in whole elements, counts that end a wave on its last lane or
    just past it (vector counts that are multiples of 64 and their
    neighbours), with guard bytes around dst checked untouched, and src
    placed both at the start and flush with the end of its allocation."""
    st = O.storage(dt)
    sz = np.dtype(st).itemsize
    op = "sum"
    granule = 2 << 20
    bs, bd = dev_ctx.alloc(granule), dev_ctx.alloc(granule)
    try:
        for count in SHIFT_COUNTS:
            nb = count * sz
            src = O.fill(dt, "round", 77 + count, count)
            dst = O.fill(dt, "round", 99 + count, count)
            want = O.reduce(op, dt, src, dst)
            for sp in range(0, 16, sz):
                for dp in range(0, 16, sz):
                    if sp == dp and count not in (17, 4099):
                        continue  # the aligned kernel: covered elsewhere
                    for at_end in (False, True):
                        # at_end: the last offset of phase sp that still fits
                        so = ((granule - nb - sp) // 16) * 16 + sp if at_end else sp
                        do = 64 + dp
                        guard = np.full(do + nb + 64, 0xA5, np.uint8)
                        bd.upload(guard)
                        bd.upload(dst, do)
                        bs.upload(src, so)
                        dev_ctx.reduce_checked(op, dt, bd.ptr + do, bs.ptr + so, count)
                        dev_ctx.sync()
                        got = bd.download(st, count, do)
                        assert (O.bits(got) == O.bits(want)).all(), (count, sp, dp, at_end)
                        raw = bd.download(np.uint8, do + nb + 64)
                        assert (raw[:do] == 0xA5).all() and (raw[do + nb:] == 0xA5).all(), \
                            (count, sp, dp, "guard bytes overwritten")
    finally:
        bs.free()
        bd.free()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float32", "float16", "int8", "float64"])
def test_staged_runs_keep_the_accumulator_phase(dt):
    """Staged fragments into a device-resident recv buffer at every 16-B
    phase (the accumulator is the buffer itself): each run is laid out in the
    ring at the accumulator's phase, so the run's launch is an aligned one.
    Fragments of the reference's AM size from two interleaved senders,
    bit-exact against the per-fragment oracle in arrival order, and one
    launch per run (no more launches than with a phase-0 buffer)."""
    st = O.storage(dt)
    sz = np.dtype(st).itemsize
    n = 20_000 + 1
    frag = O.frag_length(256, sz)
    acc = O.fill(dt, "round", 17, n)
    peers = [O.fill(dt, "round", 18 + p, n) for p in range(2)]
    want = acc.copy()
    order = [(p, off) for off in range(0, n * sz, frag) for p in range(2)]
    for p, off in order:
        cnt = min(frag, n * sz - off) // sz
        i0 = off // sz
        want[i0:i0 + cnt] = O.reduce("sum", dt, peers[p][i0:i0 + cnt], want[i0:i0 + cnt])
    launches = {}
    for phase in range(0, 16, sz):
        ctx = xucg_amd.DevContext(device=0, stage_bytes=16 << 10, stage_slots=4)
        try:
            buf = ctx.alloc(n * sz + 64)
            buf.upload(acc, phase)
            assert ctx.stage_begin(buf.ptr + phase, n * sz) == 0, _lib.last_error()
            for p, off in order:
                cnt = min(frag, n * sz - off) // sz
                i0 = off // sz
                piece = np.ascontiguousarray(peers[p][i0:i0 + cnt])
                assert ctx.combine("sum", dt, off, piece, cnt) == 0, _lib.last_error()
            assert ctx.stage_end() == 0, _lib.last_error()
            got = buf.download(st, n, phase)
            assert (bits(got) == bits(want)).all(), (dt, phase)
            launches[phase] = ctx.counters()["launches"]
            buf.free()
        finally:
            ctx.close()
    assert max(launches.values()) <= min(launches.values()) + 2, launches


@pytest.mark.gpu
def test_reduce_tree_vs_oracle(dev_ctx):
    """ucg_builtin_dev_reduce_tree: the tree plan's fan-in association for
    every group size 1..16 (the NMAX 4, 8 and 16 kernels), with every operand
    in dst's phase and with one out of phase (element loop), and with dst
    aliasing the root's operand; bit-exact against the oracle's
    tree_reduce (root 0, children in ascending order)."""
    rng = np.random.default_rng(11)
    pairs = [(dt, op) for dt in O.DTYPES for op in O.OPS if O.is_supported(dt, op)]
    count = 64 * 16 * 2 + 3
    bufs = [dev_ctx.alloc(count * 8 + 64) for _ in range(16)]
    out = dev_ctx.alloc(count * 8 + 64)
    try:
        for n in range(1, 17):
            dt, op = pairs[int(rng.integers(len(pairs)))]
            st = O.storage(dt)
            sz = np.dtype(st).itemsize
            xs = [O.fill(dt, ("round", "special")[m % 2], 500 + 17 * n + m, count)
                  for m in range(n)]
            want = O.tree_reduce(op, dt, xs, root=0)
            for shifted in (False, True):
                offs = [sz if (shifted and m == n // 2) else 0 for m in range(n)]
                for b, x, o in zip(bufs, xs, offs):
                    b.upload(x, o)
                srcs = [b.ptr + o for b, o in zip(bufs, offs)]
                assert dev_ctx.reduce_tree(op, dt, out.ptr, srcs, count) == 0, _lib.last_error()
                dev_ctx.sync()
                got = out.download(st, count)
                assert (bits(got) == bits(want)).all(), (n, dt, op, shifted)
            for b, x in zip(bufs, xs):
                b.upload(x)
            srcs = [b.ptr for b in bufs[:n]]
            assert dev_ctx.reduce_tree(op, dt, bufs[0].ptr, srcs, count) == 0
            dev_ctx.sync()
            assert (bits(bufs[0].download(st, count)) == bits(want)).all(), (n, "aliased")
        assert dev_ctx.reduce_tree("sum", "float32", out.ptr, [b.ptr for b in bufs] * 2, 4) == \
            xucg_amd.UCS_ERR_INVALID_PARAM
    finally:
        for b in bufs + [out]:
            b.free()
