"""The host C layer (libucg_builtin.so): dispatch, classification, staging
and the control-path rules. CPU tests exercise the reduce_cb_f fallback; GPU
tests (marked) exercise the device path through the same entry points."""
import numpy as np
import pytest

import xucg_amd
from xucg_amd import host
from oracle import oracle as O

from mock_mpi import (MockMPI, OPS, DTYPES, OP_MINLOC, DT_DOUBLE_INT,
                      op_classifier, dt_classifier)


def host_only_combine(mpi, **kw):
    cfg = host.make_config(dev_enable=0)
    return host.BuiltinCombine(mpi.callbacks(), cfg, **kw)


def test_config_from_environment(monkeypatch):
    monkeypatch.setenv("UCX_BUILTIN_DEV_COMBINE", "n")
    monkeypatch.setenv("UCX_BUILTIN_DEV_MIN_BYTES", "64k")
    monkeypatch.setenv("UCX_BUILTIN_DEV_STAGE_BYTES", "2m")
    monkeypatch.setenv("UCX_BUILTIN_DEV_STAGE_SLOTS", "6")
    monkeypatch.setenv("UCX_BUILTIN_DEV_DEVICE", "3")
    c = host.read_config()
    assert (c.dev_enable, c.dev_min_bytes, c.stage_bytes, c.stage_slots, c.device) == \
        (0, 64 << 10, 2 << 20, 6, 3)
    monkeypatch.setenv("UCX_BUILTIN_DEV_COMBINE", "force")
    assert host.read_config().dev_enable == 2
    monkeypatch.delenv("UCX_BUILTIN_DEV_COMBINE")
    monkeypatch.delenv("UCX_BUILTIN_DEV_MIN_BYTES")
    monkeypatch.delenv("UCX_BUILTIN_DEV_STAGE_BYTES")
    c = host.read_config()
    assert c.dev_enable == 1 and c.dev_min_bytes == 1 << 20 and c.stage_bytes == 16 << 20


def test_zcopy_threshold_parsed_as_memory_units(monkeypatch):
    """UCX_BUILTIN_DEV_ZCOPY_BYTES goes through the same unit parser as the
    other size knobs: '64k' is 65536, not 64; '0' and 'never' turn it off;
    unset is the 64 KiB default."""
    from xucg_amd import _lib
    monkeypatch.delenv("UCX_BUILTIN_DEV_ZCOPY_BYTES", raising=False)
    assert host.read_config().zcopy_bytes == 64 << 10
    for text, want in (("64k", 64 << 10), ("1m", 1 << 20), ("4096", 4096),
                       ("010", 10), ("0", _lib.ZCOPY_NEVER),
                       ("never", _lib.ZCOPY_NEVER), ("off", _lib.ZCOPY_NEVER)):
        monkeypatch.setenv("UCX_BUILTIN_DEV_ZCOPY_BYTES", text)
        assert host.read_config().zcopy_bytes == want, text


def test_completion_mode_from_environment(monkeypatch):
    """UCX_BUILTIN_DEV_COMPLETION: 'sync' selects hipStreamSynchronize in
    stage_end; unset (or anything else) the completion word."""
    from xucg_amd import _lib
    monkeypatch.delenv("UCX_BUILTIN_DEV_COMPLETION", raising=False)
    assert host.read_config().completion == _lib.COMPLETION["signal"]
    for text, want in (("sync", "sync"), ("SYNC", "sync"), ("signal", "signal")):
        monkeypatch.setenv("UCX_BUILTIN_DEV_COMPLETION", text)
        assert host.read_config().completion == _lib.COMPLETION[want], text


def test_classification_through_api_callbacks():
    mpi = MockMPI()
    cmb = host_only_combine(mpi)
    dev = {n: i for i, n in enumerate(O.DTYPES)}
    # without the private classifier only SUM is identifiable (is_sum_f)
    assert cmb.classify(OPS["sum"], DTYPES["int32"]) == (0, dev["int32"])
    assert cmb.classify(OPS["sum"], DTYPES["uint64"]) == (0, dev["uint64"])
    assert cmb.classify(OPS["sum"], DTYPES["float64"]) == (0, dev["float64"])
    # api/ cannot tell fp16 from bf16: a 2-byte float is taken as fp16
    assert cmb.classify(OPS["sum"], DTYPES["bfloat16"]) == (0, dev["float16"])
    assert cmb.classify(OPS["max"], DTYPES["int32"]) is None
    assert cmb.classify(OPS["sum"], DT_DOUBLE_INT) is None
    cmb.close()


def test_private_classifier_widens_the_device_set():
    mpi = MockMPI()
    cmb = host_only_combine(mpi, op_classifier=op_classifier, dt_classifier=dt_classifier)
    assert cmb.classify(OPS["max"], DTYPES["int32"]) == (2, 4)
    assert cmb.classify(OPS["bxor"], DTYPES["uint8"]) == (9, 1)
    assert cmb.classify(OPS["sum"], DTYPES["bfloat16"]) == (0, 9)
    assert cmb.classify(OPS["band"], DTYPES["float32"]) is None   # MPI-invalid
    assert cmb.classify(OP_MINLOC, DTYPES["float64"]) is None
    cmb.close()


@pytest.mark.parametrize("dt,op", [("float32", "sum"), ("int64", "prod"),
                                   ("float16", "max"), ("uint8", "bxor")])
def test_host_fallback_is_the_callback(dt, op):
    mpi = MockMPI()
    cmb = host_only_combine(mpi)
    src = O.fill(dt, "round", 1, 1001)
    dst = O.fill(dt, "round", 2, 1001)
    want = O.reduce(op, dt, src, dst)
    assert cmb.reduce(OPS[op], src, dst, 1001, DTYPES[dt]) == 0
    assert (O.bits(dst) == O.bits(want)).all()
    assert mpi.calls == [(OPS[op], 1001, DTYPES[dt])]
    assert cmb.stats()["host_calls"] == 1 and cmb.stats()["dev_calls"] == 0
    assert cmb.reduce(OPS[op], src, dst, 0, DTYPES[dt]) == 0     # no-op
    assert len(mpi.calls) == 1
    cmb.close()


def test_callback_errors_are_propagated():
    mpi = MockMPI()
    cmb = host_only_combine(mpi)
    a = np.zeros(8, np.float32)
    mpi.fail_next = True
    assert cmb.reduce(OPS["sum"], a, a.copy(), 8, DTYPES["float32"]) == xucg_amd._lib.UCS_ERR_IO_ERROR
    assert cmb.stats()["cb_errors"] == 1
    cmb.close()


def test_fragmented_step_on_host_follows_the_fragment_rule():
    """ucg_builtin_mpi_reduce_fragment: count = length / dtype_length for each
    AM-short fragment (builtin_comp_step.inl:112-120)."""
    mpi = MockMPI()
    cmb = host_only_combine(mpi)
    n = 4096 // 8 + 3
    acc = O.fill("float64", "round", 5, n)
    src = O.fill("float64", "round", 6, n)
    want = O.reduce("sum", "float64", src, acc)
    frag = host.fragment_length(256, 8)
    assert frag == 248
    assert cmb.step_begin(OPS["sum"], DTYPES["float64"], acc, acc.nbytes) == 0
    assert cmb.step_begin(OPS["sum"], DTYPES["float64"], acc, acc.nbytes) == -15  # BUSY
    raw = src.view(np.uint8)
    for off in range(0, acc.nbytes, frag):
        ln = min(frag, acc.nbytes - off)
        assert cmb.fragment(off, raw[off:off + ln].copy(), ln) == 0
    assert cmb.fragment(acc.nbytes - 8, raw[:16].copy(), 16) == xucg_amd._lib.UCS_ERR_OUT_OF_RANGE
    assert cmb.step_end() == 0
    assert (O.bits(acc) == O.bits(want)).all()
    counts = [c for _, c, _ in mpi.calls]
    assert counts == [31] * (len(counts) - 1) + [(acc.nbytes % frag) // 8]
    assert len(counts) == host.fragments_total(acc.nbytes, frag, 1)
    cmb.close()


def test_control_rules_match_the_oracle():
    for ms in (64, 256, 2048, 8192, 65536):
        for dl in (1, 2, 4, 8, 12, 16):
            assert host.fragment_length(ms, dl) == O.frag_length(ms, dl)
            for ln in (1, 100, 4096, 1 << 20):
                fl = host.fragment_length(ms, dl)
                assert host.fragments_total(ln, fl, 3) == O.fragments_total(ln, fl, 3)
    assert host.fragment_length(8, 4) == 0
    # chunk sizing: whole fragments per slot, capped by the step
    assert host.dev_chunk_bytes(1 << 30, 248, 8 << 20) == (8 << 20) // 248 * 248
    assert host.dev_chunk_bytes(1000, 248, 8 << 20) == 1000
    # recursive K-ing (builtin_recursive.c:76-88, 158-169)
    assert host.recursive_steps(8, 2) == 3
    assert host.recursive_steps(4, 2) == 2
    assert host.recursive_steps(6, 2) == 0
    assert host.recursive_steps(27, 3) == 3
    assert host.recursive_steps(1, 2) == 0
    for size in (2, 4, 8, 16):
        for my in range(size):
            for step in range(1, host.recursive_steps(size) + 1):
                assert host.recursive_peer(my, step) == O.recursive_peer(my, step)


def test_recursive_factor3_peers_partition_the_group():
    size, factor = 27, 3
    for step in range(1, host.recursive_steps(size, factor) + 1):
        for my in range(size):
            peers = {host.recursive_peer(my, step, factor, k) for k in range(1, factor)}
            group = peers | {my}
            assert len(group) == factor
            # every member of the group computes the same group
            for p in peers:
                assert {host.recursive_peer(p, step, factor, k) for k in range(1, factor)} | {p} == group


# --------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dt,op", [("float32", "sum"), ("float64", "sum"),
                                   ("int32", "max"), ("bfloat16", "prod")])
def test_dispatcher_offloads_large_host_calls_when_forced(dt, op):
    mpi = MockMPI()
    cfg = host.make_config(dev_enable=2, dev_min_bytes=1 << 16, stage_bytes=1 << 20)
    cmb = host.BuiltinCombine(mpi.callbacks(), cfg, op_classifier=op_classifier,
                              dt_classifier=dt_classifier)
    assert cmb.has_device
    n = (1 << 20) + 7
    src = O.fill(dt, "round", 1, n)
    dst = O.fill(dt, "round", 2, n)
    want = O.reduce(op, dt, src, dst)
    assert cmb.reduce(OPS[op], src, dst, n, DTYPES[dt]) == 0, xucg_amd._lib.last_error()
    assert (O.bits(dst) == O.bits(want)).all()
    st = cmb.stats()
    assert st["dev_calls"] == 1 and st["host_calls"] == 0 and not mpi.calls
    # small calls and unclassified ops stay on the host callback
    small_s, small_d = src[:100].copy(), dst[:100].copy()
    w2 = O.reduce(op, dt, small_s, small_d)
    assert cmb.reduce(OPS[op], small_s, small_d, 100, DTYPES[dt]) == 0
    assert (O.bits(small_d) == O.bits(w2)).all()
    assert cmb.stats()["host_calls"] == 1
    cmb.close()


@pytest.mark.gpu
def test_staged_step_on_device_matches_host_fallback():
    n = (1 << 20) + 3
    frag = host.fragment_length(8192, 4)
    src = O.fill("float32", "round", 3, n)
    results = []
    for dev in (2, 0):
        mpi = MockMPI()
        cfg = host.make_config(dev_enable=dev, dev_min_bytes=1 << 16, stage_bytes=1 << 20)
        cmb = host.BuiltinCombine(mpi.callbacks(), cfg)
        acc = O.fill("float32", "round", 4, n)
        assert cmb.step_begin(OPS["sum"], DTYPES["float32"], acc, acc.nbytes) == 0
        raw = src.view(np.uint8)
        for off in range(0, acc.nbytes, frag):
            ln = min(frag, acc.nbytes - off)
            assert cmb.fragment(off, raw[off:off + ln], ln) == 0
        assert cmb.step_end() == 0, xucg_amd._lib.last_error()
        st = cmb.stats()
        if dev:
            assert st["dev_steps"] == 1 and st["host_calls"] == 0
        else:
            assert st["dev_steps"] == 0 and st["host_calls"] > 100
        results.append(acc)
        cmb.close()
    assert (O.bits(results[0]) == O.bits(results[1])).all()


def test_atomic_packer_condition():
    """ucg_builtin_step_select_packers (builtin_control.c:535-575): the atomic
    packers apply to unsigned integer SUM only, element length 1/2/4/8."""
    from xucg_amd import _lib
    from mock_mpi import MockMPI, OPS, DTYPES
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    f = _lib.host().ucg_builtin_combine_atomic_sum_length
    for dt in DTYPES:
        want = O.storage(dt)().itemsize if dt.startswith("uint") else 0
        assert f(cmb.handle, OPS["sum"], DTYPES[dt]) == want, dt
        assert f(cmb.handle, OPS["max"], DTYPES[dt]) == 0, dt
    cmb.close()


@pytest.mark.gpu
def test_stage_bench_c_harness_bit_exact():
    """tests/c/stage_bench.c: a fragmented step staged on the device from C,
    bit-exact against the oracle's per-fragment combine."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "_build", "stage_bench")
    p = subprocess.run([exe, str(3 << 20), "8184", "1"], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["bit_exact"] is True and line["fragments"] == -(-(3 << 20) // 8184)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0x5EEDF022, 0xF022A])
def test_stage_fuzz_c_harness_bit_exact(seed):
    """tests/c/stage_fuzz.c: the fragment aggregator against the oracle over
    random dtype x op, step length, fragment size, 1-4 interleaved senders,
    arrival order, host (any element offset) or device recv buffer and ring
    geometry; every AM payload is poisoned and freed right after its
    combine returns (the borrowed-src contract). A quarter of the cases take
    the whole-buffer form (combine_host) with src and dst each pageable,
    pinned or device memory at any element offset."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "_build", "stage_fuzz")
    p = subprocess.run([exe, "150", hex(seed)], capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["bit_exact"] is True and line["cases"] == 150
    assert line["host_recv"] > 0 and line["device_recv"] > 0 and line["whole_buffer"] > 0


@pytest.mark.gpu
def test_thread_fuzz_c_harness_bit_exact():
    """tests/c/thread_fuzz.c: one combine object (and its device context)
    shared by four host threads, as UCG shares it between the progress
    thread and the async resend thread: staged steps fragment by fragment on
    one, whole-buffer combines on pageable, pinned and device-resident
    buffers on three, every result bit-exact against the oracle."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "_build", "thread_fuzz")
    p = subprocess.run([exe, "40"], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["bit_exact"] is True and line["steps_on_device"] == 40
    assert line["device_calls"] > 240


@pytest.mark.gpu
def test_default_policy_host_buffers_stay_on_host_device_buffers_on_gpu(in_child):
    """UCX_BUILTIN_DEV_COMBINE=y (default): a host recv buffer is combined by
    reduce_cb_f (staging would cross PCIe); a device-resident one
    (GPU-aware MPI) on the GPU in place, whatever its size, with a host or a
    device src; an op the device cannot classify is refused for device
    memory (the host callback cannot dereference it). Torch tensors: runs in
    a child process."""
    if in_child():
        return
    import torch
    from xucg_amd import _lib
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(), op_classifier=op_classifier,
                              dt_classifier=dt_classifier)
    assert cmb.has_device
    n = (1 << 21) + 5
    src = O.fill("float32", "round", 5, n)
    dst = O.fill("float32", "round", 6, n)
    want = O.reduce("sum", "float32", src, dst)
    assert _lib.dev().ucg_builtin_dev_mem_kind(dst.ctypes.data) == 0
    d = dst.copy()
    assert cmb.reduce(OPS["sum"], src, d, n, DTYPES["float32"]) == 0
    assert (O.bits(d) == O.bits(want)).all()
    st = cmb.stats()
    assert st["dev_calls"] == 0 and st["host_calls"] == 1
    for small in (1, 100, n):
        w = O.reduce("max", "float32", src[:small], dst[:small])
        ddev = torch.from_numpy(dst[:small].copy()).cuda()
        assert _lib.dev().ucg_builtin_dev_mem_kind(ddev.data_ptr()) == 2
        for s_on_dev in (False, True):
            dd = ddev.clone()
            s = torch.from_numpy(src[:small].copy()).cuda() if s_on_dev else src[:small].copy()
            torch.cuda.synchronize()
            assert cmb.reduce(OPS["max"], s, dd, small, DTYPES["float32"]) == 0, \
                xucg_amd._lib.last_error()
            assert (O.bits(dd.cpu().numpy()) == O.bits(w)).all(), (small, s_on_dev)
    assert cmb.stats()["host_calls"] == 1
    ddev = torch.zeros(16, device="cuda")
    assert cmb.reduce(OP_MINLOC, src[:16].copy(), ddev, 8, DT_DOUBLE_INT) != 0
    cmb.close()


@pytest.mark.gpu
def test_staged_step_into_device_resident_recv_buffer(in_child):
    """A fragmented step whose recv buffer is device memory accumulates into
    it in place (no mirror copies), bit-exact with the host callback. Torch
    tensors: runs in a child process."""
    if in_child():
        return
    import torch
    n = (1 << 20) + 3
    frag = host.fragment_length(8192, 4)
    src = O.fill("float32", "round", 7, n)
    acc0 = O.fill("float32", "round", 8, n)
    want = O.reduce("sum", "float32", src, acc0, frag_bytes=frag)
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(stage_bytes=1 << 20))
    acc = torch.from_numpy(acc0.copy()).cuda()
    torch.cuda.synchronize()
    assert cmb.step_begin(OPS["sum"], DTYPES["float32"], acc, acc0.nbytes) == 0
    raw = src.view(np.uint8)
    for off in range(0, acc0.nbytes, frag):
        ln = min(frag, acc0.nbytes - off)
        assert cmb.fragment(off, raw[off:off + ln], ln) == 0
    assert cmb.step_end() == 0, xucg_amd._lib.last_error()
    assert cmb.stats()["dev_steps"] == 1 and cmb.stats()["host_calls"] == 0
    assert (O.bits(acc.cpu().numpy()) == O.bits(want)).all()
    cmb.close()
