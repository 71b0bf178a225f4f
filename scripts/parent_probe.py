"""Do the 5-member device-buffer workers stall because their parent process
holds an initialised GPU context? Times the same worker group launched from
this process (1) before it touches the GPU, (2) after a device context was
created and closed, (3) with a device context open, (4) after 2 more
groups. A group that needs more than its deadline is reported as such."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _launch import launch  # noqa: E402

os.environ.setdefault("UCX_BUILTIN_WAIT_TIMEOUT", "90")
spec = sys.argv[1] if len(sys.argv) > 1 else "5:1:0:2:2:16"
n = int(spec.split(":")[0])


def group(tag):
    t0 = time.time()
    codes, outs = launch("_worker_topo.py", n, args=(f"probe_{os.getpid()}_{tag}", "rma", 256,
                                                     spec), timeout=60)
    slow = [l for o in outs for l in o.splitlines() if "ucg slow" in l]
    print(f"{tag}: {time.time() - t0:.1f} s codes {codes} slow notes {len(slow)}", flush=True)
    for l in slow[:6]:
        print("   ", l, flush=True)


group("fresh-parent")
if len(sys.argv) > 2 and sys.argv[2] == "torch":
    # only torch's device context in the parent (test_host_combine.py's t2 / t3
    # use torch tensors; r02s14)
    import torch
    x = torch.zeros(1 << 20, device="cuda")
    torch.cuda.synchronize()
    group("torch-tensor-alive")
    del x
    torch.cuda.empty_cache()
    group("torch-tensor-freed")
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] == "torchinit-ctx-nolaunch":
    # torch's device context, then this build's library loaded and a device
    # context created (streams, pinned words) with no kernel launched
    import torch
    import xucg_amd
    x = torch.ones(16, device="cuda")
    torch.cuda.synchronize()
    ctx = xucg_amd.DevContext(device=0)
    group(sys.argv[2])
    ctx.close()
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] in ("torchinit-tiny", "torchinit-tiny-nt"):
    # torch's device context initialised, then one kernel of a separate
    # one-kernel code object (scripts/tiny_kernel.hip -> tools/libtiny_kernel.so),
    # none of this build's: is it any foreign code object, or this build's?
    import ctypes
    import torch
    x = torch.ones(1 << 20, device="cuda")
    y = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libtiny_kernel.so"))
    fn = lib.tiny_add_nt if sys.argv[2].endswith("-nt") else lib.tiny_add
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong]
    assert fn(x.data_ptr(), y.data_ptr(), 1 << 20) == 0
    assert float(x[0]) == 2.0
    group(sys.argv[2])
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] == "rocm-first-torchinit-own":
    # torchinit-own with this build's library (and /opt/rocm's HIP runtime)
    # loaded before torch, so one runtime, /opt/rocm's, serves both
    from xucg_amd import _lib
    _lib.dev()
    sys.argv[2] = "torchinit-own"
    import torch
    with open("/proc/self/maps") as f:
        print(sorted({l.split()[-1] for l in f if "amdhip64" in l}), flush=True)
if len(sys.argv) > 2 and sys.argv[2] == "torchinit-own":
    # torch's device context initialised, the combine on the shim's own buffers
    import torch
    import xucg_amd
    x = torch.zeros(16, device="cuda")
    torch.cuda.synchronize()
    ctx = xucg_amd.DevContext(device=0)
    a, b = ctx.alloc(4 << 20), ctx.alloc(4 << 20)
    ctx.reduce_checked("sum", "float32", b, a, 1 << 20)
    ctx.sync()
    group(sys.argv[2])
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] in ("devctx-on-torch-keep", "torchstream-on-torch"):
    # devctx-on-torch with the context left open, or with the context on
    # torch's current stream (DevContext.on_torch_stream) instead of its own
    import torch
    import xucg_amd
    a = torch.ones(1 << 20, device="cuda")
    b = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    ctx = (xucg_amd.DevContext(device=0) if sys.argv[2] == "devctx-on-torch-keep"
           else xucg_amd.DevContext.on_torch_stream(0))
    ctx.reduce_checked("sum", "float32", b, a, 1 << 20)
    ctx.sync()
    torch.cuda.synchronize()
    group(sys.argv[2])
    ctx.close()
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] in ("devctx-on-torch", "combine-on-own"):
    # which half of torch-xucg sets it off: (devctx-on-torch) the device
    # shim's own context combining two torch tensors, or (combine-on-own)
    # BuiltinCombine.reduce on two buffers of the shim's allocator
    import torch
    import xucg_amd
    if sys.argv[2] == "devctx-on-torch":
        a = torch.ones(1 << 20, device="cuda")
        b = torch.ones(1 << 20, device="cuda")
        torch.cuda.synchronize()
        ctx = xucg_amd.DevContext(device=0)
        ctx.reduce_checked("sum", "float32", b, a, 1 << 20)
        ctx.sync()
        ctx.close()
    else:
        from mock_mpi import MockMPI, OPS, DTYPES
        from xucg_amd import host
        ctx = xucg_amd.DevContext(device=0)
        a, b = ctx.alloc(4 << 20), ctx.alloc(4 << 20)
        cmb = host.BuiltinCombine(MockMPI().callbacks(), host.make_config())
        assert cmb.reduce(OPS["sum"], a.ptr, b.ptr, 1 << 20, DTYPES["float32"]) == 0
        cmb.close()
    group(sys.argv[2])
    sys.exit(0)
if len(sys.argv) > 2 and sys.argv[2] == "torch-xucg":
    # bench.py's parent: torch imported first (its bundled runtime serves
    # both), a device context running the combine on its own buffers, and a
    # combine on torch tensors as test_host_combine.py's t2 does
    import torch
    import xucg_amd
    ctx = xucg_amd.DevContext(device=0)
    nn = 1 << 22
    s_, d_ = ctx.alloc(nn * 4), ctx.alloc(nn * 4)
    ctx.profile_reduce("sum", "float32", d_.ptr, s_.ptr, nn, 20)
    s_.free()
    d_.free()
    ctx.close()
    group("torch-then-xucg-buffers")
    from mock_mpi import MockMPI, OPS, DTYPES
    from xucg_amd import host
    cmb = host.BuiltinCombine(MockMPI().callbacks(), host.make_config())
    a = torch.ones(1 << 20, device="cuda")
    b = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    assert cmb.reduce(OPS["sum"], a, b, 1 << 20, DTYPES["float32"]) == 0
    cmb.close()
    group("combine-on-torch-tensors")
    sys.exit(0)
import xucg_amd  # noqa: E402
ctx = xucg_amd.DevContext(device=0)
ctx.close()
group("after-closed-context")
ctx = xucg_amd.DevContext(device=0)
group("open-context")
ctx.close()
group("again")
