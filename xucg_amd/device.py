"""Python handle over the C-ABI device combine (include/ucg_builtin_dev.h).

`DevContext` is the per-group device context of UCG's builtin planner
(`struct ucg_builtin_group_ctx`, reference builtin/builtin.c:66-90). Its
methods map one-to-one onto the C entry points; buffers are passed as raw
device pointers (ints), `DevBuffer` objects, or torch tensors (`data_ptr()`).
Torch is not required by this module.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, dt_index, op_index, dist_index, DTYPE_SIZE

NP_STORAGE = {"int8": np.int8, "uint8": np.uint8, "int16": np.int16,
              "uint16": np.uint16, "int32": np.int32, "uint32": np.uint32,
              "int64": np.int64, "uint64": np.uint64, "float16": np.float16,
              "bfloat16": np.uint16, "float32": np.float32,
              "float64": np.float64}


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, (DevBuffer, HostBuffer)):
        return x.ptr
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take a device pointer of {type(x)}")


def dtype_size(dt):
    return DTYPE_SIZE[dt_index(dt)]


def is_supported(dt, op):
    return bool(_lib.dev().ucg_builtin_dev_is_supported(dt_index(dt), op_index(op)))


def device_count():
    return _lib.dev().ucg_builtin_dev_device_count()


class DevBuffer:
    """A device buffer owned by a DevContext: hipMalloc'ed, or (shareable)
    HIP virtual memory that peers map by its physical allocation."""

    def __init__(self, ctx, nbytes, shareable=False):
        self.ctx = ctx
        self.nbytes = nbytes
        fn = (_lib.dev().ucg_builtin_dev_malloc_shareable if shareable
              else _lib.dev().ucg_builtin_dev_malloc)
        self.ptr = fn(ctx.handle, nbytes)
        if not self.ptr:
            raise MemoryError(f"device allocation of {nbytes} B failed: {_lib.last_error()}")

    def offset(self, nbytes):
        return self.ptr + nbytes

    def upload(self, arr, offset=0):
        arr = np.ascontiguousarray(arr)
        assert offset + arr.nbytes <= self.nbytes
        check(_lib.dev().ucg_builtin_dev_memcpy(self.ctx.handle, self.ptr + offset,
                                                arr.ctypes.data, arr.nbytes), "memcpy H2D")

    def download(self, dtype, count, offset=0):
        out = np.empty(count, dtype=dtype)
        assert offset + out.nbytes <= self.nbytes
        check(_lib.dev().ucg_builtin_dev_memcpy(self.ctx.handle, out.ctypes.data,
                                                self.ptr + offset, out.nbytes), "memcpy D2H")
        return out

    def free(self):
        if self.ptr:
            _lib.dev().ucg_builtin_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostBuffer:
    """Pinned (hipHostMalloc) host memory viewed as a numpy array."""

    def __init__(self, nbytes):
        self.nbytes = nbytes
        self.ptr = _lib.dev().ucg_builtin_dev_host_alloc(nbytes)
        if not self.ptr:
            raise MemoryError(f"hipHostMalloc({nbytes}) failed: {_lib.last_error()}")

    def view(self, dtype, count=None):
        dtype = np.dtype(dtype)
        count = self.nbytes // dtype.itemsize if count is None else count
        buf = (ctypes.c_char * (count * dtype.itemsize)).from_address(self.ptr)
        return np.frombuffer(buf, dtype=dtype, count=count)

    def free(self):
        if self.ptr:
            _lib.dev().ucg_builtin_dev_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DevContext:
    """Per-group device context: one HIP stream, a pinned staging ring and the
    per-step device accumulator."""

    def __init__(self, device=-1, stream=None, stage_bytes=0, stage_slots=0,
                 zcopy_bytes=0, completion="signal"):
        if stream is not None and stream == 0:
            # the C ABI reads NULL as "create a stream": the legacy null stream
            # cannot be shared, and a private non-blocking stream would not be
            # ordered with the caller's work. Share a real stream instead.
            raise ValueError("stream 0 (the null stream) cannot be shared; use "
                             "DevContext.on_torch_stream()")
        L = _lib.dev()
        # zcopy_bytes: 0 = the library default (64 KiB), None = never
        zc = _lib.ZCOPY_NEVER if zcopy_bytes is None else zcopy_bytes
        # completion: how stage_end waits ("signal": pinned completion word,
        # "sync": hipStreamSynchronize)
        p = _lib.DevCtxParams(device, stream, stage_bytes, stage_slots, zc,
                              _lib.COMPLETION[completion])
        h = ctypes.c_void_p()
        check(L.ucg_builtin_dev_ctx_create(ctypes.byref(p), ctypes.byref(h)),
              "ucg_builtin_dev_ctx_create")
        self.handle = h.value

    @classmethod
    def on_torch_stream(cls, device=0, **kw):
        """A context that launches on torch's current stream, made a fresh
        (non-null) stream here: torch ops, RCCL collectives (which order
        themselves against the caller's current stream) and this context's
        combines are then stream-ordered with no host syncs."""
        import torch
        torch.cuda.set_device(device)
        s = torch.cuda.Stream(device=device)
        torch.cuda.set_stream(s)
        ctx = cls(device=device, stream=s.cuda_stream, **kw)
        ctx.torch_stream = s        # keep the stream alive with the context
        return ctx

    # -- lifecycle --------------------------------------------------------
    def close(self):
        if getattr(self, "handle", None):
            _lib.dev().ucg_builtin_dev_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return _lib.dev().ucg_builtin_dev_ctx_stream(self.handle)

    def sync(self):
        check(_lib.dev().ucg_builtin_dev_sync(self.handle), "ucg_builtin_dev_sync")

    # -- memory -----------------------------------------------------------
    def alloc(self, nbytes, shareable=False):
        return DevBuffer(self, nbytes, shareable)

    def debug_ptr(self, ptr):
        """what the runtime and the shim know about a device address, and the
        process's recent memory events near it (diagnostics)"""
        buf = ctypes.create_string_buffer(1 << 16)
        _lib.dev().ucg_builtin_dev_debug_ptr(self.handle, _ptr(ptr), buf, len(buf))
        return buf.value.decode(errors="replace")

    def fill(self, dt, dist, seed, buf, count):
        check(_lib.dev().ucg_builtin_dev_fill(self.handle, dt_index(dt), dist_index(dist),
                                              seed, _ptr(buf), count), "ucg_builtin_dev_fill")

    # -- combine ----------------------------------------------------------
    def reduce(self, op, dt, dst, src, count):
        """dst[i] = src[i] (op) dst[i] on device pointers (async)."""
        return _lib.dev().ucg_builtin_dev_reduce(self.handle, op_index(op), dt_index(dt),
                                                 _ptr(dst), _ptr(src), count)

    def reduce_checked(self, op, dt, dst, src, count):
        check(self.reduce(op, dt, dst, src, count), "ucg_builtin_dev_reduce")

    def reduce_multi(self, op, dt, dst, srcs, self_index, count):
        arr = (ctypes.c_void_p * len(srcs))(*[_ptr(s) for s in srcs])
        return _lib.dev().ucg_builtin_dev_reduce_multi(self.handle, op_index(op),
                                                       dt_index(dt), _ptr(dst), arr,
                                                       len(srcs), self_index, count)

    def reduce_tree(self, op, dt, dst, srcs, count):
        """Tree fan-in: acc = srcs[0]; acc = srcs[m] (op) acc for m = 1.. ."""
        arr = (ctypes.c_void_p * len(srcs))(*[_ptr(s) for s in srcs])
        return _lib.dev().ucg_builtin_dev_reduce_tree(self.handle, op_index(op),
                                                      dt_index(dt), _ptr(dst), arr,
                                                      len(srcs), count)

    def gather_multi(self, dst, srcs, shard_bytes):
        """dst[r * shard_bytes:...] = srcs[r][:shard_bytes] in one launch."""
        arr = (ctypes.c_void_p * len(srcs))(*[_ptr(s) for s in srcs])
        return _lib.dev().ucg_builtin_dev_gather_multi(self.handle, _ptr(dst), arr,
                                                       len(srcs), shard_bytes)

    def copy_multi(self, dsts, srcs, nbytes):
        """dsts[i][:nbytes] = srcs[i][:nbytes] for every pair, one launch."""
        n = len(dsts)
        if len(srcs) != n:
            raise ValueError("copy_multi: as many sources as destinations")
        da = (ctypes.c_void_p * n)(*[_ptr(d) for d in dsts])
        sa = (ctypes.c_void_p * n)(*[_ptr(s) for s in srcs])
        return _lib.dev().ucg_builtin_dev_copy_multi(self.handle, da, sa, n, nbytes)

    def combine_host(self, op, dt, dst_host, src_host, count):
        return _lib.dev().ucg_builtin_dev_combine_host(self.handle, op_index(op),
                                                       dt_index(dt), _ptr(dst_host),
                                                       _ptr(src_host), count)

    def stage_begin(self, host_dst, nbytes):
        return _lib.dev().ucg_builtin_dev_stage_begin(self.handle, _ptr(host_dst), nbytes)

    def combine(self, op, dt, dst_offset, host_src, count):
        return _lib.dev().ucg_builtin_dev_combine(self.handle, op_index(op), dt_index(dt),
                                                  dst_offset, _ptr(host_src), count)

    def stage_end(self):
        return _lib.dev().ucg_builtin_dev_stage_end(self.handle)

    # -- peer mapping -----------------------------------------------------
    def ipc_export(self, buf):
        """Opaque bytes naming `buf` for another process (xGMI peer)."""
        h = (ctypes.c_char * _lib.IPC_HANDLE_BYTES)()
        check(_lib.dev().ucg_builtin_dev_ipc_export(self.handle, _ptr(buf), h),
              "ucg_builtin_dev_ipc_export")
        return bytes(h)

    def ipc_import(self, blob):
        """Map a peer buffer exported by ipc_export(); returns a device pointer."""
        h = (ctypes.c_char * _lib.IPC_HANDLE_BYTES).from_buffer_copy(blob)
        p = ctypes.c_void_p()
        check(_lib.dev().ucg_builtin_dev_ipc_import(self.handle, h, ctypes.byref(p)),
              "ucg_builtin_dev_ipc_import")
        return p.value

    def ipc_release(self, ptr):
        check(_lib.dev().ucg_builtin_dev_ipc_release(self.handle, ptr),
              "ucg_builtin_dev_ipc_release")

    # -- profiling --------------------------------------------------------
    def profile_reduce(self, op, dt, dst, src, count, iters):
        us = ctypes.c_double()
        check(_lib.dev().ucg_builtin_dev_profile_reduce(self.handle, op_index(op),
                                                        dt_index(dt), _ptr(dst), _ptr(src),
                                                        count, iters, ctypes.byref(us)),
              "ucg_builtin_dev_profile_reduce")
        return us.value

    def profile_reduce_multi(self, op, dt, dst, srcs, self_index, count, iters):
        """reduce_multi launched `iters` times back to back between two HIP
        events on the context stream: average us per launch."""
        us = ctypes.c_double()
        arr = (ctypes.c_void_p * len(srcs))(*[_ptr(s) for s in srcs])
        check(_lib.dev().ucg_builtin_dev_profile_reduce_multi(
                  self.handle, op_index(op), dt_index(dt), _ptr(dst), arr, len(srcs),
                  self_index, count, iters, ctypes.byref(us)),
              "ucg_builtin_dev_profile_reduce_multi")
        return us.value

    def profile_stream(self, kind, dst, src, nbytes, iters):
        """Measured ceiling in the combine's geometry: kind 0 reads both
        buffers (no stores), kind 1 copies src -> dst. Average us per launch."""
        us = ctypes.c_double()
        check(_lib.dev().ucg_builtin_dev_profile_stream(self.handle, kind, _ptr(dst), _ptr(src),
                                                        nbytes, iters, ctypes.byref(us)),
              "ucg_builtin_dev_profile_stream")
        return us.value

    def counters(self):
        out = (ctypes.c_uint64 * _lib.NCOUNTERS)()
        _lib.dev().ucg_builtin_dev_counters(self.handle, out)
        c = {"launches": out[0], "combined_bytes": out[1], "h2d_bytes": out[2],
             "d2h_bytes": out[3], "zcopy_bytes": out[4], "signal_waits": out[5]}
        # the process-wide accounting beside the context's own (retired
        # address ranges and their cap: ucg_builtin_dev_mem_stats)
        c.update(_lib.mem_stats())
        return c


def use_shareable_torch_memory():
    """Route torch's device allocations through the shim's shareable
    allocator (torch.cuda.memory.CUDAPluggableAllocator over
    ucg_builtin_dev_torch_alloc / _free), so that every tensor of this process
    can be exported by its physical allocation (ucg_builtin_dev_ipc_export).
    Must run before torch allocates any device memory in the process; it
    replaces torch's caching allocator (every allocation is a VMM mapping of
    whole 2 MiB granules, every free waits for the device)."""
    import torch
    _lib.dev()                       # built, and loaded after torch's HIP runtime
    alloc = torch.cuda.memory.CUDAPluggableAllocator(
        _lib.DEV_LIB, "ucg_builtin_dev_torch_alloc", "ucg_builtin_dev_torch_free")
    torch.cuda.memory.change_current_allocator(alloc)
