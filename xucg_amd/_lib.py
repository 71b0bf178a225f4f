"""ctypes bindings of the in-tree native libraries.

    xucg_amd/lib/libucg_builtin_dev.so   HIP device shim (include/ucg_builtin_dev.h)
    xucg_amd/lib/libucg_builtin.so       host C builtin-combine layer
                                         (include/ucg_builtin_combine.h)

There is no Python or CPU fallback for the combine: if a library is missing
or fails to load, this module raises and the caller fails loudly.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
DEV_LIB = os.path.join(LIB_DIR, "libucg_builtin_dev.so")
HOST_LIB = os.path.join(LIB_DIR, "libucg_builtin.so")

DTYPES = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "int64",
          "uint64", "float16", "bfloat16", "float32", "float64"]
OPS = ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"]
DISTS = ["exact", "round", "special"]
DTYPE_SIZE = [1, 1, 2, 2, 4, 4, 8, 8, 2, 2, 4, 8]

# ucs_status_t values (UCX ucs/type/status.h)
UCS_OK = 0
UCS_INPROGRESS = 1
UCS_ERR_NO_RESOURCE = -2
UCS_ERR_IO_ERROR = -3
UCS_ERR_NO_MEMORY = -4
UCS_ERR_INVALID_PARAM = -5
UCS_ERR_NOT_IMPLEMENTED = -8
UCS_ERR_NO_DEVICE = -14
UCS_ERR_BUSY = -15
UCS_ERR_CANCELED = -16
UCS_ERR_OUT_OF_RANGE = -19
UCS_ERR_TIMED_OUT = -20
UCS_ERR_EXCEEDS_LIMIT = -21
UCS_ERR_UNSUPPORTED = -22
UCS_ERR_CONNECTION_RESET = -25
IPC_HANDLE_BYTES = 96  # UCG_BUILTIN_DEV_IPC_HANDLE_BYTES

# every exported C-ABI function: name -> (restype, argtypes)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_int = ctypes.c_int
_u = ctypes.c_uint
_u64 = ctypes.c_uint64
_st = ctypes.c_int


class DevCtxParams(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("stream", ctypes.c_void_p),
                ("stage_bytes", ctypes.c_size_t), ("stage_slots", ctypes.c_uint),
                ("zcopy_bytes", ctypes.c_size_t), ("completion", ctypes.c_int)]


ZCOPY_NEVER = (1 << 64) - 1   # UCG_BUILTIN_DEV_ZCOPY_NEVER
NCOUNTERS = 6                 # UCG_BUILTIN_DEV_NCOUNTERS
NMEMSTATS = 11                # UCG_BUILTIN_DEV_NMEMSTATS
MEMSTATS = ["va_retired_bytes", "va_retired_ranges", "va_retired_max",
            "plain_cache_bytes", "shareable_live_bytes", "shareable_import_bytes",
            "parked_bytes",
            "kept_bytes", "keep_max", "plain_cache_exported_bytes", "slack_bytes"]
COMPLETION = {"signal": 1, "sync": 2}   # UCG_BUILTIN_DEV_COMPLETION_*


DEV_API = {
    "ucg_builtin_dev_dtype_size": (_sz, [_int]),
    "ucg_builtin_dev_is_supported": (_int, [_int, _int]),
    "ucg_builtin_dev_version": (ctypes.c_char_p, []),
    "ucg_builtin_dev_last_error": (ctypes.c_char_p, []),
    "ucg_builtin_dev_device_count": (_int, []),
    "ucg_builtin_dev_mem_kind": (_int, [_vp]),
    "ucg_builtin_dev_ctx_create": (_st, [ctypes.POINTER(DevCtxParams),
                                         ctypes.POINTER(_vp)]),
    "ucg_builtin_dev_ctx_destroy": (None, [_vp]),
    "ucg_builtin_dev_ctx_stream": (_vp, [_vp]),
    "ucg_builtin_dev_sync": (_st, [_vp]),
    "ucg_builtin_dev_complete": (_st, [_vp]),
    "ucg_builtin_dev_reduce": (_st, [_vp, _int, _int, _vp, _vp, _sz]),
    "ucg_builtin_dev_reduce_multi": (_st, [_vp, _int, _int, _vp,
                                           ctypes.POINTER(_vp), _u, _u, _sz]),
    "ucg_builtin_dev_reduce_tree": (_st, [_vp, _int, _int, _vp, ctypes.POINTER(_vp), _u,
                                          _sz]),
    "ucg_builtin_dev_gather_multi": (_st, [_vp, _vp, ctypes.POINTER(_vp), _u, _sz]),
    "ucg_builtin_dev_copy_multi": (_st, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _u,
                                         _sz]),
    "ucg_builtin_dev_combine_host": (_st, [_vp, _int, _int, _vp, _vp, _sz]),
    "ucg_builtin_dev_stage_begin": (_st, [_vp, _vp, _sz]),
    "ucg_builtin_dev_combine": (_st, [_vp, _int, _int, _sz, _vp, _sz]),
    "ucg_builtin_dev_stage_end": (_st, [_vp]),
    "ucg_builtin_dev_ipc_export": (_st, [_vp, _vp, _vp]),
    "ucg_builtin_dev_ipc_import": (_st, [_vp, _vp, ctypes.POINTER(_vp)]),
    "ucg_builtin_dev_ipc_release": (_st, [_vp, _vp]),
    "ucg_builtin_dev_malloc": (_vp, [_vp, _sz]),
    "ucg_builtin_dev_malloc_shareable": (_vp, [_vp, _sz]),
    "ucg_builtin_dev_is_shareable": (_int, [_vp]),
    "ucg_builtin_dev_torch_alloc": (_vp, [_sz, _int, _vp]),
    "ucg_builtin_dev_torch_free": (None, [_vp, _sz, _int, _vp]),
    "ucg_builtin_dev_free": (None, [_vp, _vp]),
    "ucg_builtin_dev_park": (None, [_vp, _vp]),
    "ucg_builtin_dev_host_alloc": (_vp, [_sz]),
    "ucg_builtin_dev_host_free": (None, [_vp]),
    "ucg_builtin_dev_host_register": (_int, [_vp, _vp, _sz]),
    "ucg_builtin_dev_host_unregister": (_int, [_vp, _vp]),
    "ucg_builtin_dev_memcpy": (_st, [_vp, _vp, _vp, _sz]),
    "ucg_builtin_dev_debug_ptr": (_sz, [_vp, _vp, ctypes.c_char_p, _sz]),
    "ucg_builtin_dev_set_multi_cap": (None, [_int]),
    "ucg_builtin_dev_fill": (_st, [_vp, _int, _int, _u64, _vp, _sz]),
    "ucg_builtin_dev_profile_reduce": (_st, [_vp, _int, _int, _vp, _vp, _sz, _u,
                                             ctypes.POINTER(ctypes.c_double)]),
    "ucg_builtin_dev_profile_reduce_multi": (_st, [_vp, _int, _int, _vp, ctypes.POINTER(_vp),
                                                   _u, _u, _sz, _u,
                                                   ctypes.POINTER(ctypes.c_double)]),
    "ucg_builtin_dev_profile_stream": (_st, [_vp, _int, _vp, _vp, _sz, _u,
                                             ctypes.POINTER(ctypes.c_double)]),
    "ucg_builtin_dev_counters": (None, [_vp, ctypes.POINTER(_u64)]),
    "ucg_builtin_dev_mem_stats": (None, [ctypes.POINTER(_u64)]),
    "ucg_builtin_dev_set_keep_max": (None, [_u64]),
    "ucg_builtin_dev_set_va_retired_max": (None, [_u64]),
    "ucg_builtin_dev_inject_failure": (_u, [_u]),
}


def code_object_sha16(path=None):
    """First 16 hex digits of the sha256 of the library's device code: its
    .hip_fatbin section (every kernel's gfx950 code object), read from the
    ELF section table. Host-only edits leave it unchanged, so PMC counters of
    a kernel stay attributable to the library that ships.
    None if the file or the section is missing."""
    import hashlib
    import struct
    path = path or DEV_LIB
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    if data[:4] != b"\x7fELF" or data[4] != 2:          # 64-bit ELF only
        return None
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sect(i):
        name, _typ, _flags, _addr, off, size = struct.unpack_from(
            "<IIQQQQ", data, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sect(shstrndx)
    for i in range(shnum):
        name, off, size = sect(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    return None


def mem_stats():
    """The shim's process-wide memory accounting (ucg_builtin_dev_mem_stats):
    retired address ranges and their cap, the reuse cache, live shareable
    allocations and imports, as a dict of MEMSTATS."""
    out = (_u64 * NMEMSTATS)()
    dev().ucg_builtin_dev_mem_stats(out)
    return dict(zip(MEMSTATS, list(out)))

_dev = None
_host = None


class NativeLibraryMissing(ImportError):
    pass


def _bind(lib, api):
    for name, (res, args) in api.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def dev():
    """The HIP device shim; raises NativeLibraryMissing if not built."""
    global _dev
    if _dev is None:
        if not os.path.exists(DEV_LIB):
            raise NativeLibraryMissing(
                f"{DEV_LIB} not built: run `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (hipcc --offload-arch=gfx950)")
        _load_torch_runtime_first()
        _dev = _bind(ctypes.CDLL(DEV_LIB), DEV_API)
    return _dev


def _load_torch_runtime_first():
    """PyTorch-ROCm bundles its own libamdhip64 with the same soname
    (libamdhip64.so.7) as /opt/rocm's. Whichever loads first serves the whole
    process; torch fails to initialise ("No HIP GPUs are available") on the
    /opt/rocm runtime, while this library runs on either. So when torch is
    installed and not yet imported, import it before loading the shim: one
    HIP runtime per process, and torch tensors / streams stay usable here."""
    import importlib.util
    import sys
    if ("torch" in sys.modules or not os.path.exists("/dev/kfd") or
            os.environ.get("XUCG_NO_TORCH_PRELOAD") == "1"):
        return      # already loaded, no GPU driver, or the caller opted out
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def host():
    """The host C builtin-combine layer (include/ucg_builtin_combine.h)."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise NativeLibraryMissing(f"{HOST_LIB} not built")
        from . import host_api
        dev()  # load the dependency first (rpath also resolves it)
        _host = _bind(ctypes.CDLL(HOST_LIB), host_api.HOST_API)
    return _host


def last_error():
    return dev().ucg_builtin_dev_last_error().decode(errors="replace")


class UcsError(RuntimeError):
    def __init__(self, status, what):
        self.status = status
        super().__init__(f"{what} failed with ucs_status_t {status}: {last_error()}")


def check(status, what):
    if status != UCS_OK:
        raise UcsError(status, what)
    return status


def dt_index(dt):
    return DTYPES.index(dt) if isinstance(dt, str) else int(dt)


def op_index(op):
    return OPS.index(op) if isinstance(op, str) else int(op)


def dist_index(d):
    return DISTS.index(d) if isinstance(d, str) else int(d)
