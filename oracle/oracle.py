"""ctypes wrapper around the CPU oracle (oracle/combine_ref.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker or the timed CPU baseline,
never by the product package `xucg_amd`.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UCG_ORACLE_LIB", os.path.join(HERE, "_build", "liboracle.so"))

DTYPES = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "int64",
          "uint64", "float16", "bfloat16", "float32", "float64"]
OPS = ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"]
DISTS = ["exact", "round", "special"]
# numpy storage type per dtype (bf16 is carried as raw uint16 bits)
NP_STORAGE = {"int8": np.int8, "uint8": np.uint8, "int16": np.int16,
              "uint16": np.uint16, "int32": np.int32, "uint32": np.uint32,
              "int64": np.int64, "uint64": np.uint64, "float16": np.float16,
              "bfloat16": np.uint16, "float32": np.float32,
              "float64": np.float64}
# unsigned view used for bit-exact comparison
NP_BITS = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}

_lib = None


def build(force=False):
    """Compile liboracle.so with the committed Makefile."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def build_native():
    """Build oracle/_build/native/liboracle.so with -march=native on THIS host
    (used by bench.py's cpu_baseline on the GPU box)."""
    subprocess.run(["make", "-s", "-C", HERE, "native"], check=True)
    return os.path.join(HERE, "_build", "native", "liboracle.so")


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        L.ucg_oracle_reduce.argtypes = [i, i, vp, vp, sz]
        L.ucg_oracle_reduce.restype = i
        L.ucg_oracle_reduce_fragmented.argtypes = [i, i, vp, vp, sz, sz]
        L.ucg_oracle_reduce_fragmented.restype = i
        L.ucg_oracle_reduce_multi.argtypes = [i, i, vp, ctypes.POINTER(vp),
                                              ctypes.c_uint, ctypes.c_uint, sz]
        L.ucg_oracle_reduce_multi.restype = i
        L.ucg_oracle_tree_reduce.argtypes = [i, i, vp, ctypes.POINTER(vp), ctypes.c_uint,
                                             ctypes.c_uint, ctypes.POINTER(ctypes.c_uint),
                                             sz]
        L.ucg_oracle_tree_reduce.restype = i
        pu = ctypes.POINTER(ctypes.c_uint)
        L.ucg_oracle_tree_intra.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                            pu, pu, pu, pu]
        L.ucg_oracle_tree_intra.restype = i
        L.ucg_oracle_fill.argtypes = [i, i, u64, vp, sz]
        L.ucg_oracle_fill.restype = None
        L.ucg_oracle_fill_range.argtypes = [i, i, u64, sz, vp, sz]
        L.ucg_oracle_fill_range.restype = None
        L.ucg_oracle_is_supported.argtypes = [i, i]
        L.ucg_oracle_is_supported.restype = i
        L.ucg_oracle_dtype_size.argtypes = [i]
        L.ucg_oracle_dtype_size.restype = sz
        L.ucg_oracle_special_table.argtypes = [i, ctypes.POINTER(u64), sz]
        L.ucg_oracle_special_table.restype = sz
        L.ucg_oracle_half_to_float.argtypes = [ctypes.c_uint16]
        L.ucg_oracle_half_to_float.restype = ctypes.c_float
        L.ucg_oracle_float_to_half.argtypes = [ctypes.c_float]
        L.ucg_oracle_float_to_half.restype = ctypes.c_uint16
        L.ucg_oracle_frag_length.argtypes = [sz, sz]
        L.ucg_oracle_frag_length.restype = sz
        L.ucg_oracle_fragments_total.argtypes = [sz, sz, ctypes.c_uint]
        L.ucg_oracle_fragments_total.restype = u64
        L.ucg_oracle_recursive_peer.argtypes = [u64, ctypes.c_uint]
        L.ucg_oracle_recursive_peer.restype = u64
        L.ucg_oracle_splitmix64.argtypes = [u64]
        L.ucg_oracle_splitmix64.restype = u64
        L.ucg_oracle_time_reduce.argtypes = [i, i, vp, vp, sz, sz, i, i,
                                             ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]
        L.ucg_oracle_time_reduce.restype = i
        _lib = L
    return _lib


def dt_index(dt):
    return DTYPES.index(dt) if isinstance(dt, str) else int(dt)


def op_index(op):
    return OPS.index(op) if isinstance(op, str) else int(op)


def storage(dt):
    return NP_STORAGE[DTYPES[dt_index(dt)]]


def is_supported(dt, op):
    return bool(lib().ucg_oracle_is_supported(dt_index(dt), op_index(op)))


def bits(a):
    """Unsigned bit view of an array (for bit-exact comparisons)."""
    a = np.ascontiguousarray(a)
    return a.view(NP_BITS[a.dtype.itemsize])


def fill(dt, dist, seed, count):
    out = np.empty(count, dtype=storage(dt))
    d = DISTS.index(dist) if isinstance(dist, str) else int(dist)
    lib().ucg_oracle_fill(dt_index(dt), d, seed, out.ctypes.data, count)
    return out


def fill_range(dt, dist, seed, start, count):
    """Elements [start, start + count) of fill(dt, dist, seed, ...)."""
    out = np.empty(count, dtype=storage(dt))
    d = DISTS.index(dist) if isinstance(dist, str) else int(dist)
    lib().ucg_oracle_fill_range(dt_index(dt), d, seed, start, out.ctypes.data, count)
    return out


def reduce(op, dt, src, dst, frag_bytes=0):
    """Return a new array = src (op) dst with the reference's semantics."""
    src = np.ascontiguousarray(src, dtype=storage(dt))
    out = np.array(dst, dtype=storage(dt), copy=True)
    assert src.size == out.size
    if frag_bytes:
        rc = lib().ucg_oracle_reduce_fragmented(op_index(op), dt_index(dt),
                                                src.ctypes.data, out.ctypes.data,
                                                out.size, frag_bytes)
    else:
        rc = lib().ucg_oracle_reduce(op_index(op), dt_index(dt),
                                     src.ctypes.data, out.ctypes.data, out.size)
    if rc != 0:
        raise ValueError(f"unsupported combine {op}/{dt}")
    return out


def reduce_multi(op, dt, srcs, self_index):
    srcs = [np.ascontiguousarray(s, dtype=storage(dt)) for s in srcs]
    out = np.empty_like(srcs[0])
    arr = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    rc = lib().ucg_oracle_reduce_multi(op_index(op), dt_index(dt), out.ctypes.data,
                                       arr, len(srcs), self_index, out.size)
    if rc != 0:
        raise ValueError("reduce_multi failed")
    return out


def tree_reduce(op, dt, srcs, root=0, order=None):
    """Tree fan-in result at the root: children reduced in `order`
    (default ascending member index)."""
    srcs = [np.ascontiguousarray(s, dtype=storage(dt)) for s in srcs]
    out = np.empty_like(srcs[0])
    arr = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    ordp = None
    if order is not None:
        ordp = (ctypes.c_uint * len(order))(*order)
    rc = lib().ucg_oracle_tree_reduce(op_index(op), dt_index(dt), out.ctypes.data,
                                      arr, len(srcs), root, ordp, out.size)
    if rc != 0:
        raise ValueError("tree_reduce failed")
    return out


def tree_intra(my, size, root=0):
    up, down = (ctypes.c_uint * 64)(), (ctypes.c_uint * 64)()
    nu, nd = ctypes.c_uint(), ctypes.c_uint()
    lib().ucg_oracle_tree_intra(my, size, root, up, ctypes.byref(nu), down,
                                ctypes.byref(nd))
    return list(up[:nu.value]), list(down[:nd.value])


def special_table(dt):
    buf = (ctypes.c_uint64 * 64)()
    n = lib().ucg_oracle_special_table(dt_index(dt), buf, 64)
    return [buf[i] for i in range(n)]


def frag_length(max_short, dt_len):
    return lib().ucg_oracle_frag_length(max_short, dt_len)


def fragments_total(length, frag_len, ep_cnt):
    return lib().ucg_oracle_fragments_total(length, frag_len, ep_cnt)


def recursive_peer(my, step):
    return lib().ucg_oracle_recursive_peer(my, step)


def time_reduce(op, dt, src, dst, frag_bytes=0, threads=1, reps=5):
    """CPU baseline: (best_s, median_s) for one whole-buffer or fragmented
    combine of src into dst (dst is modified in place)."""
    best, med = ctypes.c_double(), ctypes.c_double()
    rc = lib().ucg_oracle_time_reduce(op_index(op), dt_index(dt), src.ctypes.data,
                                      dst.ctypes.data, dst.size, frag_bytes,
                                      threads, reps, ctypes.byref(best),
                                      ctypes.byref(med))
    if rc != 0:
        raise ValueError("time_reduce failed")
    return best.value, med.value
