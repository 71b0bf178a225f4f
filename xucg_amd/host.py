"""Python handle over the host C layer (include/ucg_builtin_combine.h).

`BuiltinCombine` is the per-group combine state of UCG's builtin planner: it
owns the user's reduce/datatype callbacks (the ucg_params_t.reduce_op and
.datatype blocks of api/ucg.h:129-160) and, when a GPU is present, a device
context. Its `reduce` is the replacement of ucg_builtin_mpi_reduce
(builtin/ops/builtin_comp_step.inl:96-102); `step_begin/fragment/step_end`
bracket one REDUCE step of a plan.
"""
import ctypes

from . import _lib
from .host_api import (REDUCE_CB, OP_FN, CONVERT_FN, IS_INT_FN, DT_FN,
                       ReduceParams, CombineConfig)

STAT_NAMES = ["host_calls", "host_bytes", "dev_calls", "dev_bytes",
              "dev_steps", "cb_errors"]


def _vp(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    if hasattr(x, "ptr"):
        return x.ptr
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x


def read_config():
    cfg = CombineConfig()
    _lib.host().ucg_builtin_combine_config_read(ctypes.byref(cfg))
    return cfg


def make_config(dev_enable=1, dev_min_bytes=1 << 20, stage_bytes=8 << 20,
                stage_slots=4, device=-1, zcopy_bytes=0, completion="signal",
                stream=None):
    """zcopy_bytes: 0 = the device library's default (64 KiB), None = never;
    completion: "signal" (pinned completion word) or "sync" (stage_end);
    stream: the caller's HIP stream (an int, e.g. torch's
    current_stream().cuda_stream) the device work is queued on, None = a
    private one"""
    zc = _lib.ZCOPY_NEVER if zcopy_bytes is None else zcopy_bytes
    return CombineConfig(dev_enable, dev_min_bytes, stage_bytes, stage_slots, device, zc,
                         _lib.COMPLETION[completion], stream)


class BuiltinCombine:
    """callbacks: dict with reduce_cb_f(op, src, dst, count, dtype) -> int and
    optionally is_sum_f(op), is_loc_expected_f(op), is_commutative_f(op),
    convert(dtype) -> ucp_datatype or None, is_integer_f(dtype) ->
    (bool, is_signed), is_floating_point_f(dtype) -> bool. Handles are ints."""

    def __init__(self, callbacks, config=None, op_classifier=None,
                 dt_classifier=None):
        self.stream = getattr(config, "stream", None) if config is not None else None
        cb = callbacks
        # keep every ctypes thunk alive for the lifetime of the object
        self._thunks = []

        def keep(f):
            self._thunks.append(f)
            return f

        def reduce_cb(op, src, dst, count, dtype):
            return int(cb["reduce_cb_f"](op or 0, src or 0, dst or 0, count, dtype or 0))

        def op_pred(name):
            fn = cb.get(name)
            return keep(OP_FN(lambda op: int(bool(fn(op or 0))))) if fn else OP_FN()

        def convert(dtype, out):
            v = cb["convert"](dtype or 0)
            if v is None:
                return -1
            out[0] = v
            return 0

        def is_int(dtype, signed):
            ok, sgn = cb["is_integer_f"](dtype or 0)
            signed[0] = int(bool(sgn))
            return int(bool(ok))

        p = ReduceParams()
        p.reduce_cb_f = keep(REDUCE_CB(reduce_cb))
        p.is_sum_f = op_pred("is_sum_f")
        p.is_loc_expected_f = op_pred("is_loc_expected_f")
        p.is_commutative_f = op_pred("is_commutative_f")
        p.convert = keep(CONVERT_FN(convert)) if "convert" in cb else CONVERT_FN()
        p.is_integer_f = keep(IS_INT_FN(is_int)) if "is_integer_f" in cb else IS_INT_FN()
        p.is_floating_point_f = (keep(DT_FN(lambda d: int(bool(cb["is_floating_point_f"](d or 0)))))
                                 if "is_floating_point_f" in cb else DT_FN())
        self._params = p
        h = ctypes.c_void_p()
        cfg = ctypes.byref(config) if config is not None else None
        _lib.check(_lib.host().ucg_builtin_combine_create(ctypes.byref(p), cfg,
                                                          ctypes.byref(h)),
                   "ucg_builtin_combine_create")
        self.handle = h.value
        if op_classifier or dt_classifier:
            ocf = keep(OP_FN(lambda op: int(op_classifier(op or 0)))) if op_classifier else OP_FN()
            dcf = keep(DT_FN(lambda d: int(dt_classifier(d or 0)))) if dt_classifier else DT_FN()
            _lib.host().ucg_builtin_combine_set_classifier(self.handle, ocf, dcf)

    def close(self):
        if getattr(self, "handle", None):
            _lib.host().ucg_builtin_combine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def has_device(self):
        return bool(_lib.host().ucg_builtin_combine_has_device(self.handle))

    def classify(self, op, dtype):
        o, d = ctypes.c_int(-1), ctypes.c_int(-1)
        ok = _lib.host().ucg_builtin_combine_classify(self.handle, op, dtype,
                                                      ctypes.byref(o), ctypes.byref(d))
        return (o.value, d.value) if ok else None

    def check_reduction(self, op):
        """0, or UCS_ERR_UNSUPPORTED for MINLOC/MAXLOC and non-commutative
        ops (builtin_control.c:872-888)."""
        return _lib.host().ucg_builtin_combine_check_reduction(self.handle, op)

    def reduce(self, op, src, dst, count, dtype):
        return _lib.host().ucg_builtin_combine_reduce(self.handle, op, _vp(src),
                                                      _vp(dst), count, dtype)

    def step_begin(self, op, dtype, recv_buffer, length):
        return _lib.host().ucg_builtin_combine_step_begin(self.handle, op, dtype,
                                                          _vp(recv_buffer), length)

    def fragment(self, offset, src, length):
        return _lib.host().ucg_builtin_combine_fragment(self.handle, offset, _vp(src),
                                                        length)

    def step_end(self):
        return _lib.host().ucg_builtin_combine_step_end(self.handle)

    def stats(self):
        out = (ctypes.c_uint64 * 6)()
        _lib.host().ucg_builtin_combine_stats(self.handle, out)
        return dict(zip(STAT_NAMES, list(out)))


def fragment_length(max_short, dt_len):
    return _lib.host().ucg_builtin_step_fragment_length(max_short, dt_len)


def fragments_total(length, frag_len, ep_cnt):
    return _lib.host().ucg_builtin_step_fragments_total(length, frag_len, ep_cnt)


def dev_chunk_bytes(length, frag_len, slot_bytes):
    return _lib.host().ucg_builtin_dev_chunk_bytes(length, frag_len, slot_bytes)


def recursive_steps(count, factor=2):
    return _lib.host().ucg_builtin_recursive_steps(count, factor)


def recursive_peer(my, step, factor=2, peer_idx=1):
    return _lib.host().ucg_builtin_recursive_peer(my, step, factor, peer_idx)
