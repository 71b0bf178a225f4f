"""Python handle over the builtin operation engine and its shared-memory
transport (include/ucg_builtin_ops.h): one process per group member."""
import ctypes

from . import _lib


class ShmIface:
    """Shared-memory active-message transport among the members of one host
    (the UCT iface of the reference's builtin planner)."""

    def __init__(self, name, members, my_index, max_short=256, ring_cells=64):
        h = ctypes.c_void_p()
        _lib.check(_lib.host().ucg_builtin_shm_iface_open(name.encode(), members,
                                                          my_index, max_short,
                                                          ring_cells, ctypes.byref(h)),
                   "ucg_builtin_shm_iface_open")
        self.handle = h.value

    def barrier(self):
        _lib.host().ucg_builtin_shm_barrier(self.handle)

    def close(self):
        if getattr(self, "handle", None):
            _lib.host().ucg_builtin_shm_iface_close(self.handle)
            self.handle = None


class Group:
    def __init__(self, iface, group_id, members, my_index, combine):
        h = ctypes.c_void_p()
        _lib.check(_lib.host().ucg_builtin_lgroup_create(iface.handle, group_id, members,
                                                         my_index, combine.handle,
                                                         ctypes.byref(h)),
                   "ucg_builtin_lgroup_create")
        self.handle = h.value
        self.iface = iface
        self.combine = combine

    def progress(self):
        return _lib.host().ucg_builtin_lgroup_progress(self.handle)

    def stats(self):
        out = (ctypes.c_uint64 * 4)()
        _lib.host().ucg_builtin_lgroup_stats(self.handle, out)
        return {"sent": out[0], "direct": out[1], "stashed": out[2], "resends": out[3]}

    def allreduce(self, sbuf, rbuf, count, dtype, op):
        return Allreduce(self, sbuf, rbuf, count, dtype, op)

    def reduce(self, sbuf, rbuf, count, dtype, op, root=0):
        return Reduce(self, sbuf, rbuf, count, dtype, op, root)

    def close(self):
        if getattr(self, "handle", None):
            _lib.host().ucg_builtin_lgroup_destroy(self.handle)
            self.handle = None


def _addr(x):
    if isinstance(x, int):
        return x
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return x.ptr


class _Collective:
    """A persistent collective of the builtin planner (status != 0: the
    create call failed and `handle` is None)."""

    def start(self):
        return _lib.host().ucg_builtin_lcoll_start(self.handle)

    def wait(self):
        return _lib.host().ucg_builtin_lcoll_wait(self.handle)

    def run(self):
        st = self.start()
        if st == _lib.UCS_INPROGRESS:
            st = self.wait()
        return st

    def describe(self):
        buf = ctypes.create_string_buffer(4096)
        n = _lib.host().ucg_builtin_lcoll_describe(self.handle, buf, len(buf))
        return buf.raw[:n].decode()

    def close(self):
        if self.handle:
            _lib.host().ucg_builtin_lcoll_destroy(self.handle)
            self.handle = None


class Allreduce(_Collective):
    """MPI_Allreduce: recursive doubling (power-of-two groups) or tree."""

    def __init__(self, group, sbuf, rbuf, count, dtype, op):
        self.group = group
        h = ctypes.c_void_p()
        self.status = _lib.host().ucg_builtin_lcoll_allreduce(
            group.handle, _addr(sbuf), _addr(rbuf), count, dtype, op, ctypes.byref(h))
        self.handle = h.value if self.status == 0 else None


class Reduce(_Collective):
    """MPI_Reduce: tree fan-in to `root` (rbuf may be None off the root)."""

    def __init__(self, group, sbuf, rbuf, count, dtype, op, root=0):
        self.group = group
        h = ctypes.c_void_p()
        self.status = _lib.host().ucg_builtin_lcoll_reduce(
            group.handle, _addr(sbuf), 0 if rbuf is None else _addr(rbuf), count,
            dtype, op, root, ctypes.byref(h))
        self.handle = h.value if self.status == 0 else None
