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
        """every member arrives; UcsError when a member's process is gone
        (UCS_ERR_CONNECTION_RESET) or the wait timed out"""
        _lib.check(_lib.host().ucg_builtin_shm_barrier(self.handle), "ucg_builtin_shm_barrier")

    def close(self):
        """unmaps the object; returns the last barrier's status (non-zero when
        a peer failed - the close still completes)"""
        st = 0
        if getattr(self, "handle", None):
            st = _lib.host().ucg_builtin_shm_iface_close(self.handle)
            self.handle = None
        return st


# enum ucg_group_member_distance (api/ucg.h:253-264)
DISTANCE = {"self": 0, "cache": 1, "socket": 7, "host": 15, "net": 253}


def layout_distances(members, my_index, ppn=None, socket=None):
    """The distance array member `my_index` passes for a "by node" layout:
    hosts of `ppn` consecutive members (default: one host), each split into
    sockets of `socket` consecutive members (default: none)."""
    ppn = ppn or members
    out = []
    for m in range(members):
        if m == my_index:
            out.append(DISTANCE["self"])
        elif m // ppn != my_index // ppn:
            out.append(DISTANCE["net"])
        elif socket and m // socket != my_index // socket:
            out.append(DISTANCE["host"])
        elif socket:
            out.append(DISTANCE["socket"])
        else:
            out.append(DISTANCE["host"])
    return out


class Group:
    """distance: the member's distance array (ucg_group_params_t.distance),
    None = one host; radix / sock_thresh / factor: the planner's
    TREE_RADIX, TREE_SOCKET_LEVEL_PPN_THRESH and RECURSIVE_FACTOR (0 = the
    environment or the default)."""

    def __init__(self, iface, group_id, members, my_index, combine, distance=None,
                 radix=0, sock_thresh=0, factor=0):
        from .host_api import GroupParams
        h = ctypes.c_void_p()
        self._dist = None
        params = None
        if distance is not None or radix or sock_thresh or factor:
            if distance is not None:
                self._dist = (ctypes.c_uint8 * members)(*distance)
            params = GroupParams(self._dist, radix, sock_thresh, factor)
        _lib.check(_lib.host().ucg_builtin_lgroup_create_ex(
            iface.handle, group_id, members, my_index, combine.handle,
            ctypes.byref(params) if params is not None else None, ctypes.byref(h)),
            "ucg_builtin_lgroup_create_ex")
        self.handle = h.value
        self.iface = iface
        self.combine = combine

    def progress(self):
        return _lib.host().ucg_builtin_lgroup_progress(self.handle)

    def stats(self):
        out = (ctypes.c_uint64 * 4)()
        _lib.host().ucg_builtin_lgroup_stats(self.handle, out)
        return {"sent": out[0], "direct": out[1], "stashed": out[2], "resends": out[3]}

    def mem_alloc(self, nbytes, device=True):
        """registered group memory (an address): an op's send buffer taken
        from here is exposed in place by remote-key steps"""
        p = _lib.host().ucg_builtin_lgroup_mem_alloc(self.handle, nbytes, int(device))
        if not p:
            raise MemoryError(f"ucg_builtin_lgroup_mem_alloc({nbytes}, {device}) failed")
        return p

    def mem_free(self, ptr):
        _lib.host().ucg_builtin_lgroup_mem_free(self.handle, ptr)

    def allreduce(self, sbuf, rbuf, count, dtype, op):
        return Allreduce(self, sbuf, rbuf, count, dtype, op)

    def reduce(self, sbuf, rbuf, count, dtype, op, root=0):
        return Reduce(self, sbuf, rbuf, count, dtype, op, root)

    def close(self):
        if getattr(self, "handle", None):
            _lib.host().ucg_builtin_lgroup_destroy(self.handle)
            self.handle = None


def _addr(x):
    """an address, a numpy array, a torch tensor (device buffers run as
    remote-key steps) or a DevBuffer / HostBuffer"""
    if isinstance(x, int):
        return x
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ptr


def _torch_cuda(*bufs):
    return any(getattr(b, "is_cuda", False) for b in bufs)


class _Collective:
    """A persistent collective of the builtin planner (status != 0: the
    create call failed and `handle` is None).

    Torch CUDA tensors as buffers: the engine's device work runs on the
    combine's stream (host.make_config(stream=...)), so work torch queued on
    another stream that produces the send buffer must be complete first:
    start() synchronizes torch's current stream unless it is the combine's."""

    _torch_sync = False
    _stream = None

    def _note_buffers(self, group, *bufs):
        if _torch_cuda(*bufs):
            self._torch_sync = True
            self._stream = getattr(group.combine, "stream", None)

    def start(self):
        if self._torch_sync:
            import torch
            cur = torch.cuda.current_stream()
            if not self._stream or cur.cuda_stream != self._stream:
                cur.synchronize()
        return _lib.host().ucg_builtin_lcoll_start(self.handle)

    def wait(self):
        return _lib.host().ucg_builtin_lcoll_wait(self.handle)

    def run(self):
        st = self.start()
        if st == _lib.UCS_INPROGRESS:
            st = self.wait()
        return st

    def set_completion(self, cb=None, req=None, flag_offset=0, status_offset=0):
        """ucg_params_t.completion: cb(req, status) from the completing call,
        or (cb None) a flag byte and the status written into `req` (an
        address) at the offsets"""
        from .host_api import COMP_CB
        self._comp = COMP_CB(lambda r, st: cb(r, st)) if cb else None
        return _lib.host().ucg_builtin_lcoll_set_completion(
            self.handle, ctypes.cast(self._comp, ctypes.c_void_p) if cb else None,
            req, flag_offset, status_offset)

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
        self._note_buffers(group, sbuf, rbuf)


class Reduce(_Collective):
    """MPI_Reduce: tree fan-in to `root` (rbuf may be None off the root)."""

    def __init__(self, group, sbuf, rbuf, count, dtype, op, root=0):
        self.group = group
        h = ctypes.c_void_p()
        self.status = _lib.host().ucg_builtin_lcoll_reduce(
            group.handle, _addr(sbuf), 0 if rbuf is None else _addr(rbuf), count,
            dtype, op, root, ctypes.byref(h))
        self.handle = h.value if self.status == 0 else None
        self._note_buffers(group, sbuf, rbuf)
