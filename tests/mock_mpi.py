"""A stand-in for the MPI library on the other side of UCG's callbacks.

Ops and datatypes are opaque integer handles, as MPI_Op/MPI_Datatype are in
an MPICH-style integration. reduce_cb_f performs MPI_Reduce_local semantics
through the CPU oracle (itself pinned against MPICH 3.3.2), so a combine that
falls back to the host computes exactly what the reference would.
"""
import ctypes

import numpy as np

from oracle import oracle as O

OP_BASE = 0x4000
DT_BASE = 0x8000
OPS = {name: OP_BASE + i for i, name in enumerate(O.OPS)}
DTYPES = {name: DT_BASE + i for i, name in enumerate(O.DTYPES)}
OP_MINLOC = OP_BASE + 0x100      # an op the device path cannot classify
DT_DOUBLE_INT = DT_BASE + 0x100  # a contiguous 12-byte struct type


def op_name(h):
    return O.OPS[h - OP_BASE]


def dt_name(h):
    return O.DTYPES[h - DT_BASE]


class MockMPI:
    def __init__(self):
        self.calls = []       # (op, count, dtype) per reduce_cb_f call
        self.fail_next = False

    def reduce_cb_f(self, op, src, dst, count, dtype):
        self.calls.append((op, count, dtype))
        if self.fail_next:
            self.fail_next = False
            return 1
        if op == OP_MINLOC or dtype == DT_DOUBLE_INT:
            return 1
        dt = dt_name(dtype)
        st = O.storage(dt)
        sz = np.dtype(st).itemsize
        s = np.ctypeslib.as_array((ctypes.c_uint8 * (count * sz)).from_address(src)).view(st)
        d = np.ctypeslib.as_array((ctypes.c_uint8 * (count * sz)).from_address(dst)).view(st)
        d[:] = O.reduce(op_name(op), dt, s.copy(), d)
        return 0

    @staticmethod
    def is_sum_f(op):
        return op == OPS["sum"]

    @staticmethod
    def is_loc_expected_f(op):
        return op == OP_MINLOC

    @staticmethod
    def is_commutative_f(op):
        return True

    @staticmethod
    def convert(dtype):
        if dtype == DT_DOUBLE_INT:
            return 12 << 3
        return O.lib().ucg_oracle_dtype_size(dtype - DT_BASE) << 3  # contig

    @staticmethod
    def is_integer_f(dtype):
        if dtype == DT_DOUBLE_INT:
            return False, False
        name = dt_name(dtype)
        return name.startswith(("int", "uint")), name.startswith("int")

    @staticmethod
    def is_floating_point_f(dtype):
        return dtype != DT_DOUBLE_INT and "float" in dt_name(dtype)

    def callbacks(self):
        return {"reduce_cb_f": self.reduce_cb_f, "is_sum_f": self.is_sum_f,
                "is_loc_expected_f": self.is_loc_expected_f,
                "is_commutative_f": self.is_commutative_f, "convert": self.convert,
                "is_integer_f": self.is_integer_f,
                "is_floating_point_f": self.is_floating_point_f}


def op_classifier(op):
    """builtin-private classifier: MPI op handle -> ucg_dev_op_t or -1."""
    return op - OP_BASE if OP_BASE <= op < OP_BASE + len(O.OPS) else -1


def dt_classifier(dtype):
    return dtype - DT_BASE if DT_BASE <= dtype < DT_BASE + len(O.DTYPES) else -1
