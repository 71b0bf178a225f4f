"""xucg_amd - MI355X-native UCG builtin combine path.

The product is two native libraries behind UCG's builtin plan component:
    xucg_amd/lib/libucg_builtin_dev.so   HIP/gfx950 kernels + C-ABI shim
    xucg_amd/lib/libucg_builtin.so       host C: the ucg_builtin_mpi_reduce
                                         dispatcher, fragment/chunk sizing,
                                         recursive-doubling plan, loopback
                                         transport
This package holds the ctypes view of both (used by tests and bench.py).
"""
from ._lib import (DTYPES, OPS, DISTS, UcsError, NativeLibraryMissing,  # noqa: F401
                   UCS_OK, UCS_ERR_UNSUPPORTED, UCS_ERR_INVALID_PARAM,
                   UCS_ERR_NO_DEVICE, UCS_ERR_OUT_OF_RANGE)
from .device import (DevContext, DevBuffer, HostBuffer, dtype_size,  # noqa: F401
                     is_supported, device_count, NP_STORAGE,
                     use_shareable_torch_memory)

__version__ = "0.1.0"
