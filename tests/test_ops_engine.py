"""The builtin operation engine end to end:
multi-process allreduce over the shared-memory transport, every combine
through the dispatcher. BASELINE config 1 is the 4-rank 4 KiB fp32 case."""
import os
import uuid

import numpy as np
import pytest

from xucg_amd import host, ops
from oracle import oracle as O
from _launch import launch, launch_exe
from mock_mpi import MockMPI, OPS, DTYPES


def shm_name():
    return f"ucg_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"


@pytest.mark.parametrize("world,max_short,cells", [(4, 256, 64), (2, 64, 64), (8, 256, 64),
                                                 (4, 8192, 64), (4, 64, 2)])
def test_allreduce_multiprocess_host(world, max_short, cells):
    """cells = 2 forces UCS_ERR_NO_RESOURCE and the resend path
    (builtin_data.c:650-663, builtin.c:329-337)."""
    codes, outs = launch("_worker_ops.py", world,
                         args=(shm_name(), "host", max_short, 200, cells), timeout=240)
    assert codes == [0] * world, "\n".join(outs)
    if world == 4 and max_short == 256 and cells == 64:
        print(outs[0])


@pytest.mark.parametrize("max_short", [256, 8192])
def test_c1_harness_bit_exact(max_short):
    """BASELINE config 1 from plain C: 4 processes, 4 KiB fp32 SUM."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "_build", "c1_allreduce")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe) + "/.."], check=True)
    codes, outs = launch_exe(exe, 4, (shm_name(), 2000, max_short))
    assert codes == [0] * 4, "\n".join(outs)
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["bit_exact"] and line["ranks"] == 4 and line["bytes"] == 4096


def test_plan_description_and_unsupported_sizes():
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    # a 1-member "group": no peers, so the transport is never used
    iface = ops.ShmIface(shm_name(), 1, 0, max_short=256)
    g = ops.Group(iface, 3, 1, 0, cmb)
    x = np.arange(16, dtype=np.float32)
    y = np.zeros_like(x)
    c = g.allreduce(x, y, 16, DTYPES["float32"], OPS["sum"])
    assert c.run() == 0 and (y == x).all()    # init_reduce only
    c.close()
    g.close()
    iface.close()
    cmb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_allreduce_multiprocess_device_staging(world):
    """Same engine, every step staged on the GPU (dev_min_bytes = 0)."""
    codes, outs = launch("_worker_ops.py", world, args=(shm_name(), "dev", 256, 20),
                         timeout=300)
    assert codes == [0] * world, "\n".join(outs)
