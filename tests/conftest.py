import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# a timed-out engine wait prints the op's state and the stash (builtin_ops.c,
# timeout_dump) into the worker's output, which a failing test shows
os.environ.setdefault("UCX_BUILTIN_TIMEOUT_DUMP", "y")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def dev_ctx():
    """One device context for the whole GPU session (device 0)."""
    import xucg_amd
    ctx = xucg_amd.DevContext(device=0)
    yield ctx
    ctx.close()
