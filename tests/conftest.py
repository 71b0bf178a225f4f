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


@pytest.fixture
def in_child(request):
    """For GPU tests that initialise torch's device context: in the pytest
    process, run this test in a child pytest and return True (the caller then
    returns at once); in that child return False (run the body). torch's
    context held by the pytest process for the rest of the session slowed the
    multi-process device tests that follow it (stalls)."""
    import subprocess

    def run():
        if os.environ.get("XUCG_IN_CHILD") == request.node.nodeid:
            return False
        env = dict(os.environ, XUCG_IN_CHILD=request.node.nodeid)
        p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                            "-m", "gpu", request.node.nodeid], cwd=ROOT, env=env,
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0 and " passed" in p.stdout, p.stdout[-3000:] + p.stderr[-2000:]
        return True
    return run
