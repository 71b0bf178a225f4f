"""The plan-component boundary: `ucg_builtin_component`
driven through its vtable as base/ drives it (tests/c/component_test.c).

- over this build's declaration of the API (include/ucg_api_abi.h), linked
  with libucg_builtin.so: allreduce and reduce through query / init / create /
  plan / prepare / trigger / progress / discard / destroy, 1-4 processes;
- over the reference's unchanged api/ucg.h, api/ucg_plan_component.h and
  api/ucg_mpi.h (compat/ for the UCX types, /root/reference present only):
  the component source compiles against the reference's types with every
  vtable signature checked by the compiler, the layout of every type base/
  and the component exchange equals this build's declaration, the reference's
  MPI helpers build the same parameters, and the same collectives run;
- on GPU buffers (-m gpu): the same vtable on device memory, where the
  component's ops run as remote-key steps with the combine kernels.
"""
import os
import shutil
import subprocess

import pytest

from _launch import launch_exe, ROOT

REF_API = "/root/reference/api"
BUILD = os.path.join(ROOT, "tests", "c", "_build")
EXE = os.path.join(BUILD, "component_test")
ENGINE = ["builtin_component.c", "builtin_combine.c", "builtin_shm.c", "builtin_ops.c",
          "builtin_plan.c", "builtin_rma.c"]


@pytest.fixture(scope="module")
def ref_exe(tmp_path_factory):
    """component_test and the component built over the reference's own api/
    headers: the headers stay where they are (symlinked into a temporary
    include tree as <ucg/api/...>); compat/ supplies the UCX types and the
    generated ucg_version.h."""
    if not os.path.isdir(REF_API):
        pytest.skip("the reference tree is not present")
    tmp = tmp_path_factory.mktemp("refapi")
    inc = tmp / "inc" / "ucg" / "api"
    inc.mkdir(parents=True)
    for h in ("ucg.h", "ucg_def.h", "ucg_mpi.h", "ucg_plan_component.h"):
        os.symlink(os.path.join(REF_API, h), inc / h)
    exe = tmp / "component_test_ref"
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-Werror=incompatible-pointer-types",
           "-Werror=int-conversion", "-Werror=implicit-function-declaration",
           "-DXUCG_REFERENCE_API", f"-I{tmp / 'inc'}", f"-I{ROOT}/compat", f"-I{ROOT}/include",
           "-o", str(exe), os.path.join(ROOT, "tests", "c", "component_test.c")]
    cmd += [os.path.join(ROOT, "xucg_amd", "csrc", f) for f in ENGINE]
    cmd += [f"-L{ROOT}/xucg_amd/lib", "-lucg_builtin_dev",
            f"-Wl,-rpath,{ROOT}/xucg_amd/lib", "-lpthread", "-lrt"]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-4000:]
    return str(exe)


def _run(exe, world, mode="host", env=None):
    codes, outs = launch_exe(exe, world, args=(mode,), timeout=120, env_extra=env)
    assert codes == [0] * world, "\n".join(outs)
    assert all(f"rank {r}: ok" in outs[r] for r in range(world)), "\n".join(outs)
    return outs


def test_layout_equals_reference_api(ref_exe):
    """Every offset, size and enum value base/ and the component exchange."""
    ours = subprocess.run([EXE, "layout"], capture_output=True, text=True, check=True).stdout
    ref = subprocess.run([ref_exe, "layout"], capture_output=True, text=True,
                         check=True).stdout
    assert len(ours.splitlines()) > 100
    assert ours == ref


@pytest.mark.parametrize("world", [4, 3, 1])
def test_vtable_host_buffers(world):
    outs = _run(EXE, world)
    if world == 4:
        # component->print: the reference plan for 4 members
        assert "Planner:       builtin" in outs[0]
        assert "recursive doubling" in outs[0]


def test_vtable_group_id_zero():
    """a caller's group id 0 (which base/ accepts) is planned and
    runs; the wire gets a non-zero internal id (builtin_control.c:645 needs
    one) on the group's own transport object."""
    _run(EXE, 2, env={"COMP_GROUP_ID": "0"})


@pytest.mark.parametrize("world", [4, 3])
def test_vtable_over_reference_api(ref_exe, world):
    _run(ref_exe, world)


@pytest.mark.parametrize("world", [4, 3])
def test_vtable_latency_mode_bit_exact(world):
    """BASELINE config 1 through the vtable (bench.py's
    c1_loopback_allreduce_4kib_fp32.component_vtable_max_short_256): a
    persistent fp32 SUM allreduce of 1024 elements started repeatedly,
    bit-exact at the end (exact inputs)."""
    import json
    codes, outs = launch_exe(EXE, world, args=("latency", 300, 1024), timeout=120)
    assert codes == [0] * world, "\n".join(outs)
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["bit_exact"] is True and line["ranks"] == world and line["latency_us"] > 0


def test_component_source_has_no_reference_text():
    """The reference headers are read where they lie, never copied here."""
    for d in ("include", "compat"):
        for root, _, files in os.walk(os.path.join(ROOT, d)):
            for f in files:
                assert f not in ("ucg.h", "ucg_def.h", "ucg_mpi.h", "ucg_plan_component.h"), \
                    os.path.join(root, f)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 3])
def test_vtable_device_buffers(world):
    """Device buffers through the vtable: remote-key steps, combine kernels."""
    _run(EXE, world, "device")
