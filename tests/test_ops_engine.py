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


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


@pytest.mark.parametrize("world,cells", [(4, 64), (8, 64), (2, 64), (4, 3)])
def test_allreduce_multiprocess_shm_zcopy(world, cells, monkeypatch):
    """The same worker with every message on the shared-memory remote-key
    steps (UCX_BUILTIN_SHM_ZCOPY_THRESH=1): every dtype/op case, a persistent
    op restarted, the empty op, two ops in flight at once on one group (each
    with its own registered buffers, messages told apart by coll_id), and a
    3-cell ring for the control messages (whether they meet
    UCS_ERR_NO_RESOURCE depends on the peers' timing, so resends are not
    required here; the data-carrying ring of the test above requires them)."""
    monkeypatch.setenv("UCX_BUILTIN_SHM_ZCOPY_THRESH", "1")
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "60")
    # every member's own bits on the special values (NaN payloads): no float
    # op takes the two-phase one-shot (builtin_rma.c, oneshot_split_allowed)
    monkeypatch.setenv("UCX_BUILTIN_ONESHOT_FLOAT_SPLIT", "n")
    codes, outs = launch("_worker_ops.py", world,
                         args=(shm_name(), "host", 256, 100, cells), timeout=240)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.parametrize("max_short,world", [(256, 4), (8192, 4), (256, 3)])
def test_c1_harness_bit_exact(max_short, world):
    """BASELINE config 1 from plain C: 4 processes, 4 KiB fp32 SUM (and the
    tree plan at 3 processes)."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "_build", "c1_allreduce")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe) + "/.."], check=True)
    codes, outs = launch_exe(exe, world, (shm_name(), 2000, max_short))
    assert codes == [0] * world, "\n".join(outs)
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["bit_exact"] and line["ranks"] == world and line["bytes"] == 4096


@pytest.mark.parametrize("world,max_short,plan,incast,place,pipe", [
    (4, 256, "", "", "", ""), (3, 256, "", "", "", ""), (8, 100, "", "", "", ""),
    (4, 256, "tree", "1", "", ""), (5, 64, "tree", "", "", ""),
    (8, 256, "", "", "4", ""), (12, 100, "", "", "3", ""), (8, 256, "tree", "1", "8:4", ""),
    (12, 100, "", "", "3", "y"), (8, 256, "", "", "", "zcopy"),
    (12, 256, "", "", "3", "zcopy"), (6, 256, "tree", "", "", "zcopy"),
    (8, 256, "", "", "", "zcopy-reg"), (12, 256, "", "", "3", "zcopy-reg"),
    (8, 256, "", "", "", "zcopy-single"), (6, 256, "tree", "", "", "zcopy-single"),
    (4, 256, "", "", "", "zcopy-steps")])
def test_c1_harness_host_sanitizers(monkeypatch, world, max_short, plan, incast, place,
                                    pipe):
    """The host engine (libucg_builtin.so sources) and the C1 harness rebuilt
    with ASan + UBSan (tests/c/Makefile, target asan): recursive and tree
    plans, fragmenting and resend-heavy sizes, the incast fan-in, waypoints
    forwarding fragment by fragment, the shared-memory remote-key steps
    (pipe = "zcopy"; at 8 members the one-shot reduce-scatter + all-gather,
    "zcopy-single" one pass over all buffers (at 6, the tree's), "zcopy-steps"
    the plan's steps). Any sanitizer report (invalid access, UB, leak at exit)
    fails the rank."""
    import json
    import subprocess
    cdir = os.path.join(os.path.dirname(__file__), "c")
    # one make at a time: pytest-xdist workers would otherwise rebuild the
    # same objects at once after a source change
    import fcntl
    with open(os.path.join(cdir, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", cdir, "asan"], check=True)
    exe = os.path.join(cdir, "_build", "asan", "c1_allreduce")
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=1:abort_on_error=0")
    monkeypatch.setenv("UBSAN_OPTIONS", "print_stacktrace=1")
    if plan:
        monkeypatch.setenv("UCX_BUILTIN_ALLREDUCE_PLAN", plan)
    if incast:
        monkeypatch.setenv("UCX_BUILTIN_SM_INCAST", incast)
    if pipe.startswith("zcopy"):
        monkeypatch.setenv("UCX_BUILTIN_SHM_ZCOPY_THRESH", "1")
        if pipe == "zcopy-reg":
            monkeypatch.setenv("C1_REGISTERED", "1")
        if pipe == "zcopy-single":
            monkeypatch.setenv("UCX_BUILTIN_SHM_ONESHOT_FULL", "1g")
        if pipe == "zcopy-steps":
            monkeypatch.setenv("UCX_BUILTIN_SHM_ONESHOT", "n")
    elif pipe:
        monkeypatch.setenv("UCX_BUILTIN_PIPELINE", pipe)
    if place:
        # placements (test_topology.py): hosts of C1_PPN, sockets of
        # C1_SOCKET; radix 2 so 4 hosts of 3 have an inter-host waypoint, and
        # a socket level from 4 members per host on
        ppn, _, sock = place.partition(":")
        monkeypatch.setenv("C1_PPN", ppn)
        if sock:
            monkeypatch.setenv("C1_SOCKET", sock)
        monkeypatch.setenv("UCX_BUILTIN_TREE_RADIX", "2")
        monkeypatch.setenv("UCX_BUILTIN_TREE_SOCKET_LEVEL_PPN_THRESH", "4")
    codes, outs = launch_exe(exe, world, (shm_name(), 200, max_short))
    assert codes == [0] * world, "\n".join(outs)
    for out in outs:
        assert "Sanitizer" not in out and "runtime error" not in out, out
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["bit_exact"] and line["ranks"] == world


def test_async_resend_timer_combines_on_its_thread():
    """the resend timer of the group's async context
    (builtin.c:260-294, 408-413) sends what stopped at UCS_ERR_NO_RESOURCE
    while the owner makes no call, then drains the stash - the combine runs on
    the timer's thread (tests/c/async_resend.c); results bit-exact."""
    exe = os.path.join(ROOT, "tests", "c", "_build", "async_resend")
    codes, outs = launch_exe(exe, 2, (shm_name(),), timeout=60)
    assert codes == [0, 0], "\n".join(outs)
    import json
    stats = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][0])
    assert stats["sent_before_sleep"] < 133 and stats["sent_after_sleep"] == 133
    assert stats["timer_resends"] > 0 and stats["timer_combines"] > 0


def test_async_resend_timer_four_members_rounded_inputs():
    """Row a15 at 4 members with rounded fp32 inputs: the
    timer thread sends member 0's step-1 fragments and combines the stash;
    every member's result equals, bit for bit, the oracle's simulation of the
    recursive-doubling plan (ucg_oracle_reduce_multi; builtin_recursive.c:
    158-169) - exact small-integer inputs could not tell an association
    error apart."""
    exe = os.path.join(ROOT, "tests", "c", "_build", "async_resend")
    codes, outs = launch_exe(exe, 4, (shm_name(), "host", "round"), timeout=60)
    assert codes == [0] * 4, "\n".join(outs)
    import json
    stats = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][0])
    assert stats["world"] == 4 and stats["inputs"] == "round"
    assert stats["sent_after_sleep"] >= 133 and stats["timer_combines"] > 0, stats


@pytest.mark.gpu
@pytest.mark.parametrize("mode,world,inputs", [("staged", 2, "exact"), ("device", 2, "exact"),
                                               ("staged", 4, "round"), ("device", 4, "round")])
def test_async_resend_timer_device_combines(mode, world, inputs):
    """Row a15 on the GPU: the resend timer's thread makes
    the combine's HIP calls. staged: host buffers with every step staged on
    the device, so the fragments the timer thread drains are device combines
    (ucg_builtin_dev_combine, stage_end); device: device buffers, remote-key
    steps, member 0's fold launched from its timer thread once its stuck
    messages go out. Results bit-exact, no host combine, no device error."""
    exe = os.path.join(ROOT, "tests", "c", "_build", "async_resend")
    codes, outs = launch_exe(exe, world, (shm_name(), mode, inputs), timeout=90)
    assert codes == [0] * world, "\n".join(outs)
    import json
    stats = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][0])
    assert stats["mode"] == mode and stats["world"] == world and stats["inputs"] == inputs
    assert stats["timer_resends"] > 0 and stats["timer_combines"] > 0, stats
    assert stats["host_calls"] == 0 and stats["device_calls"] > 0, stats


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["staged", "device"])
def test_async_resend_timer_device_failure_reaches_completion(monkeypatch, mode):
    """the timer thread's device combine fails (the next
    device call of member 0's process armed with
    ucg_builtin_dev_inject_failure just before its owner thread goes quiet):
    member 0's operation completes with that error, UCS_ERR_IO_ERROR, as the
    reference's recv_handle_error path ends an op (builtin_comp_step.inl:
    332-333, builtin.c:260-294); member 1 ends cleanly or, seeing that
    member 0 gave up on the op, with UCS_ERR_CANCELED - never with a wrong
    result, and without any member timed to meet the other (round 6: no
    sleep before the last barrier, whose status must be UCS_OK)."""
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "60")
    exe = os.path.join(ROOT, "tests", "c", "_build", "async_resend")
    codes, outs = launch_exe(exe, 2, (shm_name(), mode, "round", "fail"), timeout=120)
    assert codes == [0, 0], "\n".join(outs)
    import json
    lines = [json.loads(ln) for ln in outs[0].splitlines() if ln.startswith("{")]
    st0 = [x for x in lines if "status" in x][0]
    assert st0["rank"] == 0 and st0["status"] == -3 and st0["injected_fired"] == 1, st0
    st1 = [json.loads(ln) for ln in outs[1].splitlines() if ln.startswith("{")][-1]
    assert st1["status"] in (0, -16), st1          # UCS_OK or UCS_ERR_CANCELED


@pytest.mark.parametrize("mode,world,victim", [("exit-before", 3, 1), ("exit-before", 4, 0),
                                               ("exit-during", 4, 2), ("exit-during", 2, 0),
                                               ("cancel", 4, 3), ("cancel", 3, 0)])
def test_peer_failure_ends_ops_with_status_not_abort(monkeypatch, mode, world, victim):
    """a member that fails never takes its peers down. Its
    process gone (before or during the op): every survivor's op ends with
    UCS_ERR_CONNECTION_RESET and its close returns that status, within a
    fraction of the wait timeout, and the survivor exits 0 (no abort() in the
    barrier, the incast lock or close). A member that gives up on the op
    (destroys it while it runs): the others end it with UCS_ERR_CANCELED as
    soon as they see it published, and the last barrier and close succeed.
    The reference ends ops with a status (recv_handle_error,
    builtin_comp_step.inl:332-333)."""
    import json
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "60")
    codes, outs = launch("_worker_fail.py", world, args=(shm_name(), mode, victim),
                         timeout=120)
    for r in range(world):
        if r == victim and mode != "cancel":
            continue
        assert codes[r] == 0, "\n".join(outs)
        line = json.loads([ln for ln in outs[r].splitlines() if ln.startswith("{")][-1])
        if r == victim:
            assert line["close"] == 0, line
            continue
        want = _lib_status("UCS_ERR_CANCELED" if mode == "cancel" else
                           "UCS_ERR_CONNECTION_RESET")
        assert line["status"] == want and line["took_s"] < 20, (line, outs)
        assert line["close"] == (0 if mode == "cancel" else want), line
        assert "Aborted" not in outs[r] and "Fatal" not in outs[r], outs[r]


def _lib_status(name):
    from xucg_amd import _lib
    return getattr(_lib, name)


def test_job_token_skips_torchrun_none_run_id(monkeypatch):
    """torchrun sets TORCHELASTIC_RUN_ID=none for every
    static-rendezvous job; two such jobs must still get different tokens
    (from MASTER_ADDR:MASTER_PORT), and a real run id still decides."""
    from xucg_amd import _lib
    lib = _lib.host()
    for v in ("UCX_BUILTIN_JOB_TOKEN", "PMIX_NAMESPACE", "OMPI_MCA_ess_base_jobid",
              "SLURM_JOB_ID"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    a = lib.ucg_builtin_shm_job_token()
    monkeypatch.setenv("MASTER_PORT", "29501")
    b = lib.ucg_builtin_shm_job_token()
    assert a != 0 and b != 0 and a != b
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "f3a1c0de")
    c = lib.ucg_builtin_shm_job_token()
    monkeypatch.setenv("MASTER_PORT", "29500")
    assert lib.ucg_builtin_shm_job_token() == c and c not in (a, b)


@pytest.mark.parametrize("exe,world,args", [("component_test", 4, ("host",)),
                                             ("component_test", 3, ("host",)),
                                             ("async_resend", 2, None)])
def test_component_and_timer_host_sanitizers(monkeypatch, exe, world, args):
    """The plan component driven through its vtable, and the resend timer
    thread, with the engine rebuilt under ASan + UBSan."""
    import fcntl
    import subprocess
    cdir = os.path.join(os.path.dirname(__file__), "c")
    with open(os.path.join(cdir, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", cdir, "asan"], check=True)
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=1:abort_on_error=0")
    monkeypatch.setenv("UBSAN_OPTIONS", "print_stacktrace=1")
    codes, outs = launch_exe(os.path.join(cdir, "_build", "asan", exe), world,
                             args if args else (shm_name(),), timeout=120)
    assert codes == [0] * world, "\n".join(outs)
    for out in outs:
        assert "Sanitizer" not in out and "runtime error" not in out, out


@pytest.mark.parametrize("world,groups", [(4, 3), (2, 5), (3, 2)])
def test_groups_sharing_one_interface_with_timers(world, groups):
    """Several groups on one transport object, each with a resend timer
    thread, every group's allreduce in flight at once on a 2-cell ring
    (tests/c/multi_group_timers.c). Every group's progress and timer reach the
    shared rings and the group table, so the engine's lock is the
    interface's, as the reference's UCS_ASYNC_BLOCK is the worker's
    (builtin/builtin.c:263-267, 284-294, 331-335). Before round 6 it was the
    group's: two timers wrote the same ring cell and the members hung."""
    exe = os.path.join(ROOT, "tests", "c", "_build", "multi_group_timers")
    codes, outs = launch_exe(exe, world, (shm_name(), groups, 40), timeout=120)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.parametrize("exe,world,args", [("async_resend", 2, None),
                                             ("async_resend", 4, ("round",)),
                                             ("component_test", 4, ("host",)),
                                             ("multi_group_timers", 4, ("3", "40"))])
def test_engine_thread_sanitizer(monkeypatch, exe, world, args):
    """SURVEY 5, race detection: the host engine rebuilt with ThreadSanitizer
    (tests/c/Makefile, target tsan), with the resend timer's thread working
    against the owner thread (async_resend: the timer sends and combines
    while the owner sleeps, then both wait; the plan component with its
    timer running; several groups with timers on one interface). Any data
    race report fails the rank. Round 6 found three: ucg_builtin_lgroup_stats
    read the counters the timer thread writes without the group's lock; the
    interface's liveness state was plain fields; and groups sharing an
    interface each had a lock of their own for the shared rings."""
    import fcntl
    import subprocess
    cdir = os.path.join(os.path.dirname(__file__), "c")
    with open(os.path.join(cdir, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", cdir, "tsan"], check=True)
    monkeypatch.setenv("TSAN_OPTIONS", "halt_on_error=0 second_deadlock_stack=1")
    if exe == "async_resend":
        a = (shm_name(), "host") + (args or ())
    elif exe == "multi_group_timers":
        a = (shm_name(),) + args
    else:
        a = args
    codes, outs = launch_exe(os.path.join(cdir, "_build", "tsan", exe), world, a, timeout=180)
    assert codes == [0] * world, "\n".join(outs)
    for out in outs:
        assert "ThreadSanitizer" not in out, out


@pytest.mark.parametrize("world", [3, 4])
def test_completion_callback_and_flags(world):
    """ucg_params_t.completion (api/ucg.h:162-171) as
    ucg_builtin_comp_last_step_cb calls it (builtin_comp_step.inl:8-38): an
    allreduce completed by progress alone reports once through the callback
    with the caller's request, then - with no callback - through a flag byte
    and the status written into the request at the given offsets."""
    codes, outs = launch("_worker_comp.py", world, args=(shm_name(),), timeout=120)
    assert codes == [0] * world, "\n".join(outs)


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


def _digests(outs):
    per_rank = []
    for out in outs:
        per_rank.append(sorted(line for line in out.splitlines() if line.startswith("digest")))
    return per_rank


@pytest.mark.parametrize("world,max_short,cells,plan", [
    (3, 256, 64, None), (5, 64, 64, None), (6, 8192, 64, None), (7, 256, 2, None),
    (4, 256, 64, "tree"), (2, 64, 64, "tree")])
def test_tree_multiprocess_host(world, max_short, cells, plan, monkeypatch):
    """Tree fan-in / fan-out (builtin_tree.c:86-380): MPI_Reduce to several
    roots and the non-power-of-two MPI_Allreduce; plan='tree' forces the tree
    on a power-of-two group (UCX_BUILTIN_ALLREDUCE_PLAN)."""
    if plan:
        monkeypatch.setenv("UCX_BUILTIN_ALLREDUCE_PLAN", plan)
    codes, outs = launch("_worker_tree.py", world, args=(shm_name(), "host", max_short, cells),
                         timeout=240)
    assert codes == [0] * world, "\n".join(outs)
    d = _digests(outs)
    assert all(x == d[0] for x in d) and d[0], d     # every member holds the root's bits
    assert "REDUCE_TERMINAL" in outs[0] and "SEND_TERMINAL" in outs[0]
    assert ("SEND_TERMINAL, send send.buffer to 0" if world == 2 else "SEND_TO_SM_ROOT") in outs[1]
    assert "RECV_TERMINAL, receive from 0" in outs[1] and "aggregation write" in outs[1]


def test_tree_intra_restatement():
    """The oracle's ucg_builtin_tree_add_intra for one host (all members at
    DISTANCE_HOST): the root is every other member's only parent. The engine's
    plans are checked against it member by member in _worker_tree.py."""
    up, down = O.tree_intra(0, 5)
    assert up == [] and down == [1, 2, 3, 4]
    up, down = O.tree_intra(3, 5, root=1)
    assert up == [1] and down == []


def test_reductions_reject_minloc_and_noncommutative_ops():
    """builtin_control.c:872-888: a reducing plan refuses MPI_MINLOC/MAXLOC
    (is_loc_expected_f) and non-commutative ops (is_commutative_f) with
    UCS_ERR_UNSUPPORTED - here on every member, reducing or not."""
    from mock_mpi import OP_MINLOC
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    assert cmb.check_reduction(OP_MINLOC) == -22
    assert cmb.check_reduction(OPS["sum"]) == 0
    cmb.close()
    noncomm = MockMPI()
    noncomm.is_commutative_f = staticmethod(lambda op: op != OPS["prod"])
    cmb = host.BuiltinCombine(noncomm.callbacks(), host.make_config(dev_enable=0))
    assert cmb.check_reduction(OPS["prod"]) == -22
    cmb.close()
    # through the engine: a 2-member group, member 0's view (no message sent)
    iface = ops.ShmIface(shm_name(), 1, 0, max_short=256)
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    g = ops.Group(iface, 3, 1, 0, cmb)
    x = np.arange(16, dtype=np.int32)
    y = np.zeros_like(x)
    # a one-member group has no reducing step: nothing to refuse
    c = g.allreduce(x, y, 16, DTYPES["int32"], OP_MINLOC)
    assert c.status == 0
    c.close()
    g.close()
    iface.close()
    cmb.close()


def test_allreduce_rejects_bad_reduce_root():
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    iface = ops.ShmIface(shm_name(), 1, 0, max_short=256)
    g = ops.Group(iface, 3, 1, 0, cmb)
    x = np.arange(16, dtype=np.int32)
    y = np.zeros_like(x)
    assert g.reduce(x, y, 16, DTYPES["int32"], OPS["sum"], root=1).status == -5
    c = g.reduce(x, y, 16, DTYPES["int32"], OPS["sum"], root=0)
    assert c.status == 0 and c.run() == 0 and (y == x).all()
    assert "reduce" in c.describe()
    c.close()
    g.close()
    iface.close()
    cmb.close()


@pytest.mark.parametrize("world,max_short,cells", [(3, 256, 64), (5, 64, 64), (7, 256, 2),
                                                 (6, 8192, 4)])
def test_tree_incast_packers(world, max_short, cells, monkeypatch):
    """SM-root incast: children pack into one cell at the
    root - reducing packer (copy, then dst = mine (op) dst) or, for unsigned
    SUM, the atomic packer - and the root receives one message per fragment."""
    monkeypatch.setenv("UCX_BUILTIN_SM_INCAST", "y")
    codes, outs = launch("_worker_tree.py", world, args=(shm_name(), "host", max_short, cells),
                         timeout=240)
    assert codes == [0] * world, "\n".join(outs)
    d = _digests(outs)
    assert all(x == d[0] for x in d) and d[0], d
    assert "incast (reducing packer)" in outs[1] and "incast (atomic packer)" in outs[1]
    root_plan = [ln for ln in outs[0].splitlines() if "REDUCE_TERMINAL" in ln][0]
    assert "incast" in root_plan


@pytest.mark.parametrize("world,max_short,cells", [(3, 256, 64), (5, 64, 64), (7, 256, 2),
                                                 (6, 8192, 4)])
def test_tree_incast_batched(world, max_short, cells, monkeypatch):
    """The BATCHED_DATA receive (builtin_comp_step.inl:242-273, SURVEY 8a row
    a4): every child copies its fragment into its own slot of one cell at the
    root, which receives the cell as one message and reduces the children's
    chunks in arrival order; integer and exact-fp results bit-exact against
    the oracle's tree, rounded fp within tolerance and identical on every
    member."""
    monkeypatch.setenv("UCX_BUILTIN_SM_INCAST", "batched")
    codes, outs = launch("_worker_tree.py", world, args=(shm_name(), "host", max_short, cells),
                         timeout=240)
    assert codes == [0] * world, "\n".join(outs)
    d = _digests(outs)
    assert all(x == d[0] for x in d) and d[0], d
    assert "incast (batched packer)" in outs[1]
    root_plan = [ln for ln in outs[0].splitlines() if "REDUCE_TERMINAL" in ln][0]
    assert "incast (batched)" in root_plan


@pytest.mark.gpu
@pytest.mark.parametrize("world,max_short,cells,incast", [(5, 8192, 4, "y"), (3, 256, 64, "y"),
                                                        (5, 8192, 4, "batched")])
def test_tree_incast_packers_device(world, max_short, cells, incast, monkeypatch):
    """The SM-root packers on the GPU box (SURVEY 8a row a13, 8f row f4;
    builtin_pack.c:50-72, 100-148): with every combine forced onto the device,
    a child's reducing packer combines its data into the root's incast cell
    through the device path (H2D -> kernel -> D2H on the cell), the atomic
    packer adds unsigned SUMs into the zeroed cell; results bit-exact against
    the oracle's tree."""
    monkeypatch.setenv("UCX_BUILTIN_SM_INCAST", incast)
    codes, outs = launch("_worker_tree.py", world, args=(shm_name(), "dev", max_short, cells),
                         timeout=300)
    assert codes == [0] * world, "\n".join(outs)
    d = _digests(outs)
    assert all(x == d[0] for x in d) and d[0], d
    if incast == "y":
        assert "incast (reducing packer)" in outs[1] and "incast (atomic packer)" in outs[1]
        # a child's packers combined on the device
        stats = [ln for ln in outs[world - 1].splitlines() if ln.startswith("stats ")][0]
    else:
        # batched: the root combines every child's chunk, staged on the device
        assert "incast (batched packer)" in outs[1]
        stats = [ln for ln in outs[0].splitlines() if ln.startswith("stats ")][0]
    dev_calls = int(stats.split("'dev_calls': ")[1].split(",")[0])
    dev_steps = int(stats.split("'dev_steps': ")[1].split(",")[0])
    assert dev_calls + dev_steps > 0, stats


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 8])
def test_engine_group_churn_device_buffers(world):
    """Groups on device buffers created and destroyed 12 times per process,
    buffers of three recurring sizes freed and allocated in between, half of
    them sent from the group's registered (exported pool) memory: IPC keys
    are (pid, address, size) and recur, and every allreduce must still equal
    the oracle's association bit for bit (stale keys)."""
    import uuid
    codes, outs = launch("_worker_churn.py", world, args=(f"ucg_churn_{uuid.uuid4().hex[:8]}", 12),
                         timeout=180)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [3, 5])
def test_tree_multiprocess_device_staging(world):
    """Tree root's fan-in staged on the GPU: children's fragments at the same
    offsets become separate runs applied in arrival order."""
    codes, outs = launch("_worker_tree.py", world, args=(shm_name(), "dev", 256),
                         timeout=300)
    assert codes == [0] * world, "\n".join(outs)
    d = _digests(outs)
    assert all(x == d[0] for x in d), d


@pytest.mark.parametrize("seed,world,max_short,cells,env", [
    (1, 2, 256, 64, {}), (2, 3, 64, 2, {}), (3, 4, 1024, 8, {}), (4, 5, 256, 64, {}),
    (5, 6, 8192, 4, {"UCX_BUILTIN_SM_INCAST": "y"}), (6, 7, 64, 64, {}),
    (7, 8, 256, 3, {}), (8, 4, 128, 64, {"UCX_BUILTIN_ALLREDUCE_PLAN": "tree",
                                          "UCX_BUILTIN_SM_INCAST": "y"})])
def test_engine_fuzz(seed, world, max_short, cells, env, monkeypatch):
    """A seeded random sequence of 40 allreduce/reduce ops per configuration
    (world 2-8, max_short 64-8192, rings of 2-64 cells, incast on/off), every
    result bit-exact against the oracle's plan simulation."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    codes, outs = launch("_worker_fuzz.py", world, args=(shm_name(), seed, max_short, cells),
                         timeout=300)
    assert codes == [0] * world, "\n".join(outs)


ZC_FUZZ = [(11, 2, 256, 64), (12, 3, 256, 3), (13, 4, 128, 8), (14, 5, 256, 64),
           (15, 8, 256, 4), (16, 6, 1024, 64)]


@pytest.mark.parametrize("where", ["shm", "shm-reg"])
@pytest.mark.parametrize("seed,world,max_short,cells", ZC_FUZZ)
def test_engine_fuzz_shm_zcopy(seed, world, max_short, cells, where, monkeypatch):
    """The seeded 40-op sequence on the shared-memory remote-key steps: random
    integer dtype/op or exact fp SUM, count 0-6000, allreduce or reduce to a
    random root, in place or not, rings of 3-64 cells; with send buffers from
    the group's registered memory in the -reg runs."""
    monkeypatch.setenv("FUZZ_BUFFERS", where)
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "60")
    codes, outs = launch("_worker_fuzz.py", world, args=(shm_name(), seed, max_short, cells),
                         timeout=300)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["device", "device-reg"])
@pytest.mark.parametrize("seed,world,max_short,cells", ZC_FUZZ)
def test_engine_fuzz_device_buffers(seed, world, max_short, cells, where, monkeypatch):
    """The same sequence on device buffers: the remote-key steps, the one-shot
    execution (4 and 8 members), registered send buffers, in place or not."""
    monkeypatch.setenv("FUZZ_BUFFERS", where)
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "90")
    codes, outs = launch("_worker_fuzz.py", world, args=(shm_name(), seed, max_short, cells),
                         timeout=150)
    assert codes == [0] * world, "\n".join(outs)


@pytest.mark.parametrize("thresh,shm", [("8k", True), ("8192", True), ("9k", False),
                                        ("0.5m", False), ("", False)])
def test_shm_zcopy_thresh_memunits(thresh, shm, monkeypatch):
    """UCX_BUILTIN_SHM_ZCOPY_THRESH takes UCX memunits like the other size
    knobs (k/m/g suffixes, empty = off): an 8 KiB host op takes the
    shared-memory remote-key steps from 8k down, not from 9k up."""
    monkeypatch.setenv("UCX_BUILTIN_SHM_ZCOPY_THRESH", thresh)
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    iface = ops.ShmIface(shm_name(), 1, 0, max_short=256)
    g = ops.Group(iface, 3, 1, 0, cmb)
    x = np.arange(2048, dtype=np.int32)
    y = np.zeros_like(x)
    c = g.allreduce(x, y, 2048, DTYPES["int32"], OPS["sum"])
    assert c.status == 0 and c.run() == 0 and (y == x).all()
    assert ("Buffers: shared memory" in c.describe()) == shm, c.describe()
    c.close()
    g.close()
    iface.close()
    cmb.close()


def test_rma_pool_size_classes(monkeypatch):
    """Ops of many different sizes share the group's registered buffers:
    the pool grows by size class (eight per power of two, at most twice the
    class per reuse), not by every distinct message size, since a buffer is
    only returned when the group is destroyed. 300 shared-memory remote-key
    ops of random sizes in [64 KiB, 1 MiB] leave at most 2 x 8 x 4 segments."""
    import glob
    import os
    monkeypatch.setenv("UCX_BUILTIN_SHM_ZCOPY_THRESH", "1")
    mpi = MockMPI()
    cmb = host.BuiltinCombine(mpi.callbacks(), host.make_config(dev_enable=0))
    iface = ops.ShmIface(shm_name(), 1, 0, max_short=256)
    g = ops.Group(iface, 3, 1, 0, cmb)
    rng = np.random.default_rng(7)
    segs = lambda: glob.glob(f"/dev/shm/xucg_rma_{os.getpid()}_*")
    before = len(segs())
    for n in rng.integers(1 << 16, 1 << 20, 300):
        x = rng.integers(0, 255, int(n), dtype=np.uint8)
        y = np.zeros_like(x)
        c = g.allreduce(x, y, int(n), DTYPES["uint8"], OPS["sum"])
        assert c.status == 0 and c.run() == 0 and (y == x).all()
        assert "Buffers: shared memory" in c.describe()
        c.close()
    grown = len(segs()) - before
    assert 2 <= grown <= 64, grown
    g.close()
    assert len(segs()) == before
    iface.close()
    cmb.close()


ASSOC_CASES = [  # (world, kind, keys)
    (2, "allreduce", ()), (4, "allreduce", ()), (8, "allreduce", ()),
    (4, "allreduce", ("factor=4",)), (16, "allreduce", ("factor=4",)),
    (8, "allreduce", ("factor=4",)),                  # not a power of 4: one-host tree
    (3, "allreduce", ()), (5, "allreduce", ()), (6, "allreduce", ()),
    (5, "reduce", ("root=0",)), (5, "reduce", ("root=3",)),
    (8, "allreduce", ("ppn=4",)), (8, "allreduce", ("ppn=2",)),
    (6, "allreduce", ("ppn=3",)), (12, "allreduce", ("ppn=4",)),
]


@pytest.mark.parametrize("transport", ["am", "remote_key"])
@pytest.mark.parametrize("world,kind,keys", ASSOC_CASES)
def test_association_traced_against_reference_text(world, kind, keys, transport):
    """The engine's actual reduction trees, recorded by a reduce_cb_f that
    writes "(" src dst ")" into dst, checked against trees derived from the
    reference's text (tests/_worker_assoc.py). This pins the association the
    GPU's one-shot kernels reproduce without going through the planner code
    or oracle/plans.py: recursive doubling and K-ing, the one-host and
    multi-host fan-in/fan-out trees of groups that are not a power of two,
    MPI_Reduce to a non-zero root, and host fan-in + recursive doubling over
    host masters + fan-out. Several fragments per step (max_short 256: 3
    elements of 64 B per fragment); `remote_key`: every message on the
    shared-memory remote-key steps."""
    env = {"UCX_BUILTIN_SHM_ZCOPY_THRESH": "1"} if transport == "remote_key" else None
    codes, outs = launch("_worker_assoc.py", world,
                         args=(shm_name(), kind, 256, 10) + keys, timeout=120, env_extra=env)
    assert codes == [0] * world, "\n".join(outs)
    rows = {}   # member -> the hashes of its result, one per start
    for r, out in enumerate(outs):
        for line in out.splitlines():
            if " rows " in line:
                rows.setdefault(r, []).append(line.split(" rows ")[1])
    kv = dict(k.split("=") for k in keys)
    if kind == "reduce":
        assert list(rows) == [int(kv["root"])]
        return
    assert sorted(rows) == list(range(world))
    ppn, factor = int(kv.get("ppn", world)), int(kv.get("factor", 2))
    one_tree = world & (world - 1) or (ppn == world and factor ** round(
        np.log(world) / np.log(factor)) != world)
    for r in range(world):
        # a fanned-out result is a copy of the root's (the tree) or of the
        # host master's (recursive over masters), start by start
        src = 0 if one_tree else (r - r % ppn if ppn < world else r)
        assert rows[r] == rows[src], (r, src, rows)


def _stamped_object(name, owner, size=1 << 16):
    """/dev/shm/<name> with the iface header of a set-up object (builtin_shm.c
    seg_hdr_t: stamp at byte 64, then owner pid, instance, bytes, members)"""
    import struct
    path = "/dev/shm/" + name
    with open(path, "wb") as f:
        f.write(b"\0" * size)
        f.seek(64)
        f.write(struct.pack("<QQQQQ", 0x58554347534d3031, owner, 0x1234, size, 1))
    return path


def test_shm_iface_replaces_a_dead_jobs_object():
    """an object left by a crashed job (its creator's pid is
    gone) is unlinked and made anew by member 0, not shared."""
    import subprocess
    from xucg_amd import ops
    dead = subprocess.Popen(["true"])
    dead.wait()
    name = shm_name()
    path = _stamped_object(name, dead.pid)
    it = ops.ShmIface(name, 1, 0)
    try:
        import struct
        with open(path, "rb") as f:
            f.seek(64)
            stamp, owner = struct.unpack("<QQ", f.read(16))
        assert owner == os.getpid() and stamp == 0x58554347534d3031
    finally:
        it.close()
    assert not os.path.exists(path)


def test_shm_iface_refuses_a_live_jobs_object():
    """two live jobs under one name (no job uid) no longer share
    rings: member 0 of the second gets UCS_ERR_BUSY."""
    import xucg_amd
    from xucg_amd import ops
    name = shm_name()
    path = _stamped_object(name, os.getppid())       # a live process
    try:
        with pytest.raises(xucg_amd.UcsError) as e:
            ops.ShmIface(name, 1, 0)
        assert e.value.status == -15
    finally:
        os.unlink(path)


def _fnv1a64(text):
    """builtin_shm.c job_token(): FNV-1a of the token text"""
    h = 0xcbf29ce484222325
    for c in text.encode():
        h = ((h ^ c) * 0x100000001b3) & ((1 << 64) - 1)
    return h or 1


def _stamp_extra(path, pidns, job):
    """the round-5 header fields after members: pid namespace, job token"""
    import struct
    with open(path, "r+b") as f:
        f.seek(104)
        f.write(struct.pack("<QQ", pidns, job))


def test_shm_iface_peer_refuses_another_jobs_live_object(monkeypatch):
    """member 1 of a second job that shares the first job's name
    and layout no longer maps the first job's live object (its barrier would
    have thrown that job's barriers out of step): the object carries the
    creating job's token, and a member of another job is refused with
    UCS_ERR_BUSY at once."""
    import subprocess
    import sys
    import time
    import struct
    import xucg_amd
    name = shm_name()
    env = dict(os.environ, UCX_BUILTIN_JOB_TOKEN="job-A", UCX_BUILTIN_WAIT_TIMEOUT="20",
               PYTHONPATH=ROOT)
    # job A's member 0: creates and stamps the object, then waits for member 1
    a = subprocess.Popen([sys.executable, "-c",
                          "from xucg_amd import ops; ops.ShmIface(%r, 2, 0)" % name],
                         env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        path = "/dev/shm/" + name
        t0 = time.time()
        while time.time() - t0 < 30:
            try:
                with open(path, "rb") as f:
                    f.seek(64)
                    if struct.unpack("<Q", f.read(8))[0] == 0x58554347534d3031:
                        break
            except (OSError, struct.error):
                pass
            time.sleep(0.01)
        else:
            pytest.fail("job A's object never stamped")
        monkeypatch.setenv("UCX_BUILTIN_JOB_TOKEN", "job-B")
        t1 = time.time()
        with pytest.raises(xucg_amd.UcsError) as e:
            ops.ShmIface(name, 2, 1)
        assert e.value.status == -15 and time.time() - t1 < 5
    finally:
        a.kill()
        a.wait()
        try:
            os.unlink("/dev/shm/" + name)
        except OSError:
            pass


@pytest.mark.parametrize("ours", [False, True])
def test_shm_iface_creator_in_another_pid_namespace(monkeypatch, ours):
    """a creator pid of another pid namespace (containers sharing
    /dev/shm) means nothing to kill() here. Member 0 treats such an object as
    live - UCS_ERR_BUSY - unless it carries this job's own token, which makes
    it an earlier incarnation of this job to recycle; it is never judged by
    a pid that happens to be free (or taken) in this namespace."""
    import subprocess
    import xucg_amd
    monkeypatch.setenv("UCX_BUILTIN_JOB_TOKEN", "job-ns")
    dead = subprocess.Popen(["true"])
    dead.wait()
    name = shm_name()
    path = _stamped_object(name, dead.pid)
    _stamp_extra(path, 0x7fffffff12345, _fnv1a64("job-ns") if ours else 0x1234)
    try:
        if ours:
            it = ops.ShmIface(name, 1, 0)
            it.close()
        else:
            with pytest.raises(xucg_amd.UcsError) as e:
                ops.ShmIface(name, 1, 0)
            assert e.value.status == -15
    finally:
        if os.path.exists(path):
            os.unlink(path)


def test_shm_iface_reopened_at_once_by_every_member():
    """Close and reopen of one name in a loop by 4 members: a member that
    reopens before member 0 unlinked the closed object waits for the new
    instance (the barrier of each instance would hang otherwise)."""
    codes, outs = launch("_worker_reopen.py", 4, args=(shm_name(), 30), timeout=120)
    assert codes == [0] * 4, "\n".join(outs)


@pytest.mark.gpu
def test_group_destroy_parks_buffers_a_peer_may_read(monkeypatch):
    """an op on device buffers that ends before every peer is done
    (here: a timeout, member 1 never starting) leaves its exposed buffer taken,
    and destroying the group parks it (ucg_builtin_dev_park) rather than
    returning it to the reuse cache, where the next allocation of its size
    would change it under the reader."""
    monkeypatch.setenv("UCX_BUILTIN_WAIT_TIMEOUT", "8")
    codes, outs = launch("_worker_park.py", 2, args=(shm_name(),), timeout=150)
    assert codes == [0, 0], "\n".join(outs)
    assert "parked" in outs[0], outs[0]
