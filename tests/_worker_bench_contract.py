"""One rank (gloo, CPU) of the test of bench.py's multi-GPU contract: every
phase guarded and agreed on by all ranks, every failed check surfacing in
collective_failures (so the line carries collective_ok false and the run
exits non-zero), and the sampled parity check of the C5 phases - the plan's
association evaluated on the host over windows of every rank's input -
agreeing with the oracle and catching a changed element."""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out, rc = {}, 0

    def fail(msg):
        nonlocal rc
        print(f"rank {rank}: FAIL {msg}", flush=True)
        rc = 1

    def raise_on_last():
        if rank == world - 1:
            raise RuntimeError("peer mapping failed")
        return {"ms": 1.0}

    bench.agreed_phase(out, "good", lambda: {"ms": 1.0, "bit_exact_vs_x": True}, dist, "cpu")
    bench.agreed_phase(out, "raises_on_one_rank", raise_on_last, dist, "cpu")
    bench.agreed_phase(out, "mismatch", lambda: {"inner": {"bit_exact_vs_x": False}},
                       dist, "cpu")
    bench.agreed_phase(out, "tolerance", lambda: {"rccl_within_8c_tolerance": False},
                       dist, "cpu")
    bench.agreed_phase(out, "skipped", lambda: {"skipped": "not a power of two"}, dist, "cpu")
    fails = bench.collective_failures(out)
    want = {"raises_on_one_rank", "mismatch.inner.bit_exact_vs_x",
            "tolerance.rccl_within_8c_tolerance"}
    got = {f.split(":")[0] for f in fails}
    if got != want:
        fail(f"collective_failures {fails}")
    if bench.collective_failures({"a": {"bit_exact_x": True}, "b": {"skipped": "x"}}):
        fail("a clean result reported failures")

    # the sampled parity of the C5 phases vs the oracle's recursive doubling
    n = 1 << 17
    xs = [O.fill("float64", "round", 0x5EED5000 + r, n) for r in range(world)]
    init = torch.from_numpy(xs[rank].copy())
    check = bench.sampled_plan_check(dist, init, rank, world)[0]
    acc = torch.from_numpy(O.reduce_multi("sum", "float64", xs, rank))
    if not check(acc):
        fail("the plan's result fails the sampled check")
    acc[n - 1] = np.nextafter(acc[n - 1].item(), np.inf)       # the tail window
    if check(acc):
        fail("a changed element passed the sampled check")

    # phase budgets: every rank takes the slowest rank's elapsed time, so all
    # skip or all run (rank r pretends to have run r x 10 s)
    t_start = time.perf_counter() - 10.0 * rank
    need = bench.PHASE_MIN_S["c4_oneshot_xgmi_rs_4gib_fp32"]
    for limit, want_skip in ((need + 10.0 * (world - 1) + 5, False),
                             (need + 10.0 * (world - 1) - 5, True)):
        sk = bench.phase_budget_skip(dist, "cpu", t_start, limit, "c4_oneshot_xgmi_rs_4gib_fp32")
        if (sk is not None) != want_skip or (sk and "budget" not in sk["skipped"]):
            fail(f"phase_budget_skip({limit}) = {sk}")

    # the C4 phases' parity without a 4 GiB vendor collective (PlanWindows):
    # every shard's windows against the oracle's recursive doubling as that
    # shard's owner evaluates it, and one changed element caught
    from xucg_amd import group as G
    n4 = world << 16
    x4 = [O.fill("float32", "round", 0x5EED4100 + r, n4) for r in range(world)]
    plan = bench.PlanWindows(dist, torch.from_numpy(x4[rank].copy()), n4, rank, world, "cpu")
    full = np.empty(n4, np.float32)
    for r in range(world):
        lo, hi = G.shard_bounds(n4, 4, world, r)
        full[lo:hi] = O.reduce_multi("sum", "float32", x4, r)[lo:hi]
    lo, hi = G.shard_bounds(n4, 4, world, rank)
    mine = torch.from_numpy(full[lo:hi].copy())
    if not (plan.rs_ok(mine) and plan.full_ok(torch.from_numpy(full))):
        fail("the plan's result fails PlanWindows")
    mine[-1] = float(np.nextafter(mine[-1].item(), np.inf, dtype=np.float32))
    bad = full.copy()
    bad[0] = np.nextafter(bad[0], np.float32(np.inf))
    if plan.rs_ok(mine) or plan.full_ok(torch.from_numpy(bad)):
        fail("a changed element passed PlanWindows")

    # the 1-GPU rehearsal's stand-in for RCCL (bench.HostStagedDist) against
    # gloo's own results, on CPU tensors
    from xucg_amd import group as G
    pg = bench.HostStagedDist(dist)
    x = torch.arange(world * 6, dtype=torch.float64) * (rank + 1)
    ref = x.clone()
    dist.all_reduce(ref)
    a = x.clone()
    pg.all_reduce(a)
    if not torch.equal(a, ref):
        fail("HostStagedDist.all_reduce")
    rs = torch.empty(6, dtype=torch.float64)
    pg.reduce_scatter_tensor(rs, x)
    if not torch.equal(rs, ref.view(world, 6)[rank]):
        fail("HostStagedDist.reduce_scatter_tensor")
    ag = torch.empty(world * 6, dtype=torch.float64)
    pg.all_gather_into_tensor(ag, rs)
    parts = [torch.empty(6, dtype=torch.float64) for _ in range(world)]
    pg.all_gather(parts, rs)
    if not (torch.equal(ag, ref) and torch.equal(torch.cat(parts), ref)):
        fail("HostStagedDist.all_gather(_into_tensor)")
    flag = torch.tensor([float(rank)])
    pg.all_reduce(flag, op=pg.ReduceOp.MAX)
    if flag.item() != world - 1:
        fail("HostStagedDist.all_reduce MAX")
    send, recv = torch.full((5,), float(rank)), torch.empty(5)
    G.torch_exchange(pg)(send, recv, rank ^ 1)
    if not torch.equal(recv, torch.full((5,), float(rank ^ 1))):
        fail("HostStagedDist point-to-point exchange")
    objs = [None] * world
    pg.all_gather_object(objs, rank)
    if objs != list(range(world)):
        fail("HostStagedDist.all_gather_object")
    pg.barrier()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: {'ok' if rc == 0 else 'FAILED'}", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
