"""One rank (gloo, CPU) of the test of bench.py's multi-GPU contract: every
phase guarded and agreed on by all ranks, every failed check surfacing in
collective_failures (so the line carries collective_ok false and the run
exits non-zero), and the sampled parity check of the C5 phases - the plan's
association evaluated on the host over windows of every rank's input -
agreeing with the oracle and catching a changed element."""
import os
import sys

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
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: {'ok' if rc == 0 else 'FAILED'}", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
