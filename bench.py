#!/usr/bin/env python3
"""Benchmark of the MI355X combine path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one device-resident local combine dst[i] = src[i] + dst[i] of the
BASELINE config-2 workload (2 x 256 MiB fp32, 2^26 elements) through the
C-ABI (ucg_builtin_dev_reduce). With N > 1 (launched by torch.distributed.run)
every rank combines its own shard-sized buffers: the path is element-wise, so
it shards with no data-path collective (weak scaling); `value` is the
aggregate over all ranks divided by the max-over-ranks wall time.

Printed by rank 0 as ONE JSON line, with:
  roofline      the combine kernel's average duration from HIP events on the
                stream it is launched on -> algorithmic GB/s vs 8 TB/s HBM3E
  cpu_baseline  the CPU restatement of the reference's combine (oracle/,
                compiled -march=native on this host), 1 thread, bounded sample
  extra         north-star 1 GiB fp32 combine, H2D/D2H-inclusive rate
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)
WORKLOAD_COUNT = 1 << 26  # BASELINE.json configs[1]: two 256 MiB fp32 buffers


def load_baseline_metric():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        return json.load(f)["metric"]


def lib_sha16(path):
    """first 16 hex digits of the sha256 of a file (None if unreadable)"""
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_traffic(count):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json), and where it comes from: the profile, the
    device code it was measured on and whether that is the code loaded now.
    The key is the hash of the library's .hip_fatbin section - its kernels'
    code objects (_lib.code_object_sha16) - so a host-only edit of the
    library does not stale kernel counters; a summary
    without it falls back to the whole-library hash. Stale when they differ:
    the figure is then other kernels'. Not a measurement of this run - PMC
    counters need their own profiler passes."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    from xucg_amd import _lib
    loaded = lib_sha16(_lib.DEV_LIB)
    code = _lib.code_object_sha16()
    try:
        with open(path) as f:
            e = json.load(f).get(str(count))
    except (OSError, ValueError):
        e = None
    if e is None:
        return None, {"profile": None, "stale": True, "lib_sha16_loaded": loaded,
                      "code_sha16_loaded": code}
    if e.get("code_sha16"):
        key, stale = "code object (.hip_fatbin)", e["code_sha16"] != code
    else:
        key, stale = "whole library", e.get("lib_sha16") is None or e.get("lib_sha16") != loaded
    return e.get("hbm_bytes_per_launch"), {
        "profile": "profiles/pmc_traffic.json <- " + str(e.get("source")),
        "kind": "committed rocprofv3 PMC summary (FETCH_SIZE x 2 + WRITE_SIZE), not this run",
        "keyed_by": key,
        "code_sha16_profiled": e.get("code_sha16"), "code_sha16_loaded": code,
        "lib_sha16_profiled": e.get("lib_sha16"), "lib_sha16_loaded": loaded,
        "stale": stale}


def cpu_baseline(count, budget_s=10.0):
    """Time the oracle's whole-buffer combine (the reduce_cb_f call shape) on
    this host: 1 thread, fp32 SUM, same element count, ~budget_s of work."""
    from oracle import oracle as O
    os.environ.setdefault("UCG_ORACLE_LIB", O.build_native())
    O.LIB_PATH = os.environ["UCG_ORACLE_LIB"]
    O._lib = None
    src = O.fill("float32", "round", 0x5EED0000, count)
    dst = O.fill("float32", "round", 0x5EED0001, count)
    best, med = O.time_reduce("sum", "float32", src, dst, reps=3)
    reps = max(5, min(1000, int(budget_s / max(med, 1e-6))))
    t0 = time.perf_counter()
    best, med = O.time_reduce("sum", "float32", src, dst, reps=reps)
    wall = time.perf_counter() - t0
    frag = O.frag_length(8192, 4)
    _, med_frag = O.time_reduce("sum", "float32", src, dst, frag_bytes=frag, reps=5)
    threads = min(16, os.cpu_count() or 1)
    _, med_mt = O.time_reduce("sum", "float32", src, dst, threads=threads, reps=5)
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    b = 3 * count * 4
    # the combine the reference itself calls: reduce_cb_f = the MPI library's
    # MPI_Reduce_local (MPICH 3.3.2 in this image), same count, 1 thread
    mpich = None
    exe = os.path.join(ROOT, "oracle", "_build", "mpich_bench")
    if os.path.exists(exe):
        import subprocess
        try:
            p = subprocess.run([exe, str(count), "6", "8192"], capture_output=True, text=True,
                               timeout=60)
            mpich = json.loads(p.stdout.strip().splitlines()[-1])
        except Exception as e:  # reported, never fatal for the bench line
            mpich = {"error": f"{type(e).__name__}: {e}"[:300]}
    return {
        "value": round(b / med / GIB, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle/combine_ref.c (-O3 -march=native) whole-buffer fp32 SUM of "
                   f"2^{count.bit_length() - 1} elements (the reduce_cb_f call shape), "
                   f"{reps} reps, median, {wall:.1f} s of CPU work"),
        "best_gibs": round(b / best / GIB, 3),
        "fragmented_8k_gibs": round(b / med_frag / GIB, 3),
        f"threads_{threads}_gibs": round(b / med_mt / GIB, 3),
        "cpu_model": cpu_model,
        "online_cpus": os.cpu_count(),
        "reference_callback_mpich": mpich,
    }


def c1_loopback(ranks=4, iters=20000):
    """BASELINE config 1 on this host's CPUs: 4 processes allreduce 4 KiB fp32
    through the builtin operation engine over the shared-memory transport
    (tests/c/c1_allreduce.c; host combine, no GPU). Latency per allreduce.
    max_short_*: the reference's plan for 4 members (recursive doubling);
    tree_*: the tree plan forced on 4 members, plain and with the SM-root
    incast packers; tree_3_ranks: the non-power-of-two case; device_*: the
    same harness on device buffers (remote-key steps, the one-shot execution
    at 4 members) with the send buffer in the group's registered memory, at
    4 KiB and 64 MiB."""
    import subprocess
    import uuid
    exe = os.path.join(ROOT, "tests", "c", "_build", "c1_allreduce")
    dev = {"C1_DEVICE_BUFFERS": "1", "C1_REGISTERED": "1", "UCX_BUILTIN_WAIT_TIMEOUT": "60"}
    variants = [("max_short_256", ranks, 256, {}), ("max_short_8192", ranks, 8192, {}),
                ("tree_max_short_256", ranks, 256, {"UCX_BUILTIN_ALLREDUCE_PLAN": "tree"}),
                ("tree_incast_max_short_256", ranks, 256,
                 {"UCX_BUILTIN_ALLREDUCE_PLAN": "tree", "UCX_BUILTIN_SM_INCAST": "y"}),
                ("tree_3_ranks_max_short_256", 3, 256, {}),
                ("device_buffers_4kib", ranks, 256, dev, 1024, 2000),
                ("device_buffers_64mib", ranks, 256, dev, 1 << 24, 20)]
    # the same allreduce through the drop-in boundary: ucg_builtin_component's
    # vtable driven as base/ drives it (tests/c/component_test.c, "latency":
    # the op prepared once, trigger + progress per start)
    variants.append(("component_vtable_max_short_256", ranks, 256,
                     {"UCX_BUILTIN_SHORT_MAX_TX_SIZE": "256"}, 1024, iters, "component"))
    comp_exe = os.path.join(ROOT, "tests", "c", "_build", "component_test")
    # one core per rank, as an MPI launcher binds them: the lowest-numbered
    # allowed CPUs (neighbours on one CCD on EPYC); unpinned ranks land on
    # random cores and the latency moves by 2x between runs
    allowed = sorted(os.sched_getaffinity(0))
    res = {"cpus": allowed[:max(v[1] for v in variants)]}
    for key, world, max_short, extra_env, *size in variants:
        name = f"ucg_bench_c1_{os.getpid()}_{uuid.uuid4().hex[:6]}"
        count, n_iter = size[:2] if size else (1024, iters)
        if size[2:] == ["component"]:
            # the component names its transport after the job uid (MASTER_PORT here)
            cmd = [comp_exe, "latency", str(n_iter), str(count)]
            extra_env = dict(extra_env, MASTER_PORT=str(20000 + int(uuid.uuid4().int % 40000)))
        else:
            cmd = [exe, name, str(n_iter), str(max_short), str(count)]
        procs = []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), **extra_env)
            cpu = allowed[r % len(allowed)]
            procs.append(subprocess.Popen(cmd,
                                          env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                          text=True,
                                          preexec_fn=lambda c=cpu: os.sched_setaffinity(0, {c})))
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=120)[0])
            except subprocess.TimeoutExpired:
                p.kill()
                outs.append(p.communicate()[0] + " <timeout>")
        try:
            res[key] = json.loads(outs[0].strip().splitlines()[-1])
        except (ValueError, IndexError):
            res[key] = {"error": outs[0][-300:]}
    return res


XGMI_GBS = 7 * 153.0   # aggregate xGMI per MI355X
# AMD's 153.6 GB/s per link counts both directions (as MI300X's 128 GB/s
# does); a reduce-scatter's ingress into one GPU uses one direction of each
# link, so its link roofline is 7 x 76.8 GB/s
XGMI_DIR_GBS = 7 * 76.8


def max_ulps(a, b):
    """Largest distance in units in the last place between two fp32/fp64
    tensors (sign-magnitude bits mapped onto a monotonic integer line)."""
    import torch
    ity = torch.int32 if a.dtype == torch.float32 else torch.int64
    mask = (1 << 31) - 1 if ity == torch.int32 else (1 << 63) - 1

    def key(t):
        i = t.view(ity).long()
        mag = i & mask
        return torch.where(i < 0, -mag, mag)
    return int((key(a) - key(b)).abs().max().item())


def staged_step(total=64 << 20, frag=8184, reps=5):
    """Row f1's device staging from C (tests/c/stage_bench.c): one fragmented
    fp32 SUM step, one ucg_builtin_dev_combine per 8 KiB AM fragment between
    stage_begin/stage_end, pageable host buffers, beside the 1-thread CPU
    combine issued per fragment. Child process; bit-exact check inside."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "c", "_build", "stage_bench")
    try:
        p = subprocess.run([exe, str(total), str(frag), str(reps)], capture_output=True,
                           text=True, timeout=120)
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, never fatal for the bench line
        return {"error": f"{type(e).__name__}: {e}"[:300]}


def collective_failures(res, path=""):
    """Every failed check in a collective result: an "error" entry (a phase
    that raised, on any rank) or a parity flag (bit_exact* / within*) that is
    False. Skipped phases are not failures. [] = all good."""
    out = []
    if isinstance(res, dict):
        for k, v in res.items():
            p = f"{path}.{k}" if path else k
            if k == "error":
                out.append(f"{path or '<top>'}: {v}")
            elif v is False and ("bit_exact" in k or "within" in k):
                out.append(p)
            elif isinstance(v, dict):
                out += collective_failures(v, p)
    return out


def agreed_phase(out, name, fn, dist, dev, rank=0, t_start=None):
    """Run one guarded phase on every rank: an exception becomes an "error"
    entry, and every rank records it when any rank failed (a MAX all-reduce
    of the failure flag), so the ranks never diverge on what ran."""
    import torch
    err = None
    if rank == 0 and t_start is not None:  # progress on stderr: never silent
        print(f"[collective] {name} starting at {time.perf_counter() - t_start:.1f} s",
              file=sys.stderr, flush=True)
    try:
        res = fn()
    except Exception as e:  # recorded, then agreed on by every rank
        res, err = None, f"{type(e).__name__}: {e}"[:300]
    flag = torch.tensor([1.0 if err else 0.0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if err or flag.item() > 0:
        out[name] = {"error": err or "failed on another rank"}
    else:
        out[name] = res


SAMPLE_ELEMS = 8192          # 64 KiB of fp64 per window

# rehearsal only (XUCG_COLLECTIVE_BACKEND=gloo, see HostStagedDist): the C4/C5
# buffers divided by this power of two; 1 in every real run
COLL_SCALE = int(os.environ.get("XUCG_COLLECTIVE_SCALE", "1"))


def sample_starts(n, elems=SAMPLE_ELEMS, k=16, seed=0x5EED5):
    """Windows for the sampled parity check: head, tail and k windows at
    random offsets (the same on every rank)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    return [0, n - elems] + sorted(int(x) for x in rng.integers(0, n - elems, size=k))


def host_butterfly(xs, self_index):
    """V(self, log2 N) of the reference's recursive doubling
    (builtin_recursive.c:158-169) on the host, element-wise over the rows of
    xs (member m's data in row m): val[m] holds member self ^ m's
    accumulator, and level h folds val[m + h] into val[m] - the partner's
    accumulator is the src of dst = src (+) dst. numpy's float64 add is one
    IEEE add, so this is the plan's result bit for bit."""
    n = len(xs)
    vals = [xs[self_index ^ m].copy() for m in range(n)]
    h = 1
    while h < n:
        for m in range(0, n, 2 * h):
            vals[m] = vals[m + h] + vals[m]
        h *= 2
    return vals[0]


def sampled_plan_check(dist, init, rank, world):
    """The plan's association evaluated on the host over sampled windows of
    every member's actual input (gathered from all ranks): returns
    check(acc) -> True when acc holds exactly those bits there, and the
    windows' expected values (for the RCCL tolerance check)."""
    import numpy as np
    import torch
    n = init.numel()
    starts = sample_starts(n)
    idx = torch.cat([torch.arange(s, s + SAMPLE_ELEMS, device=init.device) for s in starts])
    mine = init[idx].contiguous()
    allw = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allw, mine)
    xs = np.stack([a.cpu().numpy() for a in allw])
    want = host_butterfly(xs, rank)

    idx_h = idx.cpu().numpy()

    def check(acc):
        """True when acc holds the plan's bits on every window; on a
        mismatch, check.last says where (elements, shards of the one-shot
        layout) and whether the bad values are zeros or another member's
        association."""
        from xucg_amd import group as G
        got = acc[idx].cpu().numpy()
        bad = np.nonzero(got.view(np.int64) != want.view(np.int64))[0]
        check.last = None
        if bad.size:
            bounds = [G.shard_bounds(n, 8, world, r) for r in range(world)]
            shards = sorted({r for b in bad for r, (lo, hi) in enumerate(bounds)
                             if lo <= idx_h[b] < hi})
            others = [m for m in range(world)
                      if np.array_equal(got[bad].view(np.int64),
                                        host_butterfly(xs[:, bad], m).view(np.int64))]
            check.last = {"elements": int(bad.size), "of": int(got.size),
                          "first": [int(idx_h[b]) for b in bad[:4]],
                          "got": got[bad[:3]].tolist(), "want": want[bad[:3]].tolist(),
                          "zeros": int((got[bad] == 0).sum()), "shards": shards,
                          "equals_association_of_members": others}
        return not bad.size
    check.last = None
    return check, idx, want, xs


class PlanWindows:
    """The reference plan's result on sampled windows of every shard of one
    C4 buffer. Every rank contributes its input on the head, the tail and 16
    random windows of 8,192 elements of every shard (an all_gather of those
    windows only, so the check costs no 4 GiB collective); the result of
    shard r is V(r, log2 N), the owner's association of the recursive-doubling
    plan (host_butterfly; builtin_recursive.c:158-169), which is what the
    one-shot reduce-scatter writes there. rs_ok checks this rank's reduced
    shard, full_ok a whole buffer holding every shard (the all-gather or
    allreduce result)."""

    def __init__(self, dist, x, n, rank, world, dev):
        import numpy as np
        import torch
        from xucg_amd import group as G
        self.rank = rank
        self.bounds = [G.shard_bounds(n, 4, world, r) for r in range(world)]
        self.pos = []
        for lo, hi in self.bounds:
            w = min(SAMPLE_ELEMS, hi - lo)
            self.pos.append(torch.cat([torch.arange(lo + s0, lo + s0 + w, device=dev)
                                       for s0 in sample_starts(hi - lo, w)]))
        part = x[torch.cat(self.pos)].contiguous()
        allw = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(allw, part)
        xs = np.stack([a.cpu().numpy() for a in allw])      # member x position
        self.want, first = [], 0
        for r in range(world):
            k = self.pos[r].numel()
            self.want.append(host_butterfly(xs[:, first:first + k], r))
            first += k

    def rs_ok(self, shard_t):
        import numpy as np
        got = shard_t[self.pos[self.rank] - self.bounds[self.rank][0]].cpu().numpy()
        return bool(np.array_equal(got.view(np.int32), self.want[self.rank].view(np.int32)))

    def full_ok(self, full_t):
        import numpy as np
        import torch
        got = full_t[torch.cat(self.pos)].cpu().numpy()
        return bool(np.array_equal(got.view(np.int32), np.concatenate(self.want).view(np.int32)))


# whether the vendor collectives (RCCL, or the gloo stand-in of the 1-GPU
# rehearsal) run at C4's full size: the stand-in stages every tensor through
# host memory and cannot move 4 GiB per rank in time, so the full-size
# rehearsal (XUCG_COLLECTIVE_SCALE=1) skips those legs; parity then rests on
# the plan's sampled windows (PlanWindows), which every run checks anyway
VENDOR = [True]

# Time a phase must have left, of the collective child's limit, to start
# (seconds); the limit is XUCG_COLLECTIVE_LIMIT_S (default 280 of the parent's
# 300 s). A phase that would overrun is skipped and says so; one that
# overruns anyway costs its own entry only, since rank 0 saves the finished
# phases after each (XUCG_COLLECTIVE_OUT) and the parent reads them back.
PHASE_MIN_S = {"c4_rccl_rs_ag_4gib_fp32": 30, "c4_oneshot_xgmi_rs_4gib_fp32": 60,
               "c5_recursive_allreduce_512mib_fp64": 45,
               "c5_builtin_engine_device_buffers_512mib_fp64": 45}


def phase_budget_skip(dist, dev, t_start, limit, name):
    """None when phase `name` may start, else its "skipped" entry: it needs
    PHASE_MIN_S[name] seconds of the child's `limit` left. The elapsed time
    is max-reduced over the ranks first, so every rank decides alike."""
    import torch
    el = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    left, need = limit - el.item(), PHASE_MIN_S.get(name, 30)
    if left < need:
        return {"skipped": f"budget: {left:.0f} s left of the child's {limit:.0f} s, "
                           f"the phase needs {need} s"}
    return None


def read_child_result(path, rc, tail):
    """Rank 0's view of the collective child: the phases it saved (path), the
    one running when it was stopped marked as failed, and the child's exit
    status as an error entry when it did not end cleanly."""
    res = None
    try:
        with open(path) as f:
            res = json.load(f)
        os.unlink(path)
    except (OSError, ValueError):
        pass
    running = (res or {}).pop("running", None)
    if running:
        # killed inside a phase: that phase's entry says so, the finished
        # ones stand
        res[running] = {"error": f"the collective child was stopped inside this phase ({rc})"}
    if rc != 0 or res is None:
        res = dict(res or {}, error=f"collective child exited with {rc}", tail=tail)
    return res


def collective_phases(ctx, dist, rank, world, local_rank, steps=5, warmup=2, save=None):
    """BASELINE configs 4 and 5 across the N GPUs of the node (N > 1 only).

    C4: reduce-scatter + all-gather of a 4 GiB fp32 buffer
        (a) RCCL reduce_scatter_tensor + all_gather_into_tensor (ring order)
        (b) one-shot xGMI reduce-scatter: every GPU reads its 1/N shard from
            all N peer-mapped buffers and combines them in the reference
            plan's association (ucg_builtin_dev_reduce_multi), then RCCL
            all-gather; parity vs (a) on exact-integer inputs (bit-exact)
    C5: allreduce of 512 MiB fp64 per GPU, device combine per step:
        (a) the reference recursive-doubling plan (builtin_recursive.c:
            158-169): RCCL send/recv of the whole accumulator per step;
        (b) recursive halving + doubling with the plan's peer order (same
            per-element association, 2 (N-1)/N x S sent per rank);
        parity of both: bit-exact against a local one-shot evaluation of the
        plan's association; (c) RCCL all_reduce, checked against the
        SURVEY.md 8c tolerance
    busBW = (N-1)/N x S / t per collective, also as a fraction
    of the aggregate xGMI bandwidth (7 x 153 GB/s per GPU). Every phase is
    guarded; an error is recorded in the JSON instead of aborting the line."""
    import torch
    from xucg_amd import group as G

    dev = torch.device(f"cuda:{local_rank}")
    out = {}

    t_start = time.perf_counter()

    only = [p for p in os.environ.get("XUCG_COLLECTIVE_PHASES", "").split(",") if p]
    limit = float(os.environ.get("XUCG_COLLECTIVE_LIMIT_S", "280"))
    out["phase_wall_s"] = {}

    def agreed(fn, name):
        # XUCG_COLLECTIVE_PHASES=name,...: run only those (a debugging aid)
        if only and name not in only:
            out[name] = {"skipped": "not in XUCG_COLLECTIVE_PHASES"}
            return
        skip = phase_budget_skip(dist, dev, t_start, limit, name)
        if skip:
            out[name] = skip
            return
        if save:
            save(out, running=name)
        t0 = time.perf_counter()
        agreed_phase(out, name, fn, dist, dev, rank, t_start)
        out["phase_wall_s"][name] = round(time.perf_counter() - t0, 1)
        if save:
            save(out, running=None)

    def timed(fn, iters):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item() / iters

    # With torch's memory from the shim's shareable allocator (the default,
    # collective_child) a key names the physical allocation, and a tensor may
    # be freed once its mappings are released. On the hipIpc fallback a key
    # names (pid, address, size): a tensor freed and allocated again at the
    # same address could hand the peers the old memory (r03h),
    # so there every exported tensor stays allocated until the phases end.
    exported = []

    def keep(*ts):
        if not SHAREABLE_PEER_MEMORY[0]:
            exported.extend(ts)
    n4 = (1 << 30) // COLL_SCALE      # 4 GiB fp32 (config 4)
    shard = n4 // world
    x = torch.empty(n4, dtype=torch.float32, device=dev)
    ctx.fill("float32", "exact", 0x5EED4000 + rank, x, n4)
    ctx.sync()
    rs_out = torch.empty(shard, dtype=torch.float32, device=dev)
    ag_out = torch.empty(n4, dtype=torch.float32, device=dev)
    s_bytes = n4 * 4
    bus = (world - 1) / world * s_bytes

    def rccl():
        if not VENDOR[0]:
            return {"skipped": "full-size rehearsal: the gloo stand-in cannot move 4 GiB "
                               "per rank in time"}
        for _ in range(warmup):
            dist.reduce_scatter_tensor(rs_out, x)
            dist.all_gather_into_tensor(ag_out, rs_out)
        t_rs = timed(lambda: dist.reduce_scatter_tensor(rs_out, x), steps)
        t_ag = timed(lambda: dist.all_gather_into_tensor(ag_out, rs_out), steps)
        return {"bytes": s_bytes, "rs_ms": round(t_rs * 1e3, 3),
                "ag_ms": round(t_ag * 1e3, 3),
                "rs_busbw_gbs": round(bus / t_rs / 1e9, 1),
                "ag_busbw_gbs": round(bus / t_ag / 1e9, 1),
                "rs_frac_of_xgmi": round(bus / t_rs / 1e9 / XGMI_GBS, 4),
                "rs_frac_of_xgmi_per_direction": round(bus / t_rs / 1e9 / XGMI_DIR_GBS, 4)}
    agreed(rccl, "c4_rccl_rs_ag_4gib_fp32")

    def oneshot():
        if world & (world - 1) or world > 16:
            return {"skipped": "one-shot needs a power-of-two group <= 16"}
        keep(x)
        # parity against the reference plan itself: every member's input on
        # sampled windows of every shard, the plan's association evaluated
        # on the host (exact inputs now, rounded ones below)
        plan = PlanWindows(dist, x, n4, rank, world, dev)
        peers = G.PeerBuffers(ctx, x.data_ptr(), rank, world, dist)
        mine = torch.empty(shard, dtype=torch.float32, device=dev)
        keep(mine)
        res = {"bytes": s_bytes,
               "association": "recursive doubling (builtin_recursive.c:158-169)",
               "parity": "host evaluation of the plan on 18 sampled windows of every shard"
                         + ("" if VENDOR[0] else "; the vendor (RCCL stand-in) legs skipped: "
                            "the gloo stand-in cannot move 4 GiB per rank in time")}
        try:
            def rs():
                G.oneshot_reduce_scatter(ctx, peers, mine.data_ptr(), n4, "float32",
                                         "sum", rank, world)
                torch.cuda.synchronize()  # readers done before anyone proceeds
                dist.barrier()
            for _ in range(warmup):
                rs()
            t_rs = timed(rs, steps)
            res.update({"rs_ms": round(t_rs * 1e3, 3),
                        "rs_busbw_gbs": round(bus / t_rs / 1e9, 1),
                        "rs_frac_of_xgmi": round(bus / t_rs / 1e9 / XGMI_GBS, 4),
                        "rs_frac_of_xgmi_per_direction":
                            round(bus / t_rs / 1e9 / XGMI_DIR_GBS, 4),
                        "oneshot_rs_bit_exact_vs_host_plan_sampled_exact": plan.rs_ok(mine)})
            # the same reduce-scatter with the multi-operand kernel uncapped
            # ("Occupancy cap": tuned on local HBM; here 7 of 8
            # operands come over xGMI), then capped again
            from xucg_amd import _lib as L
            L.dev().ucg_builtin_dev_set_multi_cap(0)
            try:
                rs()
                t_rs_uncapped = timed(rs, steps)
            finally:
                L.dev().ucg_builtin_dev_set_multi_cap(-1)
            res.update({"oneshot_rs_uncapped_ms": round(t_rs_uncapped * 1e3, 3),
                        "oneshot_rs_uncapped_busbw_gbs": round(bus / t_rs_uncapped / 1e9, 1)})
            ag_rccl = None
            if VENDOR[0]:
                dist.reduce_scatter_tensor(rs_out, x)
                torch.cuda.synchronize()
                res["bit_exact_vs_rccl_on_exact_inputs"] = bool(
                    torch.equal(mine.view(torch.int32), rs_out.view(torch.int32)))
                # north_star's 8-GPU target is stated on the 1 GiB buffer of
                # the single-GPU target: the first 1 GiB of x, same peers
                n1 = (1 << 28) // COLL_SCALE
                lo1, hi1 = G.shard_bounds(n1, 4, world, rank)
                mine1 = torch.empty(hi1 - lo1, dtype=torch.float32, device=dev)
                rccl1 = torch.empty(n1 // world, dtype=torch.float32, device=dev)
                x1 = x.narrow(0, 0, n1)

                def rs1():
                    G.oneshot_reduce_scatter(ctx, peers, mine1.data_ptr(), n1, "float32", "sum",
                                             rank, world)
                    torch.cuda.synchronize()
                    dist.barrier()
                for _ in range(warmup):
                    rs1()
                    dist.reduce_scatter_tensor(rccl1, x1)
                t_rs1 = timed(rs1, steps)
                t_rccl1 = timed(lambda: dist.reduce_scatter_tensor(rccl1, x1), steps)
                same1 = bool(torch.equal(mine1.view(torch.int32), rccl1.view(torch.int32)))
                bus1 = (world - 1) / world * n1 * 4
                res["rs_1gib"] = {
                    "bytes": n1 * 4, "oneshot_rs_ms": round(t_rs1 * 1e3, 3),
                    "oneshot_rs_busbw_gbs": round(bus1 / t_rs1 / 1e9, 1),
                    "oneshot_rs_frac_of_xgmi": round(bus1 / t_rs1 / 1e9 / XGMI_GBS, 4),
                    "oneshot_rs_frac_of_xgmi_per_direction":
                        round(bus1 / t_rs1 / 1e9 / XGMI_DIR_GBS, 4),
                    "rccl_rs_ms": round(t_rccl1 * 1e3, 3),
                    "rccl_rs_busbw_gbs": round(bus1 / t_rccl1 / 1e9, 1),
                    "oneshot_bit_exact_vs_rccl_on_exact_inputs": same1}
                del mine1, rccl1, x1
                t_ag = timed(lambda: dist.all_gather_into_tensor(ag_out, mine), steps)
                res["rs_ag_ms"] = round((t_rs + t_ag) * 1e3, 3)
                ag_rccl = ag_out.clone()
            # one-shot all-gather: every rank reads the N reduced shards in
            # place over xGMI (ucg_builtin_dev_gather_multi); parity: the
            # plan's result on every shard (and bit-exact with RCCL's
            # all-gather of the same shards)
            keep(ag_out)
            speers = G.PeerBuffers(ctx, mine.data_ptr(), rank, world, dist)
            try:
                def ag1():
                    G.oneshot_all_gather(ctx, speers, ag_out.data_ptr(), n4, "float32",
                                         world)
                    torch.cuda.synchronize()
                    dist.barrier()
                for _ in range(warmup):
                    ag1()
                t_ag1 = timed(ag1, steps)
                res.update({"oneshot_ag_ms": round(t_ag1 * 1e3, 3),
                            "oneshot_ag_busbw_gbs": round(bus / t_ag1 / 1e9, 1),
                            "oneshot_rs_ag_ms": round((t_rs + t_ag1) * 1e3, 3),
                            "oneshot_ag_bit_exact_vs_host_plan_sampled": plan.full_ok(ag_out)})
                if ag_rccl is not None:
                    res["oneshot_ag_bit_exact_vs_rccl"] = bool(
                        torch.equal(ag_out.view(torch.int32), ag_rccl.view(torch.int32)))
            finally:
                torch.cuda.synchronize()
                dist.barrier()
                speers.close()
            # the whole RS + AG as one operation (group.oneshot_allreduce):
            # both halves one-shot over xGMI, ordered by stream barriers (a
            # one-element RCCL all_reduce) instead of host syncs
            sbar = G.stream_barrier(dist, dev)
            rpeers = G.PeerBuffers(ctx, ag_out.data_ptr(), rank, world, dist)
            # push forms (every transfer a write into a peer's buffer): the
            # shards go into the owners' stages, combined there; the reduced
            # shard is written into every peer's recv buffer
            slot = G.stage_slot_bytes(n4, 4, world)
            stage = torch.empty(world * slot // 4, dtype=torch.float32, device=dev)
            keep(stage)
            tpeers = G.PeerBuffers(ctx, stage.data_ptr(), rank, world, dist)
            try:
                def ar1():
                    G.oneshot_allreduce(ctx, peers, rpeers, n4, "float32", "sum", rank,
                                        world, sbar)
                ag_out.zero_()
                for _ in range(warmup):
                    ar1()
                t_ar1 = timed(ar1, steps)
                res.update({"oneshot_allreduce_ms": round(t_ar1 * 1e3, 3),
                            "oneshot_allreduce_busbw_gbs": round(2 * bus / t_ar1 / 1e9, 1),
                            "oneshot_allreduce_frac_of_xgmi":
                                round(2 * bus / t_ar1 / 1e9 / XGMI_GBS, 4),
                            "oneshot_allreduce_frac_of_xgmi_per_direction":
                                round(2 * bus / t_ar1 / 1e9 / XGMI_DIR_GBS, 4),
                            "oneshot_allreduce_bit_exact_vs_host_plan_sampled":
                                plan.full_ok(ag_out)})
                if ag_rccl is not None:
                    res["oneshot_allreduce_bit_exact_vs_rccl_rs_ag"] = bool(
                        torch.equal(ag_out.view(torch.int32), ag_rccl.view(torch.int32)))

                def prs():
                    G.push_reduce_scatter(ctx, x.data_ptr(), tpeers, mine.data_ptr(), n4,
                                          "float32", "sum", rank, world, sbar)
                    sbar()
                mine.zero_()
                for _ in range(warmup):
                    prs()
                t_prs = timed(prs, steps)
                res.update({"push_rs_ms": round(t_prs * 1e3, 3),
                            "push_rs_busbw_gbs": round(bus / t_prs / 1e9, 1),
                            "push_rs_frac_of_xgmi": round(bus / t_prs / 1e9 / XGMI_GBS, 4),
                            "push_rs_frac_of_xgmi_per_direction":
                                round(bus / t_prs / 1e9 / XGMI_DIR_GBS, 4),
                            "push_rs_bit_exact_vs_host_plan_sampled": plan.rs_ok(mine)})
                if VENDOR[0]:
                    res["push_rs_bit_exact_vs_rccl"] = bool(
                        torch.equal(mine.view(torch.int32), rs_out.view(torch.int32)))

                def par():
                    G.push_allreduce(ctx, x.data_ptr(), tpeers, rpeers, n4, "float32", "sum",
                                     rank, world, sbar)
                ag_out.zero_()
                for _ in range(warmup):
                    par()
                t_par = timed(par, steps)
                res.update({"push_allreduce_ms": round(t_par * 1e3, 3),
                            "push_allreduce_busbw_gbs": round(2 * bus / t_par / 1e9, 1),
                            "push_allreduce_bit_exact_vs_host_plan_sampled":
                                plan.full_ok(ag_out)})
                if ag_rccl is not None:
                    res["push_allreduce_bit_exact_vs_rccl_rs_ag"] = bool(
                        torch.equal(ag_out.view(torch.int32), ag_rccl.view(torch.int32)))
            finally:
                torch.cuda.synchronize()
                dist.barrier()
                rpeers.close()
                tpeers.close()
            del ag_rccl, stage
            # rounded inputs: the pull RS bit for bit against the plan on
            # sampled windows; RCCL's ring order against the SURVEY.md 8c
            # bound |delta| <= 2 (n-1) u sum_i |x_i|, u = 2^-24
            torch.cuda.synchronize()
            dist.barrier()
            ctx.fill("float32", "round", 0x5EED4100 + rank, x, n4)
            torch.cuda.synchronize()
            dist.barrier()
            rs()
            plan_r = PlanWindows(dist, x, n4, rank, world, dev)
            res["oneshot_rs_bit_exact_vs_host_plan_sampled_rounded"] = plan_r.rs_ok(mine)
            if VENDOR[0]:
                dist.reduce_scatter_tensor(rs_out, x)
                absx = x.abs()
                abs_rs = torch.empty_like(rs_out)
                dist.reduce_scatter_tensor(abs_rs, absx)
                del absx
                tol = 2 * (world - 1) * 2.0 ** -24 * abs_rs
                err = (mine - rs_out).abs()
                res["rccl_within_8c_tolerance_on_rounded_inputs"] = bool((err <= tol).all())
                res["max_err_over_tolerance"] = round(
                    float((err / tol.clamp_min(1e-30)).max()), 4)
                res["max_ulps_vs_rccl_on_rounded_inputs"] = max_ulps(mine, rs_out)
                del abs_rs, tol, err
        finally:
            torch.cuda.synchronize()
            dist.barrier()
            peers.close()
        return res
    agreed(oneshot, "c4_oneshot_xgmi_rs_4gib_fp32")
    del x, rs_out, ag_out
    torch.cuda.empty_cache()

    def recursive_doubling():
        if world & (world - 1):
            return {"skipped": "recursive doubling / halving need a power-of-two group"}
        n5 = (1 << 26) // COLL_SCALE  # 512 MiB fp64 per rank (config 5)
        init = torch.empty(n5, dtype=torch.float64, device=dev)
        ctx.fill("float64", "round", 0x5EED5000 + rank, init, n5)
        acc = torch.empty_like(init)
        tmp = torch.empty_like(init)
        exchange = G.torch_exchange(dist)

        def combine(a, t):
            ctx.reduce_checked("sum", "float64", a, t, n5)

        def combine_n(a, t, n):
            ctx.reduce_checked("sum", "float64", a, t, n)

        def once():
            acc.copy_(init)           # ucg_builtin_init_reduce: recv <- send
            G.recursive_doubling_allreduce(acc, tmp, rank, world, combine, exchange)

        def once_halving():
            acc.copy_(init)
            G.recursive_halving_allreduce(acc, tmp, rank, world, combine_n, exchange,
                                          n5, 8)

        sbar = G.stream_barrier(dist, dev)
        keep(init, acc)
        ipeers = G.PeerBuffers(ctx, init.data_ptr(), rank, world, dist)
        apeers = G.PeerBuffers(ctx, acc.data_ptr(), rank, world, dist)

        slot5 = G.stage_slot_bytes(n5, 8, world)
        stage5 = torch.empty(world * slot5 // 8, dtype=torch.float64, device=dev)
        keep(stage5)
        tpeers = G.PeerBuffers(ctx, stage5.data_ptr(), rank, world, dist)

        def once_oneshot():
            # reads every member's send buffer in place: no init_reduce copy
            G.oneshot_allreduce(ctx, ipeers, apeers, n5, "float64", "sum", rank, world,
                                sbar)

        def once_push():
            G.push_allreduce(ctx, init.data_ptr(), tpeers, apeers, n5, "float64", "sum",
                             rank, world, sbar)


        # parity: the plan's association evaluated on the host over sampled
        # windows of every member's input (head, tail, 16 random 64 KiB)
        check, idx, want_w, xs_w = sampled_plan_check(dist, init, rank, world)

        def head_ok(pb, xs, want):
            """per member: does its buffer's head window, read through the
            peer mapping by DMA / by a kernel, hold its input (xs) or the
            plan's result (want)? "ok/ok", "ok/BAD", ..."""
            import numpy as np
            from xucg_amd import _lib
            torch.cuda.synchronize()
            out = []
            loc = torch.empty(SAMPLE_ELEMS, dtype=torch.float64, device=dev)
            for p, ptr in enumerate(pb.ptrs):
                ref = (xs[p][:SAMPLE_ELEMS] if xs is not None else want[:SAMPLE_ELEMS]
                       ).view(np.int64)
                h = np.empty(SAMPLE_ELEMS, np.float64)       # by DMA
                _lib.check(_lib.dev().ucg_builtin_dev_memcpy(
                    ctx.handle, h.ctypes.data, ptr, SAMPLE_ELEMS * 8), "memcpy")
                _lib.check(ctx.copy_multi([loc.data_ptr()], [ptr], SAMPLE_ELEMS * 8),
                           "copy_multi")                      # by a kernel
                torch.cuda.synchronize()
                k = loc.cpu().numpy()
                v = ("ok" if np.array_equal(h.view(np.int64), ref) else "BAD") + "/" + \
                    ("ok" if np.array_equal(k.view(np.int64), ref) else "BAD")
                if "BAD" in v and xs is not None:
                    # whose data the mapping shows, and the key it came from
                    whose = [q for q in range(len(xs)) if np.array_equal(
                        h.view(np.int64), xs[q][:SAMPLE_ELEMS].view(np.int64))]
                    b = pb.blobs[p] or b""
                    v += (f" shows {whose or ('zeros' if not h.any() else '?')}"
                          f" key {b[:64].hex()} off {int.from_bytes(b[64:72], 'little')}"
                          f" size {int.from_bytes(b[72:80], 'little')} at 0x{ptr:x}")
                out.append(v)
            return out
        res = {"bytes_per_rank": n5 * 8, "steps": G.recursive_steps(world),
               "parity": "host evaluation of the plan's association on 18 sampled "
                         "64 KiB windows of every member's input"}
        for name, fn, link_bytes in (
                ("doubling", once, n5 * 8 * G.recursive_steps(world)),
                ("halving", once_halving, 2 * (world - 1) * n5 * 8 // world),
                ("oneshot_xgmi", once_oneshot, 2 * (world - 1) * n5 * 8 // world),
                ("oneshot_xgmi_push", once_push, 2 * (world - 1) * n5 * 8 // world)):
            acc.zero_()
            fn()
            torch.cuda.synchronize()
            same = check(acc)
            for _ in range(warmup):
                fn()
            t = timed(fn, steps)
            res[name] = {"ms": round(t * 1e3, 3),
                         "algbw_gbs": round(n5 * 8 / t / 1e9, 1),
                         "sent_bytes_per_rank": link_bytes,
                         "link_gbs": round(link_bytes / t / 1e9, 1),
                         "bit_exact_vs_host_plan_sampled": same}
            if not same:
                res[name]["mismatch"] = mm = dict(check.last)
                # where it went wrong: the head window of every member's
                # input and of every member's result, read through the maps
                # (local reads only, after the form's last collective)
                try:
                    mm["inputs_via_map_ok"] = head_ok(ipeers, xs_w, None)
                    mm["results_via_map_ok"] = head_ok(apeers, None, want_w)
                except Exception as e:  # noqa: BLE001 - a diagnostic only
                    mm["diagnostic_error"] = f"{type(e).__name__}: {e}"[:200]
        torch.cuda.synchronize()
        dist.barrier()
        ipeers.close()
        apeers.close()
        tpeers.close()
        del stage5
        # vendor baseline on the same buffer (ring association: tolerance only)
        acc.copy_(init)
        dist.all_reduce(acc)
        torch.cuda.synchronize()
        # |delta| <= 2 (n-1) u sum_i |x_i|, u = 2^-53, on the
        # sampled windows against the host evaluation of the plan
        import numpy as np
        got_w = acc[idx].cpu().numpy()
        tol = 2 * (world - 1) * 2.0 ** -53 * np.abs(xs_w).sum(axis=0)
        err = np.abs(got_w - want_w)
        res["rccl_allreduce_within_8c_tolerance_of_plan"] = bool((err <= tol).all())
        res["rccl_allreduce_max_abs_err_over_tol"] = float((err / np.maximum(tol, 1e-300)).max())
        res["rccl_allreduce_max_ulps"] = max_ulps(torch.from_numpy(got_w),
                                                  torch.from_numpy(want_w))
        del tol, err
        t = timed(lambda: dist.all_reduce(acc), steps)
        res["rccl_allreduce"] = {"ms": round(t * 1e3, 3),
                                 "algbw_gbs": round(n5 * 8 / t / 1e9, 1)}
        return res
    agreed(recursive_doubling, "c5_recursive_allreduce_512mib_fp64")

    def engine_c5():
        """(e) C5 through the builtin plan itself: the operation engine
        (libucg_builtin.so) on device buffers - remote-key steps, the partner's
        buffer read over xGMI by the fold kernel. Its own phase, so a failure
        here costs this entry only."""
        if world & (world - 1):
            return {"skipped": "the recursive plan needs a power-of-two group"}
        n5 = (1 << 26) // COLL_SCALE
        init = torch.empty(n5, dtype=torch.float64, device=dev)
        ctx.fill("float64", "round", 0x5EED5000 + rank, init, n5)
        acc = torch.zeros_like(init)
        check = sampled_plan_check(dist, init, rank, world)[0]

        def measure():
            acc.zero_()
            eng = builtin_engine(rank, world, local_rank, init.data_ptr(), acc.data_ptr(),
                                 n5, ctx=ctx)
            try:
                eng.run()
                torch.cuda.synchronize()
                same = check(acc)
                for _ in range(warmup):
                    eng.run()
                t = timed(eng.run, steps)
                text = eng.describe()
                executed = [ln for ln in text.splitlines() if ln.startswith("Executed as")]
                link = n5 * 8 * G.recursive_steps(world)
                return {"plan": text.splitlines()[0],
                        "executed_as": executed[0] if executed else "the plan's steps",
                        "ms": round(t * 1e3, 3), "algbw_gbs": round(n5 * 8 / t / 1e9, 1),
                        "sent_bytes_per_rank": link, "link_gbs": round(link / t / 1e9, 1),
                        "bit_exact_vs_host_plan_sampled": same,
                        **({} if same else {"mismatch": check.last})}
            finally:
                torch.cuda.synchronize()
                dist.barrier()
                eng.close()
                dist.barrier()      # every rank closed before the name is reused
        # the default (fp64 SUM: the two-phase one-shot over all links from 4
        # GPUs on), and UCX_BUILTIN_ONESHOT_FLOAT_SPLIT=n: every member's own
        # association, i.e. the plan's recursive-doubling steps (same bits here:
        # no NaN in these inputs)
        res = measure()
        if 4 <= world <= 16:
            os.environ["UCX_BUILTIN_ONESHOT_FLOAT_SPLIT"] = "n"
            try:
                res["steps"] = measure()
            finally:
                del os.environ["UCX_BUILTIN_ONESHOT_FLOAT_SPLIT"]
        return res
    agreed(engine_c5, "c5_builtin_engine_device_buffers_512mib_fp64")
    out["wall_s"] = round(time.perf_counter() - t_start, 1)
    torch.cuda.synchronize()
    dist.barrier()          # no peer maps any of them any more
    del exported
    return out


class builtin_engine:
    """An fp64 SUM allreduce through the builtin operation engine on device
    buffers (include/ucg_builtin_ops.h): the shared-memory AM transport
    between the node's ranks for keys, READY and DONE, the data read over
    xGMI by the combine kernels. The "MPI library" behind reduce_cb_f knows
    one op (SUM) and one type (double): handles are the device enums + 1."""

    def __init__(self, rank, world, local_rank, sbuf, rbuf, count, ctx=None):
        import ctypes
        import numpy as np
        from xucg_amd import host, ops, OPS, DTYPES
        sum_h, f64_h = OPS.index("sum") + 1, DTYPES.index("float64") + 1

        def reduce_cb(op, src, dst, n, dtype):     # host buffers only
            s = np.ctypeslib.as_array((ctypes.c_double * n).from_address(src))
            d = np.ctypeslib.as_array((ctypes.c_double * n).from_address(dst))
            d[:] = s + d
            return 0
        cbs = {"reduce_cb_f": reduce_cb, "is_sum_f": lambda op: op == sum_h,
               "is_loc_expected_f": lambda op: False, "is_commutative_f": lambda op: True,
               "convert": lambda dt: 8 << 3, "is_integer_f": lambda dt: (False, False),
               "is_floating_point_f": lambda dt: True}
        self.cmb = host.BuiltinCombine(cbs, host.make_config(device=local_rank),
                                       op_classifier=lambda op: op - 1,
                                       dt_classifier=lambda dt: dt - 1)
        self.iface = ops.ShmIface(f"/xucg_bench_{os.environ.get('MASTER_PORT', '0')}",
                                  world, rank, max_short=256)
        self.group = ops.Group(self.iface, 7, world, rank, self.cmb)
        # the send buffer in the group's registered memory, exposed in place
        # (ucg_builtin_lgroup_mem_alloc): no init copy inside the timed op
        self.reg = None
        if ctx is not None:
            self.reg = self.group.mem_alloc(count * 8, device=True)
            rc = ctx.copy_multi([self.reg], [sbuf], count * 8)
            ctx.sync()
            if rc != 0:
                raise RuntimeError("copy into registered memory failed")
            sbuf = self.reg
        self.coll = self.group.allreduce(sbuf, rbuf, count, f64_h, sum_h)
        if self.coll.status != 0:
            raise RuntimeError(f"builtin allreduce create failed: {self.coll.status}")

    def run(self):
        st = self.coll.run()
        if st != 0:
            raise RuntimeError(f"builtin allreduce failed: {st}")

    def describe(self):
        return self.coll.describe()

    def close(self):
        self.coll.close()
        if self.reg:
            self.group.mem_free(self.reg)
        self.group.close()
        self.iface.close()
        self.cmb.close()


def same_box_reference(n, iters=50):
    """Vendor kernels on the same box, same buffers, same bytes: PyTorch's
    in-place add (dst += src, 3N bytes) and a device-to-device copy (2N
    bytes), timed with events on torch's stream. HBM throughput differs by a
    few per cent from box to box; these put the combine's number in context."""
    import torch
    ab = torch.rand(2 * n, device="cuda")      # one allocation, as the headline pair
    a, b = ab[:n], ab[n:]

    def time_us(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / iters
    add_us = time_us(lambda: b.add_(a))
    copy_us = time_us(lambda: b.copy_(a))
    del a, b, ab
    torch.cuda.empty_cache()
    return {"torch_add_inplace_us": round(add_us, 3),
            "torch_add_inplace_gbs": round(3 * n * 4 / (add_us * 1e-6) / 1e9, 1),
            "d2d_copy_us": round(copy_us, 3),
            "d2d_copy_gbs": round(2 * n * 4 / (copy_us * 1e-6) / 1e9, 1)}


def one_shot_shape(ctx, nsrc=8, per_op=64 << 20, iters=100):
    """The C4/C5 one-shot reduce-scatter's kernel on one GPU: 8 local operands
    of 64 MiB (ucg_builtin_dev_reduce_multi, the recursive-doubling
    association, occupancy-capped), operands and output in one
    allocation. (N + 1) x S algorithmic bytes per launch; wall clock over
    back-to-back launches after a warm-up (enough of them, about 10 ms, that
    the first launch's latency and the final sync's stay below 1 %), then a
    sampled exactness check ("exact" inputs: every association gives the
    same bits)."""
    import numpy as np
    n = per_op // 4
    arena = ctx.alloc((nsrc + 1) * per_op)
    srcs = [arena.ptr + m * per_op for m in range(nsrc)]
    dst = arena.ptr + nsrc * per_op
    for m, p in enumerate(srcs):
        ctx.fill("float32", "exact", 300 + m, p, n)
    for _ in range(3):
        assert ctx.reduce_multi("sum", "float32", dst, srcs, 0, n) == 0
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        ctx.reduce_multi("sum", "float32", dst, srcs, 0, n)
    ctx.sync()
    wall_us = (time.perf_counter() - t0) / iters * 1e6
    # the kernel's own time: HIP events on the context stream around the
    # same back-to-back launches (the roofline's method), median of 3
    ev = sorted(ctx.profile_reduce_multi("sum", "float32", dst, srcs, 0, n, iters)
                for _ in range(3))
    us = ev[1]
    w = 1 << 16
    lo = (n // 2) & ~15
    want = sum(arena.download(np.float32, w, m * per_op + lo * 4).astype(np.float64)
               for m in range(nsrc))
    got = arena.download(np.float32, w, nsrc * per_op + lo * 4)
    ok = bool(np.array_equal(got.astype(np.float64), want))
    arena.free()
    gbs = (nsrc + 1) * per_op / (us * 1e-6) / 1e9
    return {"operands": nsrc, "bytes_per_operand": per_op, "us": round(us, 2),
            "achieved_gbs": round(gbs, 1), "frac_of_8tbs": round(gbs / HBM_PEAK_GBS, 4),
            "sampled_exact": ok, "wall_us": round(wall_us, 2),
            "frac_of_8tbs_wall": round((nsrc + 1) * per_op / (wall_us * 1e-6) / 1e9 /
                                       HBM_PEAK_GBS, 4),
            "note": "k_reduce_multi, operands + output in one allocation; us: HIP events "
                    f"around {iters} back-to-back launches (median of 3 batches), wall_us: "
                    "the host's clock around the same launches made from Python"}


def collective_alloc_plan(world=8):
    """One rank's device allocations in collective_phases, phase by phase, in
    order: (phase, "alloc"|"free", name, bytes). Mirrors the
    code above at full size (COLL_SCALE 1) on the default hipIpc path, where
    every exported tensor stays allocated until the phases end (keep()).
    RCCL's own buffers and the engine's pinned host ring are not in it."""
    from xucg_amd import group as G
    n4 = 1 << 30                               # C4: 4 GiB fp32
    shard = n4 // world
    lo1, hi1 = G.shard_bounds(1 << 28, 4, world, 0)
    n5 = 1 << 26                               # C5: 512 MiB fp64
    slot = G.stage_slot_bytes(n4, 4, world)
    slot5 = G.stage_slot_bytes(n5, 8, world)
    win = 18 * SAMPLE_ELEMS                    # sampled windows per shard (PlanWindows)
    return [
        ("c4", "alloc", "x (send)", n4 * 4),
        ("c4", "alloc", "rs_out (RCCL reduce-scatter output)", shard * 4),
        ("c4", "alloc", "ag_out (RCCL all-gather output, one-shot recv)", n4 * 4),
        ("c4 one-shot", "alloc", "PlanWindows index + gathered windows", 2 * world * win * 8),
        ("c4 one-shot", "alloc", "mine (one-shot shard)", shard * 4),
        ("c4 one-shot", "alloc", "mine1 (1 GiB leg shard)", (hi1 - lo1) * 4),
        ("c4 one-shot", "alloc", "rccl1 (1 GiB leg RCCL shard)", (1 << 28) // world * 4),
        ("c4 one-shot", "free", "mine1 (1 GiB leg shard)", (hi1 - lo1) * 4),
        ("c4 one-shot", "free", "rccl1 (1 GiB leg RCCL shard)", (1 << 28) // world * 4),
        ("c4 one-shot", "alloc", "ag_rccl (RCCL all-gather copy)", n4 * 4),
        ("c4 push", "alloc", "stage (push reduce-scatter)", world * slot),
        ("c4 push", "free", "ag_rccl (RCCL all-gather copy)", n4 * 4),
        ("c4 rounded", "alloc", "|x| (tolerance input)", n4 * 4),
        ("c4 rounded", "alloc", "|x| reduce-scatter", shard * 4),
        ("c4 rounded", "free", "|x| (tolerance input)", n4 * 4),
        ("c4 rounded", "alloc", "tolerance", shard * 4),
        ("c4 rounded", "alloc", "error", shard * 4),
        ("c4 rounded", "free", "|x| reduce-scatter", shard * 4),
        ("c4 rounded", "free", "tolerance", shard * 4),
        ("c4 rounded", "free", "error", shard * 4),
        ("c4 end", "free", "rs_out (RCCL reduce-scatter output)", shard * 4),
        # x, mine, ag_out and stage stay: exported (keep) until the phases end
        ("c5", "alloc", "init (send)", n5 * 8),
        ("c5", "alloc", "acc (recv)", n5 * 8),
        ("c5", "alloc", "tmp (exchange)", n5 * 8),
        ("c5", "alloc", "stage5 (push allreduce)", world * slot5),
        ("c5 end", "free", "tmp (exchange)", n5 * 8),
        # init, acc and stage5 stay: exported (keep)
        ("c5 engine", "alloc", "init (engine send)", n5 * 8),
        ("c5 engine", "alloc", "acc (engine recv)", n5 * 8),
        ("c5 engine", "alloc", "group arena (UCX_BUILTIN_DEV_ARENA_BYTES)", 32 << 20),
        ("c5 engine", "alloc", "registered send buffer (lgroup_mem_alloc)", n5 * 8),
        ("c5 engine", "alloc", "op buffer 0 (remote-key steps)", n5 * 8),
        ("c5 engine", "alloc", "op buffer 1 (remote-key steps)", n5 * 8),
    ]


def collective_dry_alloc(world=8):
    """--collective-dry-alloc: one rank's C4 and C5 buffers at full size, in
    the order collective_plan lists them, on this process's one GPU - torch
    tensors from torch's caching allocator as in the collective child, the
    engine's from the shim (ucg_builtin_dev_malloc) - and the device memory in
    use after every step (hipMemGetInfo). No collective runs. Prints one JSON
    line with the peak."""
    import torch
    import xucg_amd
    torch.cuda.set_device(0)
    ctx = xucg_amd.DevContext(device=0)
    free0, total = torch.cuda.mem_get_info()
    live, steps, peak = {}, [], 0
    for phase, act, name, nbytes in collective_alloc_plan(world):
        key = (phase.split()[0], name)
        if act == "alloc":
            if phase == "c5 engine":
                live[key] = ctx.alloc(nbytes)
            else:
                live[key] = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
                live[key].fill_(1)                      # touched, as the phases do
        else:
            k = next(k for k in live if k[1] == name)
            b = live.pop(k)
            if hasattr(b, "free"):
                b.free()
            del b
        torch.cuda.synchronize()
        used = free0 - torch.cuda.mem_get_info()[0]
        peak = max(peak, used)
        steps.append({"phase": phase, act: name, "bytes": nbytes,
                      "device_used_gib": round(used / GIB, 3)})
    res = {"collective_dry_alloc": True, "world": world, "rank_modelled": 0,
           "device_total_gib": round(total / GIB, 1),
           "peak_device_used_gib": round(peak / GIB, 3),
           "planned_peak_gib": round(plan_peak(collective_alloc_plan(world)) / GIB, 3),
           "torch_max_reserved_gib": round(torch.cuda.max_memory_reserved() / GIB, 3),
           "steps": steps,
           "not_included": "RCCL's own buffers; the engine's pinned host staging ring"}
    for b in live.values():
        if hasattr(b, "free"):
            b.free()
    live.clear()
    ctx.close()
    print(json.dumps(res), flush=True)


def plan_peak(plan):
    """the largest sum of live bytes over the plan's steps"""
    cur = peak = 0
    for _, act, _, nbytes in plan:
        cur += nbytes if act == "alloc" else -nbytes
        peak = max(peak, cur)
    return peak


def run_collective_children(dist, rank, world, timeout_s=300):
    """Run collective_phases in one child process per rank (a fresh process
    group on a new port), so that a fault in the multi-GPU phases - the IPC
    peer mappings cannot be exercised on the 1-GPU boxes this build is tested
    on - costs the collective numbers only, never the bench line. Children
    are started with subprocess (fork + exec in the child), never by
    replacing this process. Returns rank 0's result dict (or an error)."""
    import subprocess
    import tempfile
    import uuid
    import torch
    obj = [None]
    if rank == 0:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        obj[0] = {"port": port,
                  "out": os.path.join(tempfile.gettempdir(),
                                      f"xucg_collective_{os.getpid()}_{uuid.uuid4().hex}.json")}
    dist.broadcast_object_list(obj, src=0)
    torch.cuda.synchronize()
    dist.barrier()
    # a fresh rendezvous: without torchrun's agent store (TORCHELASTIC_*
    # would make the child wait for the agent's store on the new port)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(obj[0]["port"]),
               XUCG_COLLECTIVE_OUT=obj[0]["out"])
    try:
        # stderr passes through (progress lines), stdout is kept for the error tail
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--collective-child"],
                           env=env, stdout=subprocess.PIPE, text=True, timeout=timeout_s)
        rc, tail = p.returncode, p.stdout[-600:]
    except subprocess.TimeoutExpired as e:
        rc, tail = "timeout", str(e)[-300:]
    if rank != 0:
        return None, rc == 0
    return read_child_result(obj[0]["out"], rc, tail), rc == 0


class HostStagedDist:
    """Rehearsal only (XUCG_COLLECTIVE_BACKEND=gloo): the torch.distributed
    calls of collective_phases over gloo, with CUDA tensors staged through
    host memory. RCCL refuses two ranks on one GPU, so this is how the
    multi-rank glue of the phases (IPC key exchange, peer mappings, the
    one-shot and push forms, the engine over several processes, phase
    agreement and every parity check) runs on a 1-GPU box with 2-4 ranks.
    Each call synchronises the device, so the rehearsal's timings mean
    nothing; the result carries a "rehearsal" entry saying so."""

    def __init__(self, dist):
        self._d = dist
        self.ReduceOp = dist.ReduceOp

    @staticmethod
    def _sync():
        import torch
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def get_rank(self):
        return self._d.get_rank()

    def get_world_size(self):
        return self._d.get_world_size()

    def barrier(self, group=None):
        self._sync()
        self._d.barrier(group=group)

    def all_reduce(self, t, op=None, group=None):
        op = self._d.ReduceOp.SUM if op is None else op
        c = t.cpu()
        self._d.all_reduce(c, op=op, group=group)
        t.copy_(c)

    def all_gather(self, outs, t, group=None):
        cs = [torch_empty_cpu_like(t) for _ in outs]
        self._d.all_gather(cs, t.cpu(), group=group)
        for o, c in zip(outs, cs):
            o.copy_(c)

    def all_gather_object(self, outs, obj, group=None):
        self._d.all_gather_object(outs, obj, group=group)

    def broadcast_object_list(self, objs, src=0, group=None):
        self._d.broadcast_object_list(objs, src=src, group=group)

    def reduce_scatter_tensor(self, out, inp, op=None, group=None):
        c = inp.cpu()
        self._d.all_reduce(c, op=self._d.ReduceOp.SUM if op is None else op, group=group)
        r, w = self._d.get_rank(group), self._d.get_world_size(group)
        out.copy_(c.view(w, -1)[r])

    def all_gather_into_tensor(self, out, inp, group=None):
        import torch
        w = self._d.get_world_size(group)
        cs = [torch_empty_cpu_like(inp) for _ in range(w)]
        self._d.all_gather(cs, inp.cpu(), group=group)
        out.copy_(torch.cat(cs))

    # point to point: group.torch_exchange's P2POp / batch_isend_irecv
    def isend(self, *a, **k):
        raise RuntimeError("HostStagedDist: isend only through batch_isend_irecv")

    def irecv(self, *a, **k):
        raise RuntimeError("HostStagedDist: irecv only through batch_isend_irecv")

    class P2POp:
        def __init__(self, op, tensor, peer, group=None):
            self.op, self.tensor, self.peer, self.group = op, tensor, peer, group

    def batch_isend_irecv(self, ops):
        stage = []
        for p in ops:
            send = p.op == self.isend
            c = p.tensor.cpu() if send else torch_empty_cpu_like(p.tensor)
            stage.append((p, c, send))
        works = [(self._d.isend if send else self._d.irecv)(c, p.peer, group=p.group)
                 for p, c, send in stage]
        for w in works:
            w.wait()
        for p, c, send in stage:
            if not send:
                p.tensor.copy_(c)

        class _Done:
            def wait(self):
                return True
        return [_Done() for _ in ops]


def torch_empty_cpu_like(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


# whether torch's device memory comes from the shim's shareable allocator in
# this process (collective_child); a one-element list so phases can read it
SHAREABLE_PEER_MEMORY = [False]


def shareable_memory_probe(store, rank, world, local_rank):
    """Before torch allocates anything: can every rank map every other rank's
    shareable allocation (HIP VMM, fd keys from the exporter's key server)
    and read what its owner wrote? The keys and verdicts go through `store`
    (no device tensors). Returns (ok, detail); every rank gets the same ok."""
    import numpy as np
    import xucg_amd
    ctx = xucg_amd.DevContext(device=local_rank)
    buf, maps, err = None, [], ""
    try:
        buf = ctx.alloc(2 << 20, shareable=True)
        buf.upload(np.full(512, rank + 1, np.int64))
        store.set(f"vmm_key_{rank}", ctx.ipc_export(buf.ptr))
        for p in range(world):
            if p == rank:
                continue
            m = ctx.ipc_import(store.get(f"vmm_key_{p}"))
            maps.append(m)
            got = np.empty(512, np.int64)
            from xucg_amd import _lib
            _lib.check(_lib.dev().ucg_builtin_dev_memcpy(ctx.handle, got.ctypes.data, m,
                                                         got.nbytes), "memcpy")
            if not (got == p + 1).all():
                raise RuntimeError(f"member {p}'s buffer read {got[:2].tolist()}")
    except Exception as e:  # noqa: BLE001 - agreed on below
        err = f"{type(e).__name__}: {e}"[:200]
    store.set(f"vmm_ok_{rank}", err or "ok")
    verdicts = [store.get(f"vmm_ok_{p}").decode() for p in range(world)]
    for m in maps:
        ctx.ipc_release(m)
    store.add("vmm_done", 1)
    while store.add("vmm_done", 0) < world:       # nobody frees while mapped
        time.sleep(0.01)
    if buf is not None:
        buf.free()
    ctx.close()
    bad = [f"rank {p}: {v}" for p, v in enumerate(verdicts) if v != "ok"]
    return not bad, ("; ".join(bad) if bad else "every rank mapped every peer's allocation")


def collective_child():
    """--collective-child: one rank of the collective phases (see above).
    XUCG_COLLECTIVE_BACKEND=gloo is the 1-GPU rehearsal (HostStagedDist).
    The phases run on torch's own allocator with hipIpc keys, which the
    shim checks against the allocation's buffer id; exported tensors stay
    allocated until the phases end. XUCG_SHAREABLE_TORCH=y instead takes
    torch's device memory from the shim's shareable allocator when every rank
    can map every other rank's (shareable_memory_probe), so every exported
    tensor is keyed by its physical allocation. It is not the default:
    kernels reading peers' imported shareable allocations ran 5-10x longer
    on one GPU (profiles/r04/r04y)."""
    import datetime
    import torch
    import torch.distributed as dist
    import xucg_amd
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    timeout = datetime.timedelta(seconds=240)
    store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"),
                          int(os.environ["MASTER_PORT"]), world, rank == 0, timeout=timeout)
    peer_memory = {"kind": "hipIpc (torch's caching allocator)"}
    if os.environ.get("XUCG_SHAREABLE_TORCH", "n")[:1] in ("y", "1"):
        ok, detail = shareable_memory_probe(store, rank, world, local_rank)
        if ok:
            xucg_amd.use_shareable_torch_memory()
            SHAREABLE_PEER_MEMORY[0] = True
            peer_memory = {"kind": "shareable (HIP VMM, fd keys; torch memory from the shim)",
                           "probe": detail}
        else:
            peer_memory["probe"] = detail
    if not SHAREABLE_PEER_MEMORY[0]:
        # the engine's registered buffers then take hipIpc keys too
        os.environ["UCX_BUILTIN_DEV_SHAREABLE"] = "n"
    torch.cuda.set_device(local_rank)
    # the engine's waits give up after this long instead of outliving the child
    os.environ.setdefault("UCX_BUILTIN_WAIT_TIMEOUT", "30")
    rehearsal = os.environ.get("XUCG_COLLECTIVE_BACKEND", "nccl") == "gloo"
    pstore = dist.PrefixStore("pg", store)
    if rehearsal:
        dist.init_process_group("gloo", store=pstore, rank=rank, world_size=world,
                                timeout=timeout)
        pg = HostStagedDist(dist)
    else:
        if COLL_SCALE != 1:
            raise SystemExit("XUCG_COLLECTIVE_SCALE is for the gloo rehearsal only")
        dist.init_process_group("nccl", store=pstore, rank=rank, world_size=world,
                                timeout=timeout, device_id=torch.device(f"cuda:{local_rank}"))
        pg = dist
    if rehearsal and COLL_SCALE == 1 and os.environ.get("XUCG_REHEARSAL_VENDOR", "n")[:1] != "y":
        VENDOR[0] = False
    ctx = xucg_amd.DevContext.on_torch_stream(local_rank)

    def save(partial, running=None):
        """rank 0: the phases finished so far, and the one running (read by
        the parent if this child is killed at its time limit)"""
        if rank == 0:
            tmp = os.environ["XUCG_COLLECTIVE_OUT"] + ".part"
            with open(tmp, "w") as f:
                json.dump(dict(partial, running=running), f)
            os.replace(tmp, os.environ["XUCG_COLLECTIVE_OUT"])
    res = collective_phases(ctx, pg, rank, world, local_rank, save=save)
    res["peer_memory"] = peer_memory
    if rehearsal:
        res["rehearsal"] = {"backend": "gloo, CUDA tensors staged through the host",
                            "size_divisor": COLL_SCALE, "vendor_legs": VENDOR[0],
                            "note": "checks the multi-rank glue and parity; timings invalid"}
    if rank == 0:
        with open(os.environ["XUCG_COLLECTIVE_OUT"], "w") as f:
            json.dump(res, f)
    ctx.close()
    dist.destroy_process_group()


def spawn_ranks(n, timeout_s=None):
    """`--gpus N` with no launcher (WORLD_SIZE unset): start one child per GPU
    running this same command line, with RANK / LOCAL_RANK / WORLD_SIZE and a
    fresh 127.0.0.1 rendezvous, as torch.distributed.run would. Called before
    anything touches the GPU in this process (children are started with
    subprocess, never by replacing this process). Rank 0's stdout (the JSON
    line) passes through. When one rank fails the others are given 60 s and
    then killed by their exact PIDs. Returns the exit code: the first
    non-zero child code, else 0."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    base = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [None] * n
    t_fail = None
    t0 = time.monotonic()
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
        bad = [c for c in codes if c not in (None, 0)]
        now = time.monotonic()
        if bad and t_fail is None:
            t_fail = now
        late = (t_fail is not None and now - t_fail > 60) or \
            (timeout_s is not None and now - t0 > timeout_s)
        if late:
            for r, p in enumerate(procs):
                if codes[r] is None:
                    p.send_signal(signal.SIGKILL)
                    codes[r] = p.wait()
        time.sleep(0.05)
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"bench.py --gpus {n}: rank exit codes {codes}", file=sys.stderr, flush=True)
        return bad[0] if bad[0] > 0 else 1
    return 0


def plumbing(world, rank):
    """--plumbing (CPU test of the launch contract, no GPU): the ranks
    rendezvous over gloo, pass the timed region's barrier and max-over-ranks
    reduction, and rank 0 prints the world size the process group saw. No
    combine runs, so the line has no value."""
    import datetime
    import torch
    import torch.distributed as dist
    if world == 1:                      # no launcher: a private rendezvous
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    dist.barrier()
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"plumbing": True, "n_gpus": dist.get_world_size(),
                          "world_size_env": world, "max_over_ranks": t.item(),
                          "value": None}), flush=True)
    dist.destroy_process_group()


def main():
    if "--collective-child" in sys.argv:
        collective_child()
        return
    if "--collective-dry-alloc" in sys.argv:
        collective_dry_alloc(8)
        return
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU: spawned here when no launcher set WORLD_SIZE")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU test of the launch contract only (gloo, no GPU, no value)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--count", type=int, default=WORKLOAD_COUNT)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-collective", action="store_true",
                    help="N > 1: skip the RS+AG / recursive-doubling phases")
    ap.add_argument("--collective-force", action="store_true",
                    help="run the collective phases even at N = 1 (under torchrun)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus}: need at least 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: one rank per GPU, spawned before any GPU call here
        sys.exit(spawn_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: "
                         "the launcher and the flag must agree")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing:
        plumbing(world, rank)
        return

    import torch
    import xucg_amd

    dist = None
    if world > 1 or args.collective_force:
        import datetime
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=600),
                                device_id=torch.device(f"cuda:{local_rank}"))
        # the ranks RCCL itself saw, not the environment's claim
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: RCCL group has {dist.get_world_size()} ranks, "
                             f"WORLD_SIZE={world}")

    def barrier():
        if dist is not None:
            dist.barrier()

    n = args.count
    # multi-GPU: launch on torch's current stream so RCCL and the combine are
    # stream-ordered without host syncs
    ctx = xucg_amd.DevContext.on_torch_stream(local_rank) if dist else \
        xucg_amd.DevContext(device=local_rank)
    # src and dst as the two halves of ONE allocation. Two separately
    # allocated operands can alias in HBM's channel/bank map: on some boxes
    # such pairs combine at 79-83 % where this layout reads 84.5-85 % on every
    # box probed (scripts/place_probe.py "joint", scripts/alias_probe.py;
    # DESIGN.md 5, "Operand aliasing"). A fixed layout, not a measured choice.
    pair = ctx.alloc(2 * n * 4)
    src, dst = pair.ptr, pair.ptr + n * 4
    ctx.fill("float32", "round", 0x5EED0000 + 2 * rank, src, n)
    ctx.fill("float32", "round", 0x5EED0001 + 2 * rank, dst, n)
    ctx.sync()

    for _ in range(args.warmup):
        ctx.reduce_checked("sum", "float32", dst, src, n)
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.reduce_checked("sum", "float32", dst, src, n)
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    bytes_per_step = 3 * n * 4  # algorithmic: read src, read dst, write dst
    value = world * args.steps * bytes_per_step / elapsed / GIB

    # roofline of the combine kernel: HIP events on the context's own stream
    # (right after the timed steps, so the clocks are up): average launch
    # duration of each of 5 batches of 50 back-to-back launches, median batch;
    # the spread is reported because HBM runs in slower phases of seconds on
    # some boxes ("Slow phases")
    iters = 50
    batch_us = sorted(ctx.profile_reduce("sum", "float32", dst, src, n, iters)
                      for _ in range(5))
    avg_us = batch_us[len(batch_us) // 2]
    achieved = bytes_per_step / (avg_us * 1e-6) / 1e9
    # SURVEY.md 8d also asks for the median of individually timed launches
    singles = sorted(ctx.profile_reduce("sum", "float32", dst, src, n, 1) for _ in range(21))
    median_us = singles[len(singles) // 2]
    # the box's measured ceiling beside it, same geometry and buffers: both
    # operands read with no stores (2N bytes), and a copy (2N bytes); 5
    # batches of 50, median batch, interleaved with the combine
    ceil = {}
    for kind, name in ((0, "read_only"), (1, "copy")):
        ctx.profile_stream(kind, dst, src, n * 4, 20)
        b = sorted(ctx.profile_stream(kind, dst, src, n * 4, 50) for _ in range(5))
        ceil[name] = 2 * n * 4 / (b[2] * 1e-6) / 1e9
    ctx.fill("float32", "round", 0x5EED0001 + 2 * rank, dst, n)   # the copy overwrote dst

    # the user-visible layout beside the headline: src and dst
    # in two separate allocations, as a user's recv.buffer and fragment are,
    # timed the same way (5 batches of 50, median batch)
    sa, sd = ctx.alloc(n * 4), ctx.alloc(n * 4)
    ctx.fill("float32", "round", 0x5EED0000 + 2 * rank, sa.ptr, n)
    ctx.fill("float32", "round", 0x5EED0001 + 2 * rank, sd.ptr, n)
    ctx.profile_reduce("sum", "float32", sd.ptr, sa.ptr, n, 20)
    sep_us = sorted(ctx.profile_reduce("sum", "float32", sd.ptr, sa.ptr, n, iters)
                    for _ in range(5))
    sep_avg = sep_us[len(sep_us) // 2]
    sep_gbs = bytes_per_step / (sep_avg * 1e-6) / 1e9
    separate = {"achieved": round(sep_gbs, 1), "frac": round(sep_gbs / HBM_PEAK_GBS, 4),
                "kernel_avg_us": round(sep_avg, 3),
                "kernel_avg_us_batches": [round(b, 2) for b in sep_us],
                "src": hex(sa.ptr), "dst": hex(sd.ptr),
                "note": "two independent 256 MiB hipMallocs (ucg_builtin_dev_malloc), "
                        "same kernel and timing as the headline"}
    sa.free()
    sd.free()

    traffic, traffic_source = pmc_traffic(n)
    extra = {}
    if not args.no_extra and rank == 0:
        # north-star: 1 GiB fp32 combine, device-resident
        nb = 1 << 28
        pair1 = ctx.alloc(2 * nb * 4)          # one allocation, as the headline pair
        s1, d1 = pair1.ptr, pair1.ptr + nb * 4
        ctx.fill("float32", "round", 11, s1, nb)
        ctx.fill("float32", "round", 12, d1, nb)
        # steady state, as for the headline kernel: 20 launches (10 ms) bring
        # the clocks up from the idle gaps of the single-launch timings above,
        # then the median of 5 batches of 20 back-to-back launches
        ctx.profile_reduce("sum", "float32", d1, s1, nb, 20)
        batches = sorted(ctx.profile_reduce("sum", "float32", d1, s1, nb, 20)
                         for _ in range(5))
        us1 = batches[len(batches) // 2]
        g1 = 3 * nb * 4 / (us1 * 1e-6) / 1e9
        extra["north_star_1gib_fp32_sum"] = {
            "kernel_us": round(us1, 2), "achieved_gbs": round(g1, 1),
            "gibs_3n": round(3 * nb * 4 / (us1 * 1e-6) / GIB, 1),
            "frac_of_8tbs": round(g1 / HBM_PEAK_GBS, 4), "target_frac": 0.80,
            "batch_us": [round(b, 2) for b in batches],
            "timing": "20 warm launches, then median of 5 batches of 20 (HIP events)"}
        pair1.free()
        extra["one_shot_8_operands_64mib_fp32"] = one_shot_shape(ctx)
        # C4's per-GPU shard: 8 operands of 512 MiB
        extra["one_shot_8_operands_512mib_fp32"] = one_shot_shape(ctx, per_op=512 << 20,
                                                                  iters=20)
        extra["same_box_reference_kernels"] = same_box_reference(n)
        # H2D/D2H-inclusive rate: host-resident (pinned) buffers, pipelined
        hs, hd = xucg_amd.HostBuffer(n * 4), xucg_amd.HostBuffer(n * 4)
        ctx.combine_host("sum", "float32", hd, hs, n)  # warm the ring
        reps = 5
        t1 = time.perf_counter()
        for _ in range(reps):
            rc = ctx.combine_host("sum", "float32", hd, hs, n)
            assert rc == 0, xucg_amd._lib.last_error()
        th = (time.perf_counter() - t1) / reps
        extra["pcie_end_to_end_fp32_sum"] = {
            "bytes": n * 4, "ms": round(th * 1e3, 3),
            "gibs_3n": round(3 * n * 4 / th / GIB, 2),
            "gibs_n": round(n * 4 / th / GIB, 2),
            "note": "pinned host src/dst -> H2D -> kernel -> D2H, 16 MiB chunks on 2 streams"}
        hs.free()
        hd.free()

    collective, children_ok, collective_bad = None, True, False
    if (world > 1 and not args.no_collective) or args.collective_force:
        pair.free()
        ctx.close()
        collective, children_ok = run_collective_children(dist, rank, world)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n)
        extra["c1_loopback_allreduce_4kib_fp32"] = c1_loopback()
        extra["f1_staged_step_64mib_fp32"] = staged_step()

    if rank == 0:
        line = {
            "metric": load_baseline_metric(),
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": dist.get_world_size() if dist is not None else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-based splitmix64 generator, 'round' distribution)",
            "config": {
                "workload": "BASELINE config 2: device-resident local combine dst += src, "
                            "2 x 256 MiB fp32 per GPU (ucg_builtin_dev_reduce)",
                "count": n, "op": "sum", "bytes_per_step_per_gpu": bytes_per_step,
                "layout": "src and dst the two halves of one 512 MiB allocation",
                "parallelism": f"{world} independent per-rank shards (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_source,
                "kernel": "ucgdev::k_reduce<float, SUM, 1, 1, 64, XM=1, PF=3, ORD=2, XC=256>",
                "kernel_avg_us": round(avg_us, 3),
                "kernel_avg_us_batches": [round(b, 2) for b in batch_us],
                "kernel_median_us_single_launches": round(median_us, 3),
                "frac_from_median": round(bytes_per_step / (median_us * 1e-6) / 1e9
                                          / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": bytes_per_step,
                "separate_allocations": separate,
                "measured_ceiling_same_box": {
                    "read_only_gbs": round(ceil["read_only"], 1),
                    "copy_gbs": round(ceil["copy"], 1),
                    "combine_frac_of_read_only": round(achieved / ceil["read_only"], 4),
                    "note": "same geometry and buffers, both operands read with no "
                            "stores / src copied to dst (ucg_builtin_dev_profile_stream)"},
            },
            "cpu_baseline": cpu,
            # the shim's process-wide memory accounting at the end of the run:
            # retired address ranges and their cap, the reuse cache
            # (ucg_builtin_dev_mem_stats)
            "shim_memory": xucg_amd._lib.mem_stats(),
            "extra": extra,
            "collective": collective,
        }
        if collective is not None:
            # a failed multi-GPU check fails the run: the line still prints
            # (with collective_ok false and what failed), then a non-zero exit
            fails = collective_failures(collective)
            line["collective_ok"] = not fails and children_ok
            if fails:
                line["collective_failures"] = fails[:20]
            collective_bad = not line["collective_ok"]
        print(json.dumps(line), flush=True)

    ctx.close()
    if not children_ok:
        # a child died on the GPU: leave without touching the device again
        sys.stdout.flush()
        os._exit(3)
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0 and collective_bad:
        sys.exit(3)


if __name__ == "__main__":
    main()
