"""A/B of the device-buffer allreduce latency through the C1 harness
(tests/c/c1_allreduce.c, C1_DEVICE_BUFFERS=1, registered send buffers), the
same command as bench.py's extra.c1_loopback_allreduce_4kib_fp32
.device_buffers_* legs, alternating settings over several repetitions.

    python scripts/c1_dev_ab.py OUT.json [reps] [r03|r04|r05]

r03 settings: the default library (the context's second stream created with
it), UCX_BUILTIN_DEV_D2H_STREAM=lazy (created on first use, round 2's
default), the same with GPU_MAX_HW_QUEUES=2, the default with
GPU_MAX_HW_QUEUES=1, and the completion by hipStreamSynchronize
(UCX_BUILTIN_DEV_COMPLETION=sync).
r04 settings (the device-buffer latency went from 12 to 95 us between the
rounds): the default; hipMalloc memory and hipIpc keys instead of shareable
memory (UCX_BUILTIN_DEV_SHAREABLE=n); no pool arena
(UCX_BUILTIN_DEV_POOL_BYTES=0); both; the send buffer not registered.
r05 settings (the default): the default (plain pools and staging ring), the
pools in shareable memory, host buffers with every step staged on the GPU
(C1_DEVICE_STAGING), the send buffer not registered.
The parent never touches the GPU: ranks are child processes."""
import json
import os
import subprocess
import sys
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "_build", "c1_allreduce")


def run(world, count, iters, env_extra, prof=None):
    """prof: a directory; rank 0 then runs under rocprofv3 (kernel and HIP API
    traces with their statistics, no counters)"""
    allowed = sorted(os.sched_getaffinity(0))
    name = f"ucg_ab_{os.getpid()}_{uuid.uuid4().hex[:6]}"
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), C1_DEVICE_BUFFERS="1",
                   C1_REGISTERED="1", UCX_BUILTIN_WAIT_TIMEOUT="60")
        env.update(env_extra)
        env = {k: v for k, v in env.items() if v is not None}
        cmd = [EXE, name, str(iters), "256", str(count)]
        if prof and r == 0:
            cmd = ["rocprofv3", "--kernel-trace", "--hip-trace", "--stats", "--output-format",
                   "csv", "-d", prof, "-o", "c1", "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True,
                                      preexec_fn=lambda c=allowed[r % len(allowed)]:
                                      os.sched_setaffinity(0, {c})))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    try:
        return json.loads(outs[0].strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": outs[0][-400:]}


def main():
    out, reps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    which = sys.argv[3] if len(sys.argv) > 3 else "r05"
    if which == "r05":
        # round 5: pools and staging in plain memory; a process
        # owning virtual memory time-slices every process on the GPU
        settings = {"default": {},
                    "pools_shareable": {"UCX_BUILTIN_DEV_POOL_MEM": "shareable"},
                    "host_buffers_staged": {"C1_DEVICE_BUFFERS": None, "C1_REGISTERED": None,
                                            "C1_DEVICE_STAGING": "1"},
                    "send_not_registered": {"C1_REGISTERED": None}}
    elif which == "r03":
        settings = {"default": {}, "d2h_lazy": {"UCX_BUILTIN_DEV_D2H_STREAM": "lazy"},
                    "d2h_lazy_hwq2": {"UCX_BUILTIN_DEV_D2H_STREAM": "lazy",
                                      "GPU_MAX_HW_QUEUES": "2"},
                    "hwq1": {"GPU_MAX_HW_QUEUES": "1"},
                    "sync": {"UCX_BUILTIN_DEV_COMPLETION": "sync"}}
    else:
        settings = {"default": {},
                    "plain_memory": {"UCX_BUILTIN_DEV_SHAREABLE": "n"},
                    "no_arena": {"UCX_BUILTIN_DEV_POOL_BYTES": "0"},
                    "plain_no_arena": {"UCX_BUILTIN_DEV_SHAREABLE": "n",
                                       "UCX_BUILTIN_DEV_POOL_BYTES": "0"},
                    "send_not_registered": {"C1_REGISTERED": None}}
    res = {k: {"4kib_us": [], "64mib_us": []} for k in settings}
    for rep in range(reps):
        for k, env in settings.items():
            for size, count, iters in (("4kib_us", 1024, 2000), ("64mib_us", 1 << 24, 20)):
                r = run(4, count, iters, env)
                res[k][size].append(r.get("latency_us", r.get("error")))
                if not r.get("bit_exact", False):
                    res[k].setdefault("errors", []).append(r)
        print(json.dumps({"rep": rep, **res}), flush=True)
    if os.environ.get("C1_AB_PROFILE"):
        res["profiled_default_4kib"] = run(4, 1024, 2000, {}, prof=os.environ["C1_AB_PROFILE"])
        print(json.dumps(res["profiled_default_4kib"]), flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
