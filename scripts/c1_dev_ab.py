"""A/B of the device-buffer allreduce latency through the C1 harness
(tests/c/c1_allreduce.c, C1_DEVICE_BUFFERS=1, registered send buffers), the
same command as bench.py's extra.c1_loopback_allreduce_4kib_fp32
.device_buffers_* legs, alternating settings over several repetitions.

    python scripts/c1_dev_ab.py OUT.json [reps]

Settings: the default library (the context's second stream created with it),
UCX_BUILTIN_DEV_D2H_STREAM=lazy (created on first use, round 2's default),
the same with GPU_MAX_HW_QUEUES=2, the default with GPU_MAX_HW_QUEUES=1, and
the completion by hipStreamSynchronize (UCX_BUILTIN_DEV_COMPLETION=sync).
The parent never touches the GPU: ranks are child processes."""
import json
import os
import subprocess
import sys
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "_build", "c1_allreduce")


def run(world, count, iters, env_extra):
    allowed = sorted(os.sched_getaffinity(0))
    name = f"ucg_ab_{os.getpid()}_{uuid.uuid4().hex[:6]}"
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), C1_DEVICE_BUFFERS="1",
                   C1_REGISTERED="1", UCX_BUILTIN_WAIT_TIMEOUT="60", **env_extra)
        procs.append(subprocess.Popen([EXE, name, str(iters), "256", str(count)], env=env,
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
    settings = {"default": {}, "d2h_lazy": {"UCX_BUILTIN_DEV_D2H_STREAM": "lazy"},
                "d2h_lazy_hwq2": {"UCX_BUILTIN_DEV_D2H_STREAM": "lazy", "GPU_MAX_HW_QUEUES": "2"},
                "hwq1": {"GPU_MAX_HW_QUEUES": "1"},
                "sync": {"UCX_BUILTIN_DEV_COMPLETION": "sync"}}
    res = {k: {"4kib_us": [], "64mib_us": []} for k in settings}
    for rep in range(reps):
        for k, env in settings.items():
            for size, count, iters in (("4kib_us", 1024, 2000), ("64mib_us", 1 << 24, 20)):
                r = run(4, count, iters, env)
                res[k][size].append(r.get("latency_us", r.get("error")))
                if not r.get("bit_exact", False):
                    res[k].setdefault("errors", []).append(r)
        print(json.dumps({"rep": rep, **res}), flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
