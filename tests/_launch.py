"""Launch N worker processes (one per rank) as children and collect exit codes.

Workers are started with subprocess (fork + exec in the child), never by
replacing this process; every worker gets a hard time limit and is killed by
its exact PID when it overruns."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(worker, world, args=(), timeout=240, env_extra=None):
    return launch_exe(os.path.join(ROOT, "tests", worker), world, args, timeout,
                      python=True, env_extra=env_extra)


def launch_exe(exe, world, args=(), timeout=240, python=False, env_extra=None):
    port = free_port()
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["MASTER_ADDR"] = "127.0.0.1"
    env["MASTER_PORT"] = str(port)
    env["WORLD_SIZE"] = str(world)
    env.setdefault("OMP_NUM_THREADS", "1")
    # a worker that crashes names where: its Python stack, and the native one
    # (xucg_amd/csrc/dev_mem.hip, XUCG_NATIVE_BACKTRACE)
    env.setdefault("PYTHONFAULTHANDLER", "1")
    env.setdefault("XUCG_NATIVE_BACKTRACE", "1")
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        e.update(env_extra or {})
        cmd = ([sys.executable] if python else []) + [exe, *map(str, args)]
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    # one deadline for the whole group: a hung group ends after `timeout`,
    # not after world x timeout
    deadline = time.monotonic() + timeout
    outs, codes = [], []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=max(1.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
            out += "\n<killed: timeout>"
        outs.append(out)
        codes.append(p.returncode)
    # XUCG_LAUNCH_LOG=<file>: every rank's output appended there, passing
    # groups included (slow-call notes of a run that still passed)
    log = os.environ.get("XUCG_LAUNCH_LOG")
    if log:
        with open(log, "a") as f:
            f.write(f"=== {os.path.basename(exe)} {' '.join(map(str, args))} "
                    f"codes {codes}\n")
            for r, out in enumerate(outs):
                f.write("".join(f"[{r}] {line}\n" for line in out.splitlines()))
    return codes, outs
