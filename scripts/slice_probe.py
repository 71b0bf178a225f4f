#!/usr/bin/env python3
"""Run tools/slice_probe (the ~37 us quantized kernel
durations with several processes on one GPU) over its modes, NP processes
per case, started together (this parent never touches the GPU), and write
one JSON line per case with every rank's result.

    python scripts/slice_probe.py OUTDIR [NP=4] [ITERS=2000] [case ...]

A case is mem:imp:act (tools/src/slice_probe.c); the default list runs the
plain and the shareable buffer, each with no imports, imports held and
imports read, every process active, then the engine's pattern (imports
read) with only rank 0 active, and with 2 processes.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "slice_probe")

DEFAULT = ["plain:none:all", "plain:held:all", "plain:read:all",
           "shareable:none:all", "shareable:held:all", "shareable:read:all",
           "shareable:read:one", "plain:read:one", "shareable:read:all:2",
           "plain:read:all:2"]


def run_case(case, np_default, iters):
    parts = case.split(":")
    mem, imp, act = parts[:3]
    np_ = int(parts[3]) if len(parts) > 3 else np_default
    d = tempfile.mkdtemp(prefix="xucg_slice_")
    # SLICE_PROF_DIR: rank 0 runs under rocprofv3's kernel trace (the program
    # itself after --, no launcher hop)
    prof = os.environ.get("SLICE_PROF_DIR")
    try:
        procs = []
        for r in range(np_):
            cmd = [EXE, d, str(r), str(np_), mem, imp, act, str(iters)]
            if prof and r == 0:
                # SLICE_PROF_TRACE: the rocprofv3 trace options (default the
                # kernel trace; "--hsa-trace" lists the runtime's HSA calls,
                # queue creation included)
                opts = os.environ.get("SLICE_PROF_TRACE", "--kernel-trace").split()
                cmd = ["rocprofv3"] + opts + ["--stats", "-d", prof, "-o",
                                              case.replace(":", "_"), "--output-format",
                                              "csv", "--"] + cmd
            procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                          stderr=subprocess.STDOUT, text=True))
        ranks = []
        for r, p in enumerate(procs):
            try:
                out, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                p.kill()
                out = p.communicate()[0] + " <killed: timeout>"
            js = [ln for ln in out.splitlines() if ln.startswith("{")]
            line = js[-1] if js else ""
            try:
                ranks.append(json.loads(line))
            except ValueError:
                ranks.append({"rank": r, "exit": p.returncode, "tail": out[-400:]})
        return {"case": case, "np": np_, "ranks": ranks}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/slice"
    np_ = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    cases = sys.argv[4:] or DEFAULT
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "slice_probe.jsonl"), "a") as f:
        for c in cases:
            res = run_case(c, np_, iters)
            f.write(json.dumps(res) + "\n")
            f.flush()
            p50 = [r.get("op_us", {}).get("p50") for r in res["ranks"]]
            ev = [(r.get("evicted_ms_after", 0) or 0) - (r.get("evicted_ms_before", 0) or 0)
                  for r in res["ranks"]]
            print(f"{c}: p50 us {p50} evicted_ms {ev} "
                  f"queues {[r.get('queues_after_loop') for r in res['ranks']]}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
