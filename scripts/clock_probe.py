#!/usr/bin/env python3
"""Do the slow phases of the headline combine (~80 % of 8 TB/s instead of
~85 %) follow a clock? r02sh: a fresh box read 79.9 %, the same box after two
minutes of the GPU test suite 84.6 %. This probe keeps the combine running
(bench.py's geometry, batches of 200 launches timed with HIP events) for
`seconds`, while a thread samples `rocm-smi --showclocks` (sclk, mclk,
fclk, socclk) once a second, and writes both series.

    python scripts/clock_probe.py SECONDS [out.json]
"""
import json
import os
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0
N = 1 << 26
CLK = re.compile(r"(\w+) clock level: \S+ \((\d+)Mhz\)")


def sampler(stop, t0, out):
    while not stop.is_set():
        try:
            txt = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True,
                                 text=True, timeout=10).stdout
            out.append({"t": round(time.perf_counter() - t0, 2),
                        **{k: int(v) for k, v in CLK.findall(txt)}})
        except (OSError, subprocess.SubprocessError) as e:
            out.append({"t": round(time.perf_counter() - t0, 2), "error": str(e)[:80]})
        stop.wait(1.0)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    ctx = xucg_amd.DevContext(device=0)
    s, d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    ctx.fill("float32", "round", 1, s, N)
    ctx.fill("float32", "round", 2, d, N)
    ctx.sync()
    clocks, fracs = [], []
    stop = threading.Event()
    t0 = time.perf_counter()
    th = threading.Thread(target=sampler, args=(stop, t0, clocks), daemon=True)
    th.start()
    last = 0.0
    while time.perf_counter() - t0 < seconds:
        us = ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 200)
        t = time.perf_counter() - t0
        fracs.append({"t": round(t, 2), "frac": round(3 * N * 4 / (us * 1e-6) / 1e9 / PEAK, 4)})
        if t - last > 5:
            print(fracs[-1], clocks[-1] if clocks else None, flush=True)
            last = t
    stop.set()
    th.join(timeout=15)
    res = {"seconds": seconds, "combine": fracs, "clocks": clocks}
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f)
    s.free()
    d.free()
    ctx.close()


if __name__ == "__main__":
    main()
