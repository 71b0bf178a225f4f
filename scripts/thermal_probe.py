#!/usr/bin/env python3
"""Do the slow phases of the headline combine (~80 % of 8 TB/s instead of
~85 %) follow the HBM temperature? The clocks do not (clock_probe.py, r02ck /
r02cp). This probe (1) keeps bench.py's 2 x 256 MiB fp32 combine running
back to back for HEAT seconds, timing batches of 200 launches with HIP
events, then (2) times one batch every 3 s for COOL seconds with the GPU idle
in between, while a thread samples `rocm-smi --showtemp` (edge, junction,
memory sensors) once a second. Both series are written to OUT.

    python scripts/thermal_probe.py HEAT COOL OUT.json
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
TEMP = re.compile(r"Temperature \(Sensor (\w+)\) \(C\): ([\d.]+)")


def sampler(stop, t0, out):
    while not stop.is_set():
        try:
            txt = subprocess.run(["rocm-smi", "--showtemp"], capture_output=True,
                                 text=True, timeout=10).stdout
            out.append({"t": round(time.perf_counter() - t0, 2),
                        **{k: float(v) for k, v in TEMP.findall(txt)}})
        except (OSError, subprocess.SubprocessError) as e:
            out.append({"t": round(time.perf_counter() - t0, 2), "error": str(e)[:80]})
        stop.wait(1.0)


def main():
    heat, cool, out = float(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
    ctx = xucg_amd.DevContext(device=0)
    s, d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    ctx.fill("float32", "round", 1, s, N)
    ctx.fill("float32", "round", 2, d, N)
    ctx.sync()
    temps, fracs = [], []
    stop = threading.Event()
    t0 = time.perf_counter()
    th = threading.Thread(target=sampler, args=(stop, t0, temps), daemon=True)
    th.start()

    def batch(phase):
        us = ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 200)
        fracs.append({"t": round(time.perf_counter() - t0, 2), "phase": phase,
                      "frac": round(3 * N * 4 / (us * 1e-6) / 1e9 / PEAK, 4)})

    last = 0.0
    while time.perf_counter() - t0 < heat:
        batch("heat")
        if fracs[-1]["t"] - last > 10:
            print(fracs[-1], temps[-1] if temps else None, flush=True)
            last = fracs[-1]["t"]
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < cool:
        batch("cool")
        print(fracs[-1], temps[-1] if temps else None, flush=True)
        time.sleep(3.0)
    stop.set()
    th.join(timeout=15)
    with open(out, "w") as f:
        json.dump({"heat_s": heat, "cool_s": cool, "combine": fracs, "temps": temps}, f)
    s.free()
    d.free()
    ctx.close()


if __name__ == "__main__":
    main()
