#!/usr/bin/env python3
"""Timeline of the headline combine from a cold process: does the box's HBM
rate change with how long the GPU has been streaming?

bench.py measures the 2 x 256 MiB combine within its first ~100 ms of load
and the 1 GiB north-star case ~150 ms later; on some boxes the first reads
~80 % of 8 TB/s and the second ~85 % in the same process (r02d). This probe
launches the headline combine back to back in batches of 20 (HIP events on
the context stream) for `seconds`, and prints the median rate per window of
wall time, so a ramp (or a flip between two states) shows with its timing.

    python scripts/ramp_probe.py [seconds=3] [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    n = 1 << 26
    ctx = xucg_amd.DevContext(device=0)
    src, dst = ctx.alloc(n * 4), ctx.alloc(n * 4)
    ctx.fill("float32", "round", 1, src, n)
    ctx.fill("float32", "round", 2, dst, n)
    ctx.sync()
    t0 = time.perf_counter()
    samples = []
    while time.perf_counter() - t0 < seconds:
        us = ctx.profile_reduce("sum", "float32", dst, src, n, 20)
        samples.append((time.perf_counter() - t0, us))
    win = 0.05
    out = []
    k = 0
    while k < len(samples):
        w0 = samples[k][0]
        grp = []
        while k < len(samples) and samples[k][0] < w0 + win:
            grp.append(samples[k][1])
            k += 1
        grp.sort()
        med = grp[len(grp) // 2]
        out.append({"t_ms": round(w0 * 1e3, 1), "batches": len(grp), "median_us": round(med, 2),
                    "frac": round(3 * n * 4 / (med * 1e-6) / 1e9 / PEAK, 4)})
    for row in out:
        print(row, flush=True)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump({"windows": out, "batch_launches": 20, "count": n}, f, indent=1)
    src.free()
    dst.free()
    ctx.close()


if __name__ == "__main__":
    main()
