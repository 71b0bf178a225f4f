#!/usr/bin/env python3
"""Does freeing a large VRAM allocation slow the headline combine for a
while afterwards (driver-side clearing of released memory competing for
HBM)? r02s11: bench.py read 80 % right after the GPU suite (which allocates
and frees 32-64 GiB operands), and 85 % one minute later. In one process:
the 2 x 256 MiB fp32 combine timed in batches of 50 launches every 0.5 s,
(A) as is, (B) after a GIB-GiB buffer is allocated, filled and freed,
(C) after one is allocated and freed untouched.

    python scripts/free_probe.py GIB SECONDS OUT.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0
N = 1 << 26


def main():
    gib, secs, out = int(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
    ctx = xucg_amd.DevContext(device=0)
    s, d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    ctx.fill("float32", "round", 1, s, N)
    ctx.fill("float32", "round", 2, d, N)
    ctx.sync()
    res = {"gib": gib}

    def watch(tag, dur):
        t0, series = time.perf_counter(), []
        while time.perf_counter() - t0 < dur:
            us = ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 50)
            series.append((round(time.perf_counter() - t0, 2),
                           round(3 * N * 4 / (us * 1e-6) / 1e9 / PEAK, 4)))
            time.sleep(0.5)
        res[tag] = series
        fr = [f for _, f in series]
        print(f"{tag}: first 5 {fr[:5]} min {min(fr)} median {sorted(fr)[len(fr) // 2]} "
              f"last 5 {fr[-5:]}", flush=True)

    watch("A_baseline", 10)
    t = time.perf_counter()
    big = ctx.alloc(gib << 30)
    ctx.fill("uint8", "round", 3, big, gib << 30)
    ctx.sync()
    big.free()
    print(f"B: alloc+fill+free {time.perf_counter() - t:.2f} s", flush=True)
    watch("B_after_filled_free", secs)
    t = time.perf_counter()
    big = ctx.alloc(gib << 30)
    ctx.sync()
    big.free()
    print(f"C: alloc+free {time.perf_counter() - t:.2f} s", flush=True)
    watch("C_after_untouched_free", secs)
    with open(out, "w") as f:
        json.dump(res, f)
    s.free()
    d.free()
    ctx.close()


if __name__ == "__main__":
    main()
