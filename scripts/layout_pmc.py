#!/usr/bin/env python3
"""The headline combine (2 x 256 MiB fp32 SUM, k_reduce) on the two operand
layouts, for rocprofv3 counter passes: first `reps` launches
with src and dst the two halves of ONE allocation (bench.py's headline
layout), then `reps` launches with src and dst in TWO separate allocations (a
user's recv.buffer and fragment). Dispatch order tells the layouts apart in
the per-dispatch CSV (scripts/layout_pmc_summary.py). Also prints the HIP
event timing of both.

    rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum ... -- python3 scripts/layout_pmc.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import xucg_amd
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 1 << 26
    ctx = xucg_amd.DevContext(device=0)
    pair = ctx.alloc(2 * n * 4)
    a, b = ctx.alloc(n * 4), ctx.alloc(n * 4)
    layouts = {"joint": (pair.ptr + n * 4, pair.ptr), "separate": (b.ptr, a.ptr)}
    for dst, src in layouts.values():
        ctx.fill("float32", "round", 1, src, n)
        ctx.fill("float32", "round", 2, dst, n)
    ctx.sync()
    out = {}
    for name, (dst, src) in layouts.items():
        us = ctx.profile_reduce("sum", "float32", dst, src, n, reps)
        out[name] = {"dst": hex(dst), "src": hex(src), "kernel_us": round(us, 2),
                     "frac_of_8tbs": round(3 * n * 4 / (us * 1e-6) / 8e12, 4)}
    print(json.dumps(out), flush=True)
    pair.free()
    a.free()
    b.free()
    ctx.close()


if __name__ == "__main__":
    main()
