#!/usr/bin/env python3
"""Is the headline combine's rate a property of its buffers or of its size?

On some boxes the 2 x 256 MiB combine of bench.py runs at ~80 % of 8 TB/s in
the same process where the 1 GiB north-star combine runs at ~85 % (r02d). This
probe separates the two: in one process it allocates the bench's 256 MiB pair
first (as bench.py does), then a 1 GiB pair, and times, interleaved over
rounds,
  bench pair      the 256 MiB pair, full and half size
  big pair        the 1 GiB pair, full, and 64/128/256/512 MiB windows at its
                  start and in its middle (the same physical pages as the fast
                  1 GiB case, at the headline size)
  fresh pair      a 256 MiB pair allocated after everything else
Each entry: median of 3 batches of HIP-event-timed back-to-back launches on
the context stream.

    UCX_BUILTIN_DEV_VARIANT=0 python scripts/size_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0
MIB = 1 << 20


def main():
    ctx = xucg_amd.DevContext(device=0)
    n256 = 64 * MIB // 1          # elements (fp32) in 256 MiB
    c, d = ctx.alloc(n256 * 4), ctx.alloc(n256 * 4)
    nbig = 4 * n256
    a, b = ctx.alloc(nbig * 4), ctx.alloc(nbig * 4)
    e, f = ctx.alloc(n256 * 4), ctx.alloc(n256 * 4)
    for i, buf in enumerate((c, d, a, b, e, f)):
        ctx.fill("float32", "round", 100 + i, buf, buf.nbytes // 4)
    ctx.sync()

    cases = [("bench_pair_256MiB", d, c, 0, n256),
             ("bench_pair_128MiB", d, c, 0, n256 // 2),
             ("big_pair_1GiB", b, a, 0, nbig),
             ("big_pair_512MiB_at_0", b, a, 0, nbig // 2),
             ("big_pair_256MiB_at_0", b, a, 0, n256),
             ("big_pair_256MiB_at_512MiB", b, a, 2 * n256, n256),
             ("big_pair_128MiB_at_0", b, a, 0, n256 // 2),
             ("big_pair_64MiB_at_0", b, a, 0, n256 // 4),
             ("fresh_pair_256MiB", f, e, 0, n256)]
    res = {k: [] for k, *_ in cases}
    rounds = int(os.environ.get("PROBE_ROUNDS", "6"))
    for r in range(rounds):
        for name, dst, src, off, n in cases:
            iters = max(5, int(6000 / (n * 12 / 6.8e6)))   # ~6 ms per batch
            dp, sp = dst.ptr + off * 4, src.ptr + off * 4
            ctx.profile_reduce("sum", "float32", dp, sp, n, 5)
            us = sorted(ctx.profile_reduce("sum", "float32", dp, sp, n, iters)
                        for _ in range(3))[1]
            frac = 3 * n * 4 / (us * 1e-6) / 1e9 / PEAK
            res[name].append(round(frac, 4))
        print(f"round {r}: " + " ".join(f"{k}={v[-1]:.3f}" for k, v in res.items()),
              flush=True)
    summary = {k: {"median_frac": sorted(v)[len(v) // 2], "min": min(v), "max": max(v),
                   "rounds": v} for k, v in res.items()}
    summary["variant"] = os.environ.get("UCX_BUILTIN_DEV_VARIANT", "0")
    print(json.dumps(summary))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fo:
            json.dump(summary, fo, indent=1)
    for buf in (c, d, a, b, e, f):
        buf.free()
    ctx.close()


if __name__ == "__main__":
    main()
