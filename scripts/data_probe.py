#!/usr/bin/env python3
"""Does the headline kernel's HBM rate depend on the data? The same 1 GiB and
256 MiB fp32 SUM combines on the same buffers, filled with each synthetic
distribution (exact: small integers, round: random mantissas, special: the
special-value table), timed as in bench.py (20 warm launches,
median of 5 batches of 20, HIP events on the context stream). Distributions
interleaved over 3 rounds.

    python scripts/data_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    ctx = xucg_amd.DevContext(device=0)
    rows = []
    for lg in (28, 26):
        n = 1 << lg
        s, d = ctx.alloc(n * 4), ctx.alloc(n * 4)
        for rnd in range(3):
            for dist in ("exact", "round", "special"):
                ctx.fill("float32", dist, 11, s, n)
                ctx.fill("float32", dist, 12, d, n)
                ctx.profile_reduce("sum", "float32", d, s, n, 20)
                b = sorted(ctx.profile_reduce("sum", "float32", d, s, n, 20) for _ in range(5))
                us = b[2]
                gbs = 12 * n / (us * 1e-6) / 1e9
                row = {"bytes_per_operand": n * 4, "dist": dist, "round": rnd,
                       "us": round(us, 2), "frac": round(gbs / PEAK, 4)}
                print(row, flush=True)
                rows.append(row)
        s.free()
        d.free()
    ctx.close()
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
