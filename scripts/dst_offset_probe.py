#!/usr/bin/env python3
"""Does the destination's offset within a 128-B line matter? The combine
(fp32 SUM, 256 MiB operands) with dst and src at the same offset past a
256-B boundary (in phase: the aligned kernel, with a byte head when the
offset is not a multiple of 16), then with src out of phase. A wave stores a
contiguous 1 KiB; unless dst's vector region starts on a 128-B line, the
first and last lines of every wave's span are shared with its neighbours.

    python scripts/dst_offset_probe.py [out.json]
    UCX_BUILTIN_DEV_VARIANT=14 python scripts/dst_offset_probe.py   # no XCD map
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
    nbytes = int(os.environ.get("PROBE_BYTES", 256 << 20))
    n = nbytes // 4
    bs, bd = ctx.alloc(nbytes + 512), ctx.alloc(nbytes + 512)
    ctx.fill("float32", "round", 1, bs, n + 128)
    ctx.fill("float32", "round", 2, bd, n + 128)
    rows = []
    for d_off, s_off in ((0, 0), (16, 16), (32, 32), (64, 64), (112, 112), (4, 4), (68, 68),
                         (0, 4), (16, 4), (64, 68), (4, 0), (0, 16), (0, 64), (64, 0),
                         (48, 0)):
        dp, sp = bd.ptr + d_off, bs.ptr + s_off
        ctx.profile_reduce("sum", "float32", dp, sp, n, 20)
        b = sorted(ctx.profile_reduce("sum", "float32", dp, sp, n, 20) for _ in range(5))
        us = b[2]
        gbs = 3 * nbytes / (us * 1e-6) / 1e9
        row = {"dst_offset": d_off, "src_offset": s_off, "us": round(us, 2),
               "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
        print(row, flush=True)
        rows.append(row)
    ctx.close()
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
