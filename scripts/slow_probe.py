#!/usr/bin/env python3
"""What do the boxes on which the headline combine reads ~80 % of 8 TB/s
(instead of ~85 %) have in common? On them the two-stream read probe of
bench.py also drops (6.80 vs 7.21-7.27 TB/s) while the copy does not (6.70 vs
6.64-6.68 TB/s): reads slow down, writes do not. This probe times, in one
process, the combine, the two-stream read and the copy (same geometry,
HIP events, median of 3 batches) on
  - the bench's pair (two separate 256 MiB allocations), and
  - src and dst carved out of one allocation at distances of 256 MiB plus
    0, 4 KiB, 64 KiB, 1 MiB and 2 MiB + 4 KiB (where the two streams fall in
    the channel / bank interleave),
  - a one-stream read (src = dst: the second load of each lane is an L2
    hit, so HBM sees one stream of N bytes).

    python scripts/slow_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0
N = 1 << 26            # fp32 elements per operand (256 MiB)


def med3(f):
    f()
    return sorted(f() for _ in range(3))[1]


def main():
    ctx = xucg_amd.DevContext(device=0)
    a, b = ctx.alloc(N * 4), ctx.alloc(N * 4)
    big = ctx.alloc(2 * N * 4 + (4 << 20))
    for i, buf in enumerate((a, b, big)):
        ctx.fill("float32", "round", 40 + i, buf, buf.nbytes // 4)
    ctx.sync()
    pairs = [("separate allocations", b.ptr, a.ptr)]
    for extra in (0, 4096, 65536, 1 << 20, (2 << 20) + 4096):
        pairs.append((f"one allocation, dst = src + 256 MiB + {extra} B",
                      big.ptr + N * 4 + extra, big.ptr))
    rows = []
    for rnd in range(2):
        for name, d, s in pairs:
            cu = med3(lambda: ctx.profile_reduce("sum", "float32", d, s, N, 40))
            ru = med3(lambda: ctx.profile_stream(0, d, s, N * 4, 40))
            pu = med3(lambda: ctx.profile_stream(1, d, s, N * 4, 40))
            row = {"round": rnd, "pair": name,
                   "combine_frac": round(3 * N * 4 / (cu * 1e-6) / 1e9 / PEAK, 4),
                   "read2_gbs": round(2 * N * 4 / (ru * 1e-6) / 1e9, 1),
                   "copy_gbs": round(2 * N * 4 / (pu * 1e-6) / 1e9, 1)}
            ctx.fill("float32", "round", 41, d, N)      # the copy overwrote dst
            print(row, flush=True)
            rows.append(row)
        # one stream: both loads of a lane on the same address (the second
        # an L2 hit), so HBM sees N bytes of reads in one stream
        ou = med3(lambda: ctx.profile_stream(0, a.ptr, a.ptr, N * 4, 40))
        rows.append({"round": rnd, "pair": "one stream (src = dst)",
                     "read1_gbs": round(N * 4 / (ou * 1e-6) / 1e9, 1)})
        print(rows[-1], flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)
    for buf in (a, b, big):
        buf.free()
    ctx.close()


if __name__ == "__main__":
    main()
