#!/usr/bin/env python3
"""do the dtype gaps of the C3 sweep survive when each pair is
timed interleaved with the fp32 SUM reference on the same buffers? The five
lowest 1 GiB pairs of round 4's sweep (profiles/r04/c3/c3_sweep.json) and
fp32 MIN / MAX, each alternated with fp32 SUM over rounds in one process:
per round, 20 back-to-back launches of the pair and 20 of fp32 SUM, in
alternating order (HIP events on the context stream,
ucg_builtin_dev_profile_reduce). Reported per
pair: its median % of 8 TB/s, the interleaved fp32 SUM's, and the median of
the per-round ratios - a ratio near 1 means the sweep's gap was the box's
phase, not the dtype.

    python scripts/c3_interleaved.py [out.json] [rounds = 8]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

PEAK = 8000.0
PAIRS = [("uint32", "min"), ("uint16", "band"), ("int64", "bxor"), ("uint32", "sum"),
         ("uint32", "max"), ("float32", "min"), ("float32", "max")]
BYTES = 1 << 30             # per operand, the north-star size


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ctx = xucg_amd.DevContext(device=0)
    pair = ctx.alloc(2 * BYTES)            # one allocation, the bench's layout
    src, dst = pair.ptr, pair.ptr + BYTES
    res = {"bytes_per_operand": BYTES, "rounds": rounds, "launches_per_sample": 20,
           "pairs": []}
    for dt, op in PAIRS:
        sz = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
        n, nf = BYTES // sz, BYTES // 4
        ctx.fill(dt, "round", 1, src, n)
        ctx.fill(dt, "round", 2, dst, n)
        ctx.sync()
        ctx.profile_reduce(op, dt, dst, src, n, 5)
        ctx.profile_reduce("sum", "float32", dst, src, nf, 5)
        p_us, f_us = [], []
        for r in range(rounds):
            # the order alternates, so neither side always runs second
            if r % 2:
                f_us.append(ctx.profile_reduce("sum", "float32", dst, src, nf, 20))
                p_us.append(ctx.profile_reduce(op, dt, dst, src, n, 20))
            else:
                p_us.append(ctx.profile_reduce(op, dt, dst, src, n, 20))
                f_us.append(ctx.profile_reduce("sum", "float32", dst, src, nf, 20))
        frac = [3 * BYTES / (u * 1e-6) / 1e9 / PEAK for u in p_us]
        ffrac = [3 * BYTES / (u * 1e-6) / 1e9 / PEAK for u in f_us]
        row = {"dtype": dt, "op": op,
               "frac_median": round(statistics.median(frac), 4),
               "fp32_sum_frac_median": round(statistics.median(ffrac), 4),
               "ratio_median": round(statistics.median(f / p for p, f in zip(p_us, f_us)), 4),
               "pair_us": [round(u, 2) for u in p_us], "fp32_sum_us": [round(u, 2) for u in f_us]}
        res["pairs"].append(row)
        print(f"{dt:8s} {op:5s} {100 * row['frac_median']:5.1f} %  fp32 sum "
              f"{100 * row['fp32_sum_frac_median']:5.1f} %  ratio {row['ratio_median']:.4f}",
              flush=True)
    pair.free()
    ctx.close()
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
