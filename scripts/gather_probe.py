#!/usr/bin/env python3
"""Single-GPU roofline of the all-gather and push-copy kernels
(ucg_builtin_dev_gather_multi, ucg_builtin_dev_copy_multi): 8 local rows of
S bytes, 2 x 8 x S algorithmic bytes per launch (read every row, write it).
On one GPU every source is local HBM, so this isolates the kernels from xGMI.
Three layouts: rows on 16-B boundaries; rows of a ragged length at a common
unaligned offset (sources in their destination's phase: the vector kernel
with byte heads and tails); sources out of phase (realigned in registers;
UCX_BUILTIN_DEV_VARIANT=4: the byte loop it replaced).

    python scripts/gather_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

PEAK = 8000.0
NSRC = 8


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    batches = []
    for _ in range(5):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        batches.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(batches)[2]


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    ctx = xucg_amd.DevContext.on_torch_stream(0)
    rows = []
    for base in (64 << 20, 256 << 20):
        bufs = [torch.empty(base + 64, dtype=torch.uint8, device="cuda") for _ in range(NSRC)]
        outs = [torch.empty(base + 64, dtype=torch.uint8, device="cuda") for _ in range(NSRC)]
        big = torch.empty(NSRC * (base + 64) + 64, dtype=torch.uint8, device="cuda")
        for b in bufs:
            b.random_(0, 256)
        for case, shard, src_off, dst_off in (
                ("aligned", base, lambda r: 0, 0),
                ("ragged_common_offset", base + 3,
                 lambda r: (4 + r * (base + 3)) % 16, 4),
                ("out_of_phase", base + 3, lambda r: 0, 4)):
            srcs = [b.data_ptr() + src_off(r) for r, b in enumerate(bufs)]
            dst = big.data_ptr() + dst_off

            def gather():
                return ctx.gather_multi(dst, srcs, shard)
            assert gather() == 0, _lib.last_error()
            torch.cuda.synchronize()
            # spot check the first and last rows' ends
            for r in (0, NSRC - 1):
                got = big[dst_off + r * shard:dst_off + (r + 1) * shard]
                want = bufs[r][src_off(r):src_off(r) + shard]
                assert torch.equal(got[:4096], want[:4096]) and \
                    torch.equal(got[-4096:], want[-4096:]), (case, r)
            us = timed(gather)
            gbs = 2 * NSRC * shard / (us * 1e-6) / 1e9
            row = {"kernel": "gather_multi", "case": case, "rows": NSRC, "row_bytes": shard,
                   "us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
            print(row, flush=True)
            rows.append(row)

            dsts = [o.data_ptr() + dst_off for o in outs]
            copy_srcs = srcs if case != "ragged_common_offset" else \
                [b.data_ptr() + dst_off for b in bufs]

            def copy():
                return ctx.copy_multi(dsts, copy_srcs, shard)
            assert copy() == 0, _lib.last_error()
            torch.cuda.synchronize()
            us = timed(copy)
            gbs = 2 * NSRC * shard / (us * 1e-6) / 1e9
            row = {"kernel": "copy_multi", "case": case, "pairs": NSRC, "bytes": shard,
                   "us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
            print(row, flush=True)
            rows.append(row)
        del bufs, outs, big
        torch.cuda.empty_cache()
    ctx.close()
    if out_path:
        with open(out_path, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    np.random.seed(0)
    main()
