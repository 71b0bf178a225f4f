#!/usr/bin/env python3
"""Is the combine's throughput a property of the allocation? Fresh hipMalloc
pairs (interleaved with differently sized spacer allocations to move them
around), each timed with the product kernel and with torch's add_ on the same
buffers (torch tensors over the same device memory via DLPack-free views:
the combine writes through pointers, torch through its own allocations of the
same size right after).

    python scripts/alloc_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import xucg_amd  # noqa: E402

N = 1 << 26
PEAK = 8000.0


def frac(us):
    return round(3 * N * 4 / (us * 1e-6) / 1e9 / PEAK, 4)


def main():
    ctx = xucg_amd.DevContext.on_torch_stream(0)
    res = []
    spacers = []
    for trial in range(8):
        spacers.append(ctx.alloc((trial * 37 + 5) << 20))
        src, dst = ctx.alloc(N * 4), ctx.alloc(N * 4)
        ctx.fill("float32", "round", 1, src, N)
        ctx.fill("float32", "round", 2, dst, N)
        ctx.sync()
        us = min(ctx.profile_reduce("sum", "float32", dst, src, N, 50) for _ in range(3))
        a = torch.empty(N, device="cuda")
        b = torch.empty(N, device="cuda")
        ctx.fill("float32", "round", 1, a, N)
        ctx.fill("float32", "round", 2, b, N)
        us_t = min(ctx.profile_reduce("sum", "float32", b, a, N, 50) for _ in range(3))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            b.add_(a)
        e1.record()
        e1.synchronize()
        t_add = e0.elapsed_time(e1) * 1e3 / 50
        row = {"trial": trial, "src": hex(src.ptr), "dst": hex(dst.ptr),
               "combine_hipmalloc_frac": frac(us), "combine_torchalloc_frac": frac(us_t),
               "torch_add_frac": frac(t_add)}
        print(row, flush=True)
        res.append(row)
        src.free()
        dst.free()
        del a, b
    for s in spacers:
        s.free()
    ctx.close()
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
