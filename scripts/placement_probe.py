#!/usr/bin/env python3
"""Does the combine's throughput depend on where src and dst sit relative to
each other? Same 2^26-element fp32 operands carved out of one allocation at
different distances, timed with the product kernel (HIP events, 50 launches)
and with torch's in-place add on the same views.

    python scripts/placement_probe.py [out.json]
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


def main():
    ctx = xucg_amd.DevContext.on_torch_stream(0)
    pad = 64 << 20                      # elements of slack (256 MiB)
    base = torch.empty(2 * N + pad, dtype=torch.float32, device="cuda")
    ctx.fill("float32", "round", 1, base, base.numel())
    torch.cuda.synchronize()
    res = []
    # distances between src and dst starts, in bytes beyond N * 4
    for extra in (0, 256, 4096, 65536, 1 << 20, (2 << 20), (2 << 20) + 4096,
                  (8 << 20) + 12288, (32 << 20) + 65536, (64 << 20), (128 << 20) + 4096):
        off = N + extra // 4
        src = base[0:N]
        dst = base[off:off + N]
        us = []
        for _ in range(3):
            us.append(ctx.profile_reduce("sum", "float32", dst, src, N, 50))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            dst.add_(src)
        e0.record()
        for _ in range(50):
            dst.add_(src)
        e1.record()
        e1.synchronize()
        t_us = e0.elapsed_time(e1) * 1e3 / 50
        row = {"dst_minus_src_bytes": off * 4, "combine_us": round(min(us), 2),
               "combine_frac": round(3 * N * 4 / (min(us) * 1e-6) / 1e9 / PEAK, 4),
               "torch_add_us": round(t_us, 2),
               "torch_frac": round(3 * N * 4 / (t_us * 1e-6) / 1e9 / PEAK, 4)}
        print(row, flush=True)
        res.append(row)
    ctx.close()
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
