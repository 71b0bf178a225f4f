#!/usr/bin/env python3
"""Is a slow combine a property of the process? r02q: on one box bench.py
read 80.3 % (two-stream read 6.80 TB/s) while slow_probe.py, three minutes
later in another process, read 85.7 % (7.24 TB/s). This probe times the
headline combine and the two-stream read (bench.py's geometry, HIP events,
median of 5 batches of 50) in one process:
  1. on buffers allocated before torch is imported,
  2. on the same buffers after `import torch` and torch's device init,
  3. on fresh buffers allocated after that,
  4. on the first buffers again after torch allocated and freed 4 GiB.

    python scripts/proc_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402

PEAK = 8000.0
N = 1 << 26


def med5(f):
    f()
    return sorted(f() for _ in range(5))[2]


def measure(ctx, d, s, label, rows):
    cu = med5(lambda: ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 50))
    ru = med5(lambda: ctx.profile_stream(0, d.ptr, s.ptr, N * 4, 50))
    row = {"stage": label, "combine_frac": round(3 * N * 4 / (cu * 1e-6) / 1e9 / PEAK, 4),
           "read2_gbs": round(2 * N * 4 / (ru * 1e-6) / 1e9, 1),
           "src_mod_2m": s.ptr % (2 << 20), "dst_mod_2m": d.ptr % (2 << 20)}
    print(row, flush=True)
    rows.append(row)


def main():
    rows = []
    ctx = xucg_amd.DevContext(device=0)
    s, d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    ctx.fill("float32", "round", 1, s, N)
    ctx.fill("float32", "round", 2, d, N)
    ctx.sync()
    measure(ctx, d, s, "before torch", rows)
    import torch
    torch.cuda.init()
    torch.cuda.synchronize()
    measure(ctx, d, s, "after torch init", rows)
    s2, d2 = ctx.alloc(N * 4), ctx.alloc(N * 4)
    ctx.fill("float32", "round", 3, s2, N)
    ctx.fill("float32", "round", 4, d2, N)
    ctx.sync()
    measure(ctx, d2, s2, "fresh buffers after torch init", rows)
    t = torch.empty(1 << 30, dtype=torch.float32, device="cuda:0")
    t.fill_(1.0)
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()
    measure(ctx, d, s, "first buffers after torch 4 GiB", rows)
    measure(ctx, d2, s2, "fresh buffers after torch 4 GiB", rows)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)
    for b in (s, d, s2, d2):
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()
