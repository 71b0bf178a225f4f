#!/usr/bin/env python3
"""Does where the runtime places a buffer decide the slow combine? r02r: on a
fast box, a 256 MiB pair allocated after torch allocated and freed 4 GiB read
82.5-83 % of 8 TB/s while the pair allocated before read 85-86 %, in the same
process. This probe allocates fp32 pairs of bench.py's size
  - plain (hipMalloc) and contiguous (hipExtMallocWithFlags with
    hipDeviceMallocContiguous, UCX_BUILTIN_DEV_MALLOC=contiguous) on a fresh
    process,
  - both again after torch allocated and freed 4 GiB,
  - both again after 48 x 64 MiB allocations of which every other one was
    freed (a holed heap),
and times the combine and the two-stream read on every pair, in rotation, in
two rounds (HIP events, median of 5 batches of 50).

    python scripts/alloc_place.py [out.json]
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


def pair(ctx, kind, seed):
    os.environ["UCX_BUILTIN_DEV_MALLOC"] = kind
    s, d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    os.environ.pop("UCX_BUILTIN_DEV_MALLOC")
    ctx.fill("float32", "round", seed, s, N)
    ctx.fill("float32", "round", seed + 1, d, N)
    return s, d


def main():
    import torch
    ctx = xucg_amd.DevContext(device=0)
    pairs = {}
    pairs["fresh plain"] = pair(ctx, "default", 10)
    pairs["fresh contiguous"] = pair(ctx, "contiguous", 20)
    t = torch.empty(1 << 30, dtype=torch.float32, device="cuda:0")
    t.fill_(1.0)
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()
    pairs["after torch 4 GiB plain"] = pair(ctx, "default", 30)
    pairs["after torch 4 GiB contiguous"] = pair(ctx, "contiguous", 40)
    holes = [ctx.alloc(64 << 20) for _ in range(48)]
    for b in holes[::2]:
        b.free()
    pairs["holed heap plain"] = pair(ctx, "default", 50)
    pairs["holed heap contiguous"] = pair(ctx, "contiguous", 60)
    ctx.sync()
    rows = []
    for rnd in range(2):
        for name, (s, d) in pairs.items():
            cu = med5(lambda: ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 50))
            ru = med5(lambda: ctx.profile_stream(0, d.ptr, s.ptr, N * 4, 50))
            row = {"round": rnd, "pair": name,
                   "combine_frac": round(3 * N * 4 / (cu * 1e-6) / 1e9 / PEAK, 4),
                   "read2_gbs": round(2 * N * 4 / (ru * 1e-6) / 1e9, 1),
                   "src": hex(s.ptr), "dst": hex(d.ptr)}
            print(row, flush=True)
            rows.append(row)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)
    for s, d in pairs.values():
        s.free()
        d.free()
    for b in holes[1::2]:
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()
