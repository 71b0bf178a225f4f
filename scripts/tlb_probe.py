#!/usr/bin/env python3
"""Why does a 256 MiB pair allocated after a large allocation was freed run
slower (r02r, r02s: 82-83 % of 8 TB/s against 85-86 % for the process's first
pair)? Pair A is the first allocation of the process; then 4 GiB are
allocated, written and freed, and pair B is allocated. Both are timed (HIP
events, median of 5 batches of 50), then each is launched 10 times on its
own, A with N elements and B with N - 64 so that a kernel trace or a PMC pass
tells them apart by grid size (run it under rocprofv3 --pmc with the
TCP_UTCL1_* translation counters to see whether B misses the TLB more).

    python scripts/tlb_probe.py [out.json | pmc]     (pmc: no timing loops)
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


def main():
    ctx = xucg_amd.DevContext(device=0)
    a_s, a_d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    big = ctx.alloc(4 << 30)
    ctx.fill("uint8", "round", 7, big, 4 << 30)
    ctx.sync()
    big.free()
    b_s, b_d = ctx.alloc(N * 4), ctx.alloc(N * 4)
    for i, buf in enumerate((a_s, a_d, b_s, b_d)):
        ctx.fill("float32", "round", 70 + i, buf, N)
    ctx.sync()
    rows = []
    pmc = sys.argv[1:] == ["pmc"]
    for rnd in range(0 if pmc else 2):
        for name, s, d in (("A first", a_s, a_d), ("B after 4 GiB freed", b_s, b_d)):
            cu = med5(lambda: ctx.profile_reduce("sum", "float32", d.ptr, s.ptr, N, 50))
            ru = med5(lambda: ctx.profile_stream(0, d.ptr, s.ptr, N * 4, 50))
            row = {"round": rnd, "pair": name,
                   "combine_frac": round(3 * N * 4 / (cu * 1e-6) / 1e9 / PEAK, 4),
                   "read2_gbs": round(2 * N * 4 / (ru * 1e-6) / 1e9, 1)}
            print(row, flush=True)
            rows.append(row)
    for _ in range(10):
        ctx.reduce_checked("sum", "float32", a_d, a_s, N)
    ctx.sync()
    for _ in range(10):
        ctx.reduce_checked("sum", "float32", b_d, b_s, N - 64)
    ctx.sync()
    if len(sys.argv) > 1 and not pmc:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)
    for buf in (a_s, a_d, b_s, b_d):
        buf.free()
    ctx.close()


if __name__ == "__main__":
    main()
