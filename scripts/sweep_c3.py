#!/usr/bin/env python3
"""BASELINE config 3 on one MI355X: every dtype x op of the device combine,
operand sizes 1 KiB .. 1 GiB (x4 steps), device-resident, plus the
H2D/D2H-inclusive rate (pinned host buffers) and the 1-thread CPU oracle at
64 MiB per dtype.

    python scripts/sweep_c3.py [out.json]

Kernel time = HIP events around back-to-back launches on the context stream
(ucg_builtin_dev_profile_reduce). GB/s on the algorithmic basis of
3 x operand bytes per combine; fraction of 8 TB/s for sizes >= 256 MiB only
(smaller working sets can sit in the 256 MiB Infinity Cache)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

PEAK = 8000.0
SIZES = [1 << k for k in range(10, 31, 2)]          # 1 KiB .. 1 GiB per operand


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    ctx = xucg_amd.DevContext(device=0)
    maxb = SIZES[-1]
    # both operands in one allocation, the bench's layout (separately allocated
    # pairs can alias in HBM's channel/bank hash)
    pair = ctx.alloc(2 * maxb)
    src, dst = pair.ptr, pair.ptr + maxb
    res = {"sizes_bytes": SIZES, "device": [], "host_pipeline": [], "cpu_oracle_64mib": []}
    t_start = time.time()
    for dt in _lib.DTYPES:
        sz = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
        ctx.fill(dt, "round", 1, src, maxb // sz)
        ctx.fill(dt, "round", 2, dst, maxb // sz)
        ctx.sync()
        for op in _lib.OPS:
            if not xucg_amd.is_supported(dt, op):
                continue
            row = {"dtype": dt, "op": op, "us": [], "gbs": []}
            for b in SIZES:
                n = b // sz
                iters = max(5, min(200, (64 << 20) // b * 5))
                ctx.profile_reduce(op, dt, dst, src, n, 2)
                us = ctx.profile_reduce(op, dt, dst, src, n, iters)
                row["us"].append(round(us, 3))
                row["gbs"].append(round(3 * b / (us * 1e-6) / 1e9, 1))
            row["frac_1gib"] = round(row["gbs"][-1] / PEAK, 4)
            row["frac_256mib"] = round(row["gbs"][-2] / PEAK, 4)
            # src one element out of dst's 16-B phase (8 B for 16-B-phase
            # dtypes would be the same kernel): the realigning kernel
            if sz < 16:
                n = (256 << 20) // sz - 1
                ctx.profile_reduce(op, dt, dst, src + sz, n, 2)
                us = ctx.profile_reduce(op, dt, dst, src + sz, n, 20)
                row["shifted_256mib_frac"] = round(3 * n * sz / (us * 1e-6) / 1e9 / PEAK, 4)
            res["device"].append(row)
            print(f"{dt:9s} {op:5s} 1KiB {row['us'][0]:7.2f} us  256MiB "
                  f"{row['gbs'][-2]:7.0f} GB/s  1GiB {row['gbs'][-1]:7.0f} GB/s "
                  f"({100 * row['frac_1gib']:.1f}%)", flush=True)
    pair.free()

    # H2D/D2H-inclusive: host-resident (pinned) operands, pipelined
    for dt in ("int32", "int64", "float16", "float32", "float64"):
        sz = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
        for b in (1 << 20, 64 << 20, 1 << 30):
            hs, hd = xucg_amd.HostBuffer(b), xucg_amd.HostBuffer(b)
            n = b // sz
            assert ctx.combine_host("sum", dt, hd, hs, n) == 0, _lib.last_error()
            reps = 3 if b >= (1 << 30) else 10
            t0 = time.perf_counter()
            for _ in range(reps):
                assert ctx.combine_host("sum", dt, hd, hs, n) == 0
            t = (time.perf_counter() - t0) / reps
            res["host_pipeline"].append({"dtype": dt, "op": "sum", "bytes": b,
                                         "ms": round(t * 1e3, 3),
                                         "gibs_n": round(b / t / 2**30, 2),
                                         "gibs_3n": round(3 * b / t / 2**30, 2)})
            hs.free()
            hd.free()
        print(f"host pipeline {dt}: {res['host_pipeline'][-1]}", flush=True)

    # CPU oracle, 1 thread, 64 MiB per operand, SUM
    from oracle import oracle as O
    os.environ.setdefault("UCG_ORACLE_LIB", O.build_native())
    O.LIB_PATH = os.environ["UCG_ORACLE_LIB"]
    O._lib = None
    for dt in _lib.DTYPES:
        sz = _lib.DTYPE_SIZE[_lib.dt_index(dt)]
        n = (64 << 20) // sz
        s = O.fill(dt, "round", 1, n)
        d = O.fill(dt, "round", 2, n)
        _, med = O.time_reduce("sum", dt, s, d, reps=5)
        res["cpu_oracle_64mib"].append({"dtype": dt, "op": "sum",
                                        "gibs_3n": round(3 * n * sz / med / 2**30, 2)})
    res["wall_s"] = round(time.time() - t_start, 1)
    ctx.close()
    text = json.dumps(res)
    if out_path:
        with open(out_path, "w") as f:
            f.write(text + "\n")
    print("done", res["wall_s"], "s")


if __name__ == "__main__":
    main()
