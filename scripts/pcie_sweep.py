#!/usr/bin/env python3
"""H2D/D2H-inclusive combine (ucg_builtin_dev_combine_host, pinned host
operands) over staging-ring geometries: slot size x slot count, fp32 SUM of
2^26 elements (256 MiB). Also the raw pinned H2D and D2H copy rates of the
box for the bound: the pipeline moves 2N bytes H2D and N bytes D2H.

    python scripts/pcie_sweep.py [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

N = 1 << 26
GIB = float(1 << 30)


def copy_rate(ctx, dst, src, nbytes, reps=5):
    _lib.check(_lib.dev().ucg_builtin_dev_memcpy(ctx.handle, dst, src, nbytes), "memcpy")
    t = time.perf_counter()
    for _ in range(reps):
        _lib.check(_lib.dev().ucg_builtin_dev_memcpy(ctx.handle, dst, src, nbytes), "memcpy")
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    hs, hd = xucg_amd.HostBuffer(N * 4), xucg_amd.HostBuffer(N * 4)
    res = {"count": N, "dtype": "float32", "op": "sum", "rows": []}
    base = xucg_amd.DevContext(device=0)
    dbuf = base.alloc(N * 4)
    res["pinned_h2d_gbs"] = round(copy_rate(base, dbuf.ptr, hs.ptr, N * 4), 2)
    res["pinned_d2h_gbs"] = round(copy_rate(base, hd.ptr, dbuf.ptr, N * 4), 2)
    dbuf.free()
    base.close()
    for slot_mib in (2, 4, 8, 16, 32):
        for slots in (2, 4, 8):
            ctx = xucg_amd.DevContext(device=0, stage_bytes=slot_mib << 20, stage_slots=slots)
            rc = ctx.combine_host("sum", "float32", hd, hs, N)
            assert rc == 0, _lib.last_error()
            ts = []
            for _ in range(5):
                t = time.perf_counter()
                rc = ctx.combine_host("sum", "float32", hd, hs, N)
                ts.append(time.perf_counter() - t)
                assert rc == 0
            ctx.close()
            t = sorted(ts)[len(ts) // 2]
            row = {"slot_mib": slot_mib, "slots": slots, "ms": round(t * 1e3, 3),
                   "gibs_n": round(N * 4 / t / GIB, 2),
                   "h2d_gbs": round(2 * N * 4 / t / 1e9, 2)}
            res["rows"].append(row)
            print(json.dumps(row), flush=True)
    hs.free()
    hd.free()
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}))


if __name__ == "__main__":
    main()
