#!/usr/bin/env python3
"""Roofline of the combine when src and dst disagree mod 16 B: the shuffle
kernel (k_reduce_shift, product) against the element loop it replaced
(k_reduce_scalar, UCX_BUILTIN_DEV_VARIANT=4) and the aligned kernel, 256 MiB
(SHIFT_PROBE_BYTES), then the 8-operand one-shot and tree fan-in kernels with
operands in and out of dst's phase, 64 MiB
per operand, 3N algorithmic bytes, HIP events on the context stream (20 warm
launches, median of 5 batches of 20). Run once per variant:

    python scripts/shift_probe.py out.json          # product dispatch
    UCX_BUILTIN_DEV_VARIANT=4 python scripts/shift_probe.py out.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

PEAK = 8000.0
CASES = [("float32", 0), ("float32", 4), ("float32", 8), ("float32", 12),
         ("float64", 8), ("float16", 2), ("float16", 6), ("int8", 1), ("int8", 7)]
SIZE = {"float32": 4, "float64": 8, "float16": 2, "int8": 1}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    variant = os.environ.get("UCX_BUILTIN_DEV_VARIANT", "0")
    ctx = xucg_amd.DevContext(device=0)
    nbytes = int(os.environ.get("SHIFT_PROBE_BYTES", 256 << 20))
    bs, bd = ctx.alloc(nbytes + 64), ctx.alloc(nbytes + 64)
    rows = []
    for dt, shift in CASES:
        n = nbytes // SIZE[dt]
        ctx.fill(dt, "round", 1, bs, n + 8)
        ctx.fill(dt, "round", 2, bd, n)
        sp = bs.ptr + shift
        ctx.profile_reduce("sum", dt, bd, sp, n, 20)
        b = sorted(ctx.profile_reduce("sum", dt, bd, sp, n, 20) for _ in range(5))
        us = b[2]
        gbs = 3 * nbytes / (us * 1e-6) / 1e9
        row = {"dtype": dt, "src_shift_bytes": shift, "variant": variant,
               "us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
        print(row, flush=True)
        rows.append(row)
    # the one-shot multi-operand kernel, 8 operands of 64 MiB: all in phase
    # with dst, one operand 4 B out, every operand at its own phase
    n8 = (64 << 20) // 4
    bufs = [ctx.alloc(n8 * 4 + 64) for _ in range(8)]
    out8 = ctx.alloc(n8 * 4 + 64)
    for k, b in enumerate(bufs):
        ctx.fill("float32", "exact", 100 + k, b, n8 + 16)
    for name, offs in (("aligned", [0] * 8), ("one_operand_4B", [4] + [0] * 7),
                       ("all_phases", [0, 4, 8, 12, 4, 8, 12, 0]),
                       ("in_phase_off_line_16B", [16] * 8)):
        srcs = [b.ptr + o for b, o in zip(bufs, offs)]
        for kernel in ("reduce_multi", "reduce_tree"):
            if kernel == "reduce_multi":
                def call():
                    return ctx.reduce_multi("sum", "float32", out8.ptr, srcs, 0, n8)
            else:
                def call():
                    return ctx.reduce_tree("sum", "float32", out8.ptr, srcs, n8)
            assert call() == 0, _lib.last_error()
            ctx.sync()
            import time
            reps = 20
            t = []
            for _ in range(5):
                t0 = time.perf_counter()
                for _ in range(reps):
                    call()
                ctx.sync()
                t.append((time.perf_counter() - t0) / reps * 1e6)
            us = sorted(t)[2]
            gbs = 9 * n8 * 4 / (us * 1e-6) / 1e9
            row = {"kernel": kernel, "nsrc": 8, "case": name, "variant": variant,
                   "us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
            print(row, flush=True)
            rows.append(row)
    for b in bufs + [out8]:
        b.free()
    # spot parity on a small misaligned case vs a host restatement of fp32 sum
    m = 100_003
    a = np.random.default_rng(5).standard_normal(m).astype(np.float32)
    c = np.random.default_rng(6).standard_normal(m).astype(np.float32)
    bs.upload(a, 4)
    bd.upload(c, 0)
    assert ctx.reduce("sum", "float32", bd.ptr, bs.ptr + 4, m) == 0, _lib.last_error()
    ctx.sync()
    assert (bd.download(np.float32, m).view(np.uint32) == (a + c).view(np.uint32)).all()
    ctx.close()
    if out:
        old = []
        if os.path.exists(out):
            with open(out) as f:
                old = json.load(f)
        with open(out, "w") as f:
            json.dump(old + rows, f, indent=1)


if __name__ == "__main__":
    main()
