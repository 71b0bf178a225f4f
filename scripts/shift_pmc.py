#!/usr/bin/env python3
"""The realigning multi-operand kernels under rocprofv3 counter passes
(VERDICT r03 #7): N = 8 fp32 operands of 64 MiB, each in its own allocation
and 4 B out of dst's 16-B phase, through the product entry points:
  k_reduce_multi_shift   ucg_builtin_dev_reduce_multi   (N + 1) x S bytes
  k_reduce_tree_shift    ucg_builtin_dev_reduce_tree    (n + 1) x S bytes
  k_gather_multi         ucg_builtin_dev_gather_multi   2 N x S bytes
and, for reference, the in-phase k_reduce_multi (capped). Each form runs
`reps` times after one warm launch; prints the wall-clock time per launch and
the sampled exactness of the first two (exact inputs). Kernel names tell the
forms apart in the CSVs (scripts/pmc_kernels.py).

    rocprofv3 --pmc FETCH_SIZE -- python3 scripts/shift_pmc.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import xucg_amd
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    N, n = 8, (64 << 20) // 4
    S = n * 4
    ctx = xucg_amd.DevContext(device=0)
    bufs = [ctx.alloc(S + 4096) for _ in range(N)]
    dst = ctx.alloc(N * S + 4096)
    shifted = [b.ptr + 4 for b in bufs]          # 4 B out of phase with dst
    aligned = [b.ptr for b in bufs]
    for m, p in enumerate(shifted):
        ctx.fill("float32", "exact", 300 + m, p, n)
    ctx.sync()

    def timed(fn):
        fn()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        ctx.sync()
        return (time.perf_counter() - t0) / reps * 1e6

    forms = {
        "k_reduce_multi_shift": (lambda: ctx.reduce_multi("sum", "float32", dst.ptr, shifted,
                                                          0, n), (N + 1) * S),
        "k_reduce_tree_shift": (lambda: ctx.reduce_tree("sum", "float32", dst.ptr, shifted, n),
                                (N + 1) * S),
        "k_gather_multi (out of phase)": (lambda: ctx.gather_multi(dst.ptr, shifted, S),
                                          2 * N * S),
        "k_reduce_multi (in phase, capped)": (lambda: ctx.reduce_multi(
            "sum", "float32", dst.ptr, aligned, 0, n), (N + 1) * S),
    }
    out = {}
    w = 1 << 16
    for name, (fn, alg) in forms.items():
        us = timed(fn)
        out[name] = {"us": round(us, 2), "algorithmic_bytes": alg,
                     "frac_of_8tbs": round(alg / (us * 1e-6) / 8e12, 4)}
        if "shift" in name:
            lo = n // 2
            want = sum(np.asarray(bufs[m].download(np.float32, w, 4 + lo * 4),
                                  np.float64) for m in range(N))
            got = dst.download(np.float32, w, lo * 4).astype(np.float64)
            out[name]["sampled_exact"] = bool(np.array_equal(got, want))
    print(json.dumps(out), flush=True)
    for b in bufs:
        b.free()
    dst.free()
    ctx.close()


if __name__ == "__main__":
    main()
