#!/usr/bin/env python3
"""Which HIP runtime serves the process, and the headline kernel's time under
it. Run once with torch imported first (PyTorch's bundled libamdhip64) and
once with XUCG_NO_TORCH_PRELOAD=1 and no torch (/opt/rocm's).

    python scripts/runtime_probe.py [torch|plain]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
if mode == "torch":
    import torch  # noqa: F401
import xucg_amd  # noqa: E402

N = 1 << 26
ctx = xucg_amd.DevContext(device=0)
src, dst = ctx.alloc(N * 4), ctx.alloc(N * 4)
ctx.fill("float32", "round", 1, src, N)
ctx.fill("float32", "round", 2, dst, N)
ctx.sync()
us = [ctx.profile_reduce("sum", "float32", dst, src, N, 50) for _ in range(5)]
libs = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})
print(mode, "min_us %.2f" % min(us), "frac %.4f" % (3 * N * 4 / (min(us) * 1e-6) / 8e12),
      libs, flush=True)
