#!/usr/bin/env python3
"""Single-GPU roofline of the one-shot multi-operand combine
(ucg_builtin_dev_reduce_multi): N local operands of S bytes, one output,
(N + 1) x S algorithmic bytes per launch. On one GPU every operand is local
HBM, so this isolates the kernel's own efficiency from xGMI.

    python scripts/multi_probe.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import xucg_amd  # noqa: E402

PEAK = 8000.0


def main():
    ctx = xucg_amd.DevContext.on_torch_stream(0)
    res = []
    for per_op in (64 << 20, 256 << 20):
        n = per_op // 4
        for nsrc in (2, 4, 8, 16):
            srcs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(nsrc)]
            for r, s in enumerate(srcs):
                ctx.fill("float32", "exact", 100 + r, s, n)
            out = torch.empty(n, dtype=torch.float32, device="cuda")
            for _ in range(3):
                rc = ctx.reduce_multi("sum", "float32", out, srcs, 0, n)
                assert rc == 0, (rc, xucg_amd._lib.last_error())
            torch.cuda.synchronize()
            want = torch.stack(srcs).sum(0)      # exact inputs: any order is exact
            assert torch.equal(out, want), "multi-operand combine mismatch"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            iters = 20
            e0.record()
            for _ in range(iters):
                ctx.reduce_multi("sum", "float32", out, srcs, 0, n)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            gbs = (nsrc + 1) * per_op / (us * 1e-6) / 1e9
            row = {"nsrc": nsrc, "bytes_per_operand": per_op, "us": round(us, 2),
                   "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
            print(row, flush=True)
            res.append(row)
            del srcs, out
            torch.cuda.empty_cache()
    # the tree fan-in (groups that are not a power of two), 64 MiB operands
    n = (64 << 20) // 4
    for nsrc in (3, 6, 8, 12):
        srcs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(nsrc)]
        for r, s in enumerate(srcs):
            ctx.fill("float32", "exact", 200 + r, s, n)
        out = torch.empty(n, dtype=torch.float32, device="cuda")
        for _ in range(3):
            rc = ctx.reduce_tree("sum", "float32", out, srcs, n)
            assert rc == 0, (rc, xucg_amd._lib.last_error())
        torch.cuda.synchronize()
        assert torch.equal(out, torch.stack(srcs).sum(0)), "tree combine mismatch"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ctx.reduce_tree("sum", "float32", out, srcs, n)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        gbs = (nsrc + 1) * n * 4 / (us * 1e-6) / 1e9
        row = {"kernel": "reduce_tree", "nsrc": nsrc, "bytes_per_operand": n * 4,
               "us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
        print(row, flush=True)
        res.append(row)
        del srcs, out
        torch.cuda.empty_cache()
    ctx.close()
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
