#!/usr/bin/env python3
"""tools/va_reuse_probe's multi-process mode: NP
processes on the one GPU recycle hipMalloc buffers at the same address every
round, upload by DMA, and read each other's buffers through hipIpc imports
(tools/src/va_reuse_probe.hip). This parent never touches the GPU.

    python scripts/va_reuse_ipc.py OUTDIR [NP=12] [ITERS=200] [MiB=6] [mode ...]
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "va_reuse_probe")


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/va_ipc"
    np_ = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    iters = sys.argv[3] if len(sys.argv) > 3 else "200"
    mib = sys.argv[4] if len(sys.argv) > 4 else "6"
    modes = sys.argv[5:] or ["close", "hold"]
    os.makedirs(out_dir, exist_ok=True)
    rc = 0
    for mode in modes:
        d = tempfile.mkdtemp(prefix="xucg_vaipc_")
        try:
            procs = [subprocess.Popen([EXE, "ipc", d, str(r), str(np_), iters, mib, mode],
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                     for r in range(np_)]
            ranks = []
            for r, p in enumerate(procs):
                try:
                    out, _ = p.communicate(timeout=240)
                except subprocess.TimeoutExpired:
                    p.kill()
                    out = p.communicate()[0] + " <killed: timeout>"
                js = [ln for ln in out.splitlines() if ln.startswith("{")]
                try:
                    ranks.append(json.loads(js[-1]))
                except (ValueError, IndexError):
                    ranks.append({"rank": r, "exit": p.returncode, "tail": out[-400:]})
                    rc = 1
            # handles of different members in one round with equal bytes
            # (a handle naming (address, size) alone would collide between
            # processes whose allocations sit at the same address)
            same_bytes = rounds_with_same = 0
            for i in range(int(iters)):
                seen = {}
                for r in range(np_):
                    try:
                        with open(os.path.join(d, f"key_{r}_{i}"), "rb") as f:
                            b = f.read()
                    except OSError:
                        continue
                    if b.strip(b"\0"):
                        seen.setdefault(b, []).append(r)
                dups = [v for v in seen.values() if len(v) > 1]
                same_bytes += sum(len(v) for v in dups)
                rounds_with_same += bool(dups)
            handle_bytes = {"members_sharing_handle_bytes": same_bytes,
                            "rounds_with_shared_handle_bytes": rounds_with_same}
        finally:
            shutil.rmtree(d, ignore_errors=True)
        tot = {k: sum(x.get(k, 0) for x in ranks)
               for k in ("rounds", "same_va", "own_kernel_bad", "own_dma_bad", "peer_kernel_bad",
                         "peer_dma_bad", "bad_words", "zero_words", "export_fail",
                         "import_fail", "peer_checked", "dup_ptr", "bad_and_dup")}
        res = {"mode": mode, "np": np_, "iters": int(iters), "mib": int(mib), "total": tot,
               "handles": handle_bytes, "ranks": ranks}
        with open(os.path.join(out_dir, "va_reuse_ipc.jsonl"), "a") as f:
            f.write(json.dumps(res) + "\n")
        print(f"{mode}: {tot} {handle_bytes}", flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
