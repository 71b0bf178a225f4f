#!/usr/bin/env python3
"""Are HIP IPC handles of live allocations distinct, and what do they hold?
The engine's per-group mapping cache keys peers' buffers by handle bytes
(builtin_rma.c rma_import). Allocates 40 registered-size buffers (freeing
every third one as it goes, as ops come and go), exports each live one,
and reports duplicate handles among live allocations and the handle bytes
that vary.   python scripts/ipc_handles.py [out.json]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import xucg_amd  # noqa: E402
from xucg_amd import _lib  # noqa: E402

H = 96


def main():
    ctx = xucg_amd.DevContext(device=0)
    live = {}
    dups = 0
    for i in range(40):
        b = ctx.alloc(2056 + 4096 * (i % 3))
        key = (ctypes.c_uint8 * H)()
        st = _lib.dev().ucg_builtin_dev_ipc_export(ctx.handle, b.ptr, key)
        assert st == 0, _lib.last_error()
        kb = bytes(key)
        if kb in {v[1] for v in live.values()}:
            dups += 1
        live[i] = (b, kb)
        if i % 3 == 2:
            j = i - 1
            live.pop(j)[0].free()
    keys = [v[1] for v in live.values()]
    varying = [k for k in range(H) if len({kb[k] for kb in keys}) > 1]
    res = {"live": len(keys), "duplicate_handles_among_live": dups,
           "distinct": len(set(keys)), "varying_byte_offsets": varying,
           "first_handle_hex": keys[0].hex()}
    print(res)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)
    for b, _ in live.values():
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()
