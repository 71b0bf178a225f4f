"""Is the stall of the 5-member workers set off by
the parent's pageable copies? The parent copies a 16 MiB pageable numpy array
to the device and back, then either keeps the array (mode kept) or frees it
(mode freed: pages the runtime may have pinned for the copy go back to the
allocator), then times the worker group as parent_probe.py does.
   usage: parent_probe2.py kept|freed"""
import gc
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _launch import launch  # noqa: E402
import xucg_amd  # noqa: E402

os.environ.setdefault("UCX_BUILTIN_WAIT_TIMEOUT", "90")
mode = sys.argv[1]
spec = "5:1:0:2:2:16"


def group(tag):
    t0 = time.time()
    codes, outs = launch("_worker_topo.py", 5, args=(f"probe2_{os.getpid()}_{tag}", "rma", 256,
                                                     spec), timeout=60)
    slow = [l for o in outs for l in o.splitlines() if "ucg slow" in l]
    print(f"{mode} {tag}: {time.time() - t0:.1f} s codes {codes} slow notes {len(slow)}",
          flush=True)


ctx = xucg_amd.DevContext(device=0)
keep = []
for k in range(4):
    a = np.random.default_rng(k).random(2 << 20)          # 16 MiB, pageable
    b = ctx.alloc(a.nbytes)
    b.upload(a)
    back = b.download(a.dtype, a.size)
    assert (back == a).all()
    b.free()
    if mode == "kept":
        keep.append(a)
    del a, back
gc.collect()
ctx.close()
group("after-copies")
group("again")
