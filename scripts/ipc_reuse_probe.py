import sys
sys.path.insert(0, "tests")
from _launch import launch
for world, scale in ((8, 64), (8, 64), (4, 64)):
    codes, outs = launch("_worker_ipc_reuse.py", world, args=(scale, 3), timeout=200,
                         env_extra={"LOCAL_RANK": "0"})
    print(f"=== world {world} scale {scale}: codes {codes}", flush=True)
    for r, o in enumerate(outs):
        lines = o.strip().splitlines()
        print("\n".join(f"[{r}] {l}" for l in lines[-12:]), flush=True)
