"""Does initialising the GPU change this process's CPU affinity (which the
test workers it spawns would inherit)? Prints the allowed-CPU count before
and after a device context, and what a child started afterwards sees."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
print("before", len(os.sched_getaffinity(0)), flush=True)
import xucg_amd  # noqa: E402
ctx = xucg_amd.DevContext(device=0)
print("after DevContext", len(os.sched_getaffinity(0)), flush=True)
ctx.close()
print("after close", len(os.sched_getaffinity(0)), flush=True)
out = subprocess.run([sys.executable, "-c", "import os; print(len(os.sched_getaffinity(0)))"],
                     capture_output=True, text=True).stdout.strip()
print("child", out, flush=True)
with open("/proc/self/status") as f:
    print([l.strip() for l in f if l.startswith("Cpus_allowed_list")])
