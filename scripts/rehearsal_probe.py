"""Run bench.py's collective phases as a 1-GPU rehearsal (gloo, see
bench.HostStagedDist) with `world` ranks, a given phase list and repetitions;
print each run's failures. usage: python scripts/rehearsal_probe.py WORLD
REPS [PHASES]"""
import json
import os
import sys
import tempfile
import uuid

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from _launch import launch  # noqa: E402
import bench  # noqa: E402

world, reps = int(sys.argv[1]), int(sys.argv[2])
phases = sys.argv[3] if len(sys.argv) > 3 else ""
for rep in range(reps):
    out = os.path.join(tempfile.gettempdir(), f"xucg_rp_{uuid.uuid4().hex}.json")
    codes, outs = launch("../bench.py", world, args=("--collective-child",), timeout=200,
                         env_extra={"LOCAL_RANK": "0", "XUCG_COLLECTIVE_BACKEND": "gloo",
                                    "XUCG_COLLECTIVE_SCALE": "64", "XUCG_COLLECTIVE_OUT": out,
                                    "XUCG_COLLECTIVE_PHASES": phases})
    res = json.load(open(out)) if os.path.exists(out) else {}
    fails = bench.collective_failures(res)
    print(f"world {world} phases {phases or 'all'} rep {rep}: codes {codes} failures {fails}",
          flush=True)
    if any(c != 0 for c in codes):
        print("\n".join(o[-1500:] for o in outs), flush=True)
        sys.exit(1)
