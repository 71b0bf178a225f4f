#!/usr/bin/env python3
"""Per-kernel, per-grid-size summary of a rocprofv3 --kernel-trace CSV.

    python scripts/trace_summary.py <bench_kernel_trace.csv> [out.json]

rocprofv3's --stats averages every launch of a kernel symbol together; the
combine kernel runs at several sizes inside bench.py, so this splits the
launches by grid size to compare with bench.py's per-size HIP-event timing.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    groups = defaultdict(list)
    for r in rows:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        groups[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(dur)
    out = []
    for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": name, "grid_threads": grid, "calls": len(v),
                    "avg_us": round(statistics.mean(v), 3),
                    "median_us": round(statistics.median(v), 3),
                    "min_us": round(min(v), 3), "max_us": round(max(v), 3)})
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
