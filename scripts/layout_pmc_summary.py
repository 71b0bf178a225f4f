#!/usr/bin/env python3
"""Per-layout medians of the counters of scripts/layout_pmc.sh: the first
`reps` headline-kernel dispatches are the joint layout, the next `reps` the
separate one (scripts/layout_pmc.py). FETCH_SIZE is doubled and both sizes
converted from KB (MI355X_MICROARCH.md, HBM / rocprofv3).

    python scripts/layout_pmc_summary.py OUTDIR REPS
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "ucgdev::k_reduce<float, 0, 1, 1, 64, 1, "   # PF form, any prefetch depth
GRID = (1 << 26) // 4


def per_dispatch(d):
    """{counter: [value per headline dispatch, in dispatch order]}"""
    rows = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KERNEL in r["Kernel_Name"] and int(r["Grid_Size"]) == GRID:
                rows.setdefault(r["Counter_Name"], []).append(
                    (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {k: [v for _, v in sorted(x)] for k, x in rows.items()}


def main():
    out_dir, reps = sys.argv[1], int(sys.argv[2])
    res = {"kernel": KERNEL, "reps_per_layout": reps, "joint": {}, "separate": {}}
    for name in ("utcl1", "fetch", "write", "utcl2"):
        for counter, vals in per_dispatch(os.path.join(out_dir, name)).items():
            if len(vals) < 2 * reps:
                res.setdefault("short", []).append(f"{counter}: {len(vals)} dispatches")
                continue
            for layout, sl in (("joint", vals[:reps]), ("separate", vals[reps:2 * reps])):
                v = statistics.median(sl)
                if counter == "FETCH_SIZE":
                    res[layout]["hbm_read_bytes"] = int(2 * v * 1024)
                elif counter == "WRITE_SIZE":
                    res[layout]["hbm_write_bytes"] = int(v * 1024)
                else:
                    res[layout][counter] = v
    for layout in ("joint", "separate"):
        for name in ("utcl1", "fetch"):
            p = os.path.join(out_dir, f"{name}.out")
            if os.path.exists(p):
                for line in open(p):
                    if line.startswith("{"):
                        res[layout]["timing_" + name] = json.loads(line)[layout]
        m, h = res[layout].get("TCP_UTCL1_TRANSLATION_MISS_sum"), \
            res[layout].get("TCP_UTCL1_TRANSLATION_HIT_sum")
        if m is not None and h:
            res[layout]["utcl1_miss_rate"] = round(m / (m + h), 6)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
