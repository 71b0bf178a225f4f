#!/usr/bin/env python3
"""Summary of scripts/occ_pmc.sh: for the uncapped and the capped launches
(tune_occ's PMC mode alternates them: k_reduce_multi dispatch 0, 2, 4, ...
uncapped, 1, 3, 5, ... at most 8 waves per CU; the counters' LDS column shows
static LDS only) the median over dispatches of HBM bytes per launch
(FETCH_SIZE doubled per MI355X_MICROARCH.md, WRITE_SIZE), the waves resident
(SQ_WAVE_CYCLES / SQ_BUSY_CYCLES, whole chip) and the kernel time from the
trace.   python scripts/occ_pmc_summary.py OUTDIR [out.json]"""
import csv
import json
import statistics
import sys
from collections import defaultdict

base = sys.argv[1].rstrip("/") + "/"
N, S = 8, 64 << 20
KIND = ("uncapped", "cap8")
rows = defaultdict(lambda: defaultdict(list))
for f in ("pmc_FETCH_SIZE", "pmc_WRITE_SIZE", "pmc_SQ_WAVES"):
    order = {}
    for r in csv.DictReader(open(base + f + "/o_counter_collection.csv")):
        if "k_reduce_multi" not in r["Kernel_Name"]:
            continue
        k = order.setdefault(r["Dispatch_Id"], len(order)) % 2
        rows[KIND[k]][r["Counter_Name"]].append(float(r["Counter_Value"]))
trace = defaultdict(list)
i = 0
for r in csv.DictReader(open(base + "trace/o_kernel_trace.csv")):
    if "k_reduce_multi" in r["Kernel_Name"]:
        trace[KIND[i % 2]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        i += 1
out = {}
for lds, c in rows.items():
    med = {k: statistics.median(v) for k, v in c.items()}
    fetch = med.get("FETCH_SIZE", 0) * 1024 * 2          # KB, x2 on gfx950
    write = med.get("WRITE_SIZE", 0) * 1024
    us = statistics.median(trace[lds]) if trace.get(lds) else None
    out[lds] = {
        "dispatches": len(c.get("SQ_WAVES", [])),
        "fetch_bytes_x2": fetch, "write_bytes": write,
        "traffic_over_algorithmic": round((fetch + write) / ((N + 1) * S), 5),
        # waves resident, in the counters' own units (their ratio between the
        # two launch kinds is what the cap changes: 32 -> 8 waves per CU)
        "sq_wave_cycles_per_busy_cycle": round(med["SQ_WAVE_CYCLES"] / med["SQ_BUSY_CYCLES"], 1)
        if med.get("SQ_BUSY_CYCLES") else None,
        "trace_median_us": us,
        "frac_of_8tbs": round((N + 1) * S / (us * 1e-6) / 8e12, 4) if us else None}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
