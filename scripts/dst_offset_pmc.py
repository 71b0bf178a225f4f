#!/usr/bin/env python3
"""Per-case kernel time and HBM bytes of scripts/dst_offset_probe.py from a
rocprofv3 kernel trace and the FETCH_SIZE / WRITE_SIZE passes of the same
script (each case is 120 consecutive combine launches, in CASES order).
FETCH_SIZE is doubled and both counters are in KiB, as in pmc_summary.py
(MI355X_MICROARCH.md, HBM / rocprofv3).

    python scripts/dst_offset_pmc.py <trace.csv> <fetch.csv> <write.csv> [out.json]
"""
import csv
import json
import statistics
import sys

CASES = [(0, 0), (16, 16), (32, 32), (64, 64), (112, 112), (4, 4), (68, 68),
         (0, 4), (16, 4), (64, 68), (4, 0), (0, 16), (0, 64), (64, 0), (48, 0)]
PER_CASE = 120
ALG = 3 * (256 << 20)


def rows(path, counter=None):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "k_fill" in r["Kernel_Name"]:
                continue
            if counter and r["Counter_Name"] != counter:
                continue
            out.append(r)
    out.sort(key=lambda r: int(r["Dispatch_Id"]))
    return out


def main():
    tr, fe, wr = rows(sys.argv[1]), rows(sys.argv[2], "FETCH_SIZE"), rows(sys.argv[3], "WRITE_SIZE")
    assert len(tr) == len(fe) == len(wr) == PER_CASE * len(CASES), (len(tr), len(fe), len(wr))
    res = []
    for k, (d, s) in enumerate(CASES):
        sl = slice(k * PER_CASE, (k + 1) * PER_CASE)
        us = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                               for r in tr[sl])
        fb = 2 * 1024 * statistics.median(float(r["Counter_Value"]) for r in fe[sl])
        wb = 1024 * statistics.median(float(r["Counter_Value"]) for r in wr[sl])
        res.append({"dst_offset": d, "src_offset": s, "kernel": tr[sl][0]["Kernel_Name"][:80],
                    "trace_median_us": round(us, 2),
                    "frac_of_8tbs": round(ALG / (us * 1e-6) / 8e12, 4),
                    "hbm_bytes_per_launch": int(fb + wb),
                    "ratio_to_algorithmic": round((fb + wb) / ALG, 5)})
        print(res[-1])
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
