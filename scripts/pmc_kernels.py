"""Average of every PMC counter per kernel name over the counter-collection
CSVs rocprofv3 wrote under OUTDIR/pmc_*/ (scripts/multi_pmc.sh).

    python3 scripts/pmc_kernels.py OUTDIR [--json OUT.json]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    out = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(out, "pmc_*", "**", "*counter_collection.csv"),
                       recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?")
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for name, cs in sorted(acc.items()):
        res[name] = {c: sum(v) / len(v) for c, v in cs.items()}
        short = name if len(name) < 90 else name[:87] + "..."
        print(short)
        for c, v in sorted(res[name].items()):
            print(f"    {c:24s} {v:16.1f}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
