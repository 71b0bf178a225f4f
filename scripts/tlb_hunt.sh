#!/bin/bash
# timing of the first pair vs a pair allocated after 4 GiB were freed, then
# one PMC pass of TLB (UTCL1) counters and one of HBM fetch over the same
# launches; usage: scripts/tlb_hunt.sh TAG
set -u
OUT=$PWD/gpurun_out/$1; mkdir -p $OUT
ROOT=$PWD
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/tlb_probe.py $OUT/tlb_probe.json > $OUT/tlb_probe.log 2>&1 || exit $?
grep pair $OUT/tlb_probe.log
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum \
    --output-format csv -d $OUT/pmc_tlb -o tlb -- python3 $ROOT/scripts/tlb_probe.py pmc > $OUT/pmc_tlb.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 $ROOT/scripts/tlb_probe.py pmc > $OUT/pmc_fetch.log 2>&1 || exit $?
cd $ROOT
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
out = sys.argv[1]
for f in glob.glob(out + "/pmc_*/**/*counter_collection.csv", recursive=True):
    agg = {}
    for r in csv.DictReader(open(f)):
        if "k_reduce" not in r["Kernel_Name"]:
            continue
        agg.setdefault((r["Grid_Size"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for k in sorted(agg):
        print(f.split("/")[-1], k, len(agg[k]), statistics.median(agg[k]))
PY
