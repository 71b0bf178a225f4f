#!/bin/bash
# Occupancy cap of the multi-operand kernels: A/B through the product path
# (UCX_BUILTIN_DEV_MULTI_WAVES=0: no cap, unset: the measured table), two
# interleaved rounds, then the kernel sweep (tools/tune_occ) at 64 MiB and
# 256 MiB per operand.   usage: scripts/occ_ab.sh OUTDIR
set -u
OUT=$1; mkdir -p $OUT
for r in 1 2; do
  UCX_BUILTIN_DEV_MULTI_WAVES=0 timeout -k 10 200 python -u scripts/multi_probe.py $OUT/multi_nocap_$r.json > $OUT/multi_nocap_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u scripts/multi_probe.py $OUT/multi_table_$r.json > $OUT/multi_table_$r.log 2>&1 || exit 1
done
timeout -k 10 200 tools/tune_occ 24 5 > $OUT/occ_24.txt 2>&1 || exit 1
timeout -k 10 300 tools/tune_occ 26 3 > $OUT/occ_26.txt 2>&1 || exit 1
python3 - $OUT <<'PY'
import json, sys, glob
out = sys.argv[1]
rows = {}
for f in sorted(glob.glob(out + "/multi_*.json")):
    kind = "nocap" if "nocap" in f else "table"
    for r in json.load(open(f)):
        key = (r.get("kernel", "multi"), r["nsrc"], r["bytes_per_operand"] >> 20)
        rows.setdefault(key, {}).setdefault(kind, []).append(r["frac"])
for k, v in sorted(rows.items()):
    print(k, {kk: [round(x * 100, 1) for x in vv] for kk, vv in v.items()})
PY
cat $OUT/occ_24.txt $OUT/occ_26.txt
