#!/bin/bash
# Is the slow combine per process or per box phase? Alternate processes:
# proc_probe, bench (headline only), slow_probe, bench, proc_probe.
# usage: scripts/proc_hunt.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
frac() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print('bench', r['frac'], r['measured_ceiling_same_box']['read_only_gbs'])" $1; }
timeout -k 10 120 python -u scripts/proc_probe.py $OUT/proc1.json > $OUT/proc1.log 2>&1 || exit $?
grep stage $OUT/proc1.log
timeout -k 10 180 python bench.py --no-extra --no-cpu-baseline > $OUT/bench1.json 2> $OUT/bench1.err || exit $?
frac $OUT/bench1.json
timeout -k 10 120 python -u scripts/slow_probe.py $OUT/slow.json > $OUT/slow.log 2>&1 || exit $?
grep "separate" $OUT/slow.log
timeout -k 10 180 python bench.py --no-extra --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit $?
frac $OUT/bench2.json
timeout -k 10 120 python -u scripts/proc_probe.py $OUT/proc2.json > $OUT/proc2.log 2>&1 || exit $?
grep stage $OUT/proc2.log
