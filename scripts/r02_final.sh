#!/bin/bash
# Round-2 evidence on the final library, in one GPU session: clock probe,
# the GPU suite, smoke(), the driver's bench command and the default one,
# rocprofv3 kernel trace + FETCH/WRITE PMC passes of the bench, the engine on
# device buffers, and the IPC staleness probe.   usage: scripts/r02_final.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
step() { echo "== $1 $(date +%T)" | tee -a $OUT/steps.log; }
step clock
timeout -k 5 60 python -u scripts/clock_probe.py 15 $OUT/clock_probe.json > $OUT/clock.log 2>&1 || exit $?
tail -1 $OUT/clock.log
step pytest
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 250 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
step bench_driver
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit $?
step bench_default
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "
import json
for f in ('bench_driver','bench'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(f, d['value'], r['frac'], r['kernel_avg_us'], r['measured_ceiling_same_box']['read_only_gbs'], (d.get('extra') or {}).get('north_star_1gib_fp32_sum',{}).get('frac_of_8tbs'))"
step profile
bash scripts/profile_round.sh $TAG > $OUT/profile_steps.log 2>&1 || { tail -5 $OUT/profile_steps.log; exit 1; }
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" | sort | tail -n 1)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" | sort | tail -n 1)
python3 scripts/pmc_summary.py "$F" "$W" $OUT/pmc_traffic.json > $OUT/pmc_summary.txt 2>&1
tail -2 $OUT/pmc_summary.txt
step engine_devbuf
bash scripts/engine_devbuf.sh $TAG > /dev/null || exit $?
cut -c1-160 $OUT/engine_devbuf.log
step ipc_stale
bash scripts/ipc_stale.sh $TAG > /dev/null || exit $?
cat $OUT/ipc_stale.log
step done
