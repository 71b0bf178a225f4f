#!/bin/bash
# Round-3 GPU session.   usage: scripts/gpu_r03.sh TAG STEP...
#   suite     pytest -m gpu in the order the files give (no reordering)
#   c1ab      device-buffer allreduce latency A/B (scripts/c1_dev_ab.py)
#   c1prof    rocprofv3 kernel trace of rank 0 of the 4-rank 4 KiB C1 run
#   bench     the driver's bench command
#   benchfull the default bench
#   smoke     __graft_entry__.smoke()
# Every GPU step runs under its own time limit; the first failure ends the call.
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
step() { echo "== $1 $(date +%T)" | tee -a $OUT/steps.log; }
for S in "$@"; do
  case $S in
  suite)
    step suite
    timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 250 \
        --timeout-method thread -p no:cacheprovider --durations=40 > $OUT/pytest_gpu.log 2>&1
    rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
    [ $rc -eq 0 ] || exit $rc ;;
  c1ab)
    step c1ab
    timeout -k 10 400 python -u scripts/c1_dev_ab.py $OUT/c1_dev_ab.json 3 > $OUT/c1_dev_ab.log 2>&1 || { tail -5 $OUT/c1_dev_ab.log; exit 1; }
    tail -1 $OUT/c1_dev_ab.log ;;
  c1prof)
    step c1prof
    export TMPDIR=/tmp
    NAME=ucg_prof_$$
    CPUS=($(python3 -c 'import os; print(*sorted(os.sched_getaffinity(0))[:4])'))
    for r in 1 2 3; do
      RANK=$r WORLD_SIZE=4 C1_DEVICE_BUFFERS=1 C1_REGISTERED=1 UCX_BUILTIN_WAIT_TIMEOUT=60 \
        timeout -k 5 120 taskset -c ${CPUS[$r]} tests/c/_build/c1_allreduce $NAME 2000 256 1024 \
        > $OUT/c1prof_rank$r.log 2>&1 &
    done
    RANK=0 WORLD_SIZE=4 C1_DEVICE_BUFFERS=1 C1_REGISTERED=1 UCX_BUILTIN_WAIT_TIMEOUT=60 \
      timeout -k 5 150 taskset -c ${CPUS[0]} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c1prof \
      -o c1 -- tests/c/_build/c1_allreduce $NAME 2000 256 1024 > $OUT/c1prof_rank0.log 2>&1
    rc=$?; wait; tail -2 $OUT/c1prof_rank0.log; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    step bench
    timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -5 $OUT/bench_driver.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], r['frac'], r['kernel_avg_us'], json.dumps({k: v.get('latency_us') for k, v in d['extra']['c1_loopback_allreduce_4kib_fp32'].items() if isinstance(v, dict)}))" ;;
  benchfull)
    step benchfull
    timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; } ;;
  stage)
    step stage
    timeout -k 10 300 tests/c/_build/stage_bench $((64<<20)) 8184 5 > $OUT/stage_bench.json 2> $OUT/stage_bench.err || { tail -5 $OUT/stage_bench.err; exit 1; }
    cut -c1-400 $OUT/stage_bench.json ;;
  multi)
    step multi
    bash scripts/multi_pmc.sh $OUT/multi > $OUT/multi.log 2>&1 || { tail -5 $OUT/multi.log; exit 1; }
    grep -E "%|MiB" $OUT/multi/tune_multi_24.txt ;;
  profile)
    step profile
    bash scripts/profile_round.sh $TAG/prof > $OUT/profile.log 2>&1 || { tail -5 $OUT/profile.log; exit 1; }
    P=gpurun_out/$TAG/prof
    python3 scripts/pmc_summary.py $(find $P/pmc_fetch -name "*counter_collection.csv" | head -1) \
        $(find $P/pmc_write -name "*counter_collection.csv" | head -1) $OUT/pmc_traffic.json > /dev/null 2>&1
    grep -E "ratio|hbm_bytes" $OUT/pmc_traffic.json; cat $P/trace_summary.json | head -c 600 ;;
  place)
    step place
    P=$OUT/place_$(date +%H%M%S)
    timeout -k 10 200 python -u scripts/place_probe.py ${P}_plain.json 4 > ${P}_plain.log 2>&1 || { tail -5 ${P}_plain.log; exit 1; }
    timeout -k 10 200 python -u scripts/place_probe.py ${P}_torch.json 4 --torch > ${P}_torch.log 2>&1 || { tail -5 ${P}_torch.log; exit 1; }
    python3 -c "
import json, statistics as S
for k in ('plain', 'torch'):
    d = json.load(open('${P}_' + k + '.json'))['frac_of_8tbs']
    print(k, {n: round(S.median(v), 3) for n, v in d.items()})" ;;
  scan)
    step scan
    P=$OUT/scan_$(date +%H%M%S)
    timeout -k 10 200 python -u scripts/alloc_scan.py ${P}_256.json 24 256 3 > ${P}_256.log 2>&1 || { tail -5 ${P}_256.log; exit 1; }
    timeout -k 10 200 python -u scripts/alloc_scan.py ${P}_1024.json 8 1024 3 > ${P}_1024.log 2>&1 || { tail -5 ${P}_1024.log; exit 1; }
    timeout -k 10 200 python -u scripts/alloc_scan.py ${P}_arena.json 1 8192 3 512 > ${P}_arena.log 2>&1 || { tail -5 ${P}_arena.log; exit 1; }
    tail -1 ${P}_256.log; tail -1 ${P}_1024.log; tail -1 ${P}_arena.log ;;
  alias)
    step alias
    timeout -k 10 200 python -u scripts/alias_probe.py $OUT/alias_$(date +%H%M%S).json 6 2 ;;
  aliasj)
    step aliasj
    timeout -k 10 200 python -u scripts/alias_probe.py $OUT/aliasj_$(date +%H%M%S).json 4 2 --joint ;;
  smoke)
    step smoke
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log ;;
  *) echo "unknown step $S"; exit 2 ;;
  esac
done
step done
