#!/bin/bash
# Does the GPU test suite leave the box reading slower? Headline bench
# (no extras) on a fresh box, after the maximum-size operand tests (64 GiB
# operands allocated and freed), and after the rest of the suite.
# usage: scripts/state_hunt.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
b() { timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline > $OUT/bench_$1.json 2> $OUT/bench_$1.err || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], r['frac'], r['measured_ceiling_same_box']['read_only_gbs'])" $OUT/bench_$1.json $1; }
b fresh
timeout -k 10 300 python -u -m pytest tests/test_gpu_combine.py -q -m gpu -k max_size --timeout 250 --timeout-method thread > $OUT/p_max.log 2>&1 || exit $?
tail -1 $OUT/p_max.log
b after_max
timeout -k 10 300 python scripts/slow_probe.py $OUT/slow_after_max.json > $OUT/slow_after_max.log 2>&1 || exit $?
grep separate $OUT/slow_after_max.log | head -1
timeout -k 10 400 python -u -m pytest tests -q -m gpu -k "not max_size" --timeout 250 --timeout-method thread > $OUT/p_rest.log 2>&1 || exit $?
tail -1 $OUT/p_rest.log
b after_rest
b again
