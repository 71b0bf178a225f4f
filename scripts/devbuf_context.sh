#!/bin/bash
# The device-buffer placement tests after the in-process device tests in one
# pytest session (the order of the full suite, where the zeroed-allocation
# mismatches were seen), repeated.   usage: scripts/devbuf_context.sh OUTDIR [rounds]
set -u
OUT=$1; R=${2:-2}
mkdir -p $OUT
for r in $(seq 1 $R); do
  timeout -k 10 500 python -u -m pytest tests/test_gpu_combine.py tests/test_topology.py -m gpu -q \
      --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/combo_$r.log 2>&1
  rc=$?
  echo "round $r rc=$rc $(tail -1 $OUT/combo_$r.log)"
  grep -E "^FAILED" $OUT/combo_$r.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
