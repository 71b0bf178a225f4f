#!/bin/bash
# The full GPU suite R times in one call (rate of intermittent failures).
#   usage: scripts/suite_repeat.sh OUTDIR [R]
set -u
OUT=$1; R=${2:-2}; mkdir -p $OUT
for r in $(seq 1 $R); do
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread \
      -p no:cacheprovider > $OUT/suite_$r.log 2>&1
  rc=$?
  echo "suite $r rc=$rc $(tail -1 $OUT/suite_$r.log)"
  grep -E "^FAILED" $OUT/suite_$r.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
