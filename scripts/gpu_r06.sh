#!/bin/bash
# Round-6 evidence on the GPU box, one step per argument, each under its own
# time limit, stopping at the first crash or time limit:
#   suite    pytest -m gpu (test failures recorded, the script goes on)
#   tests:A,B   a pytest -m gpu subset (-k "A or B")
#   bench    the driver's command (python bench.py), then smoke()
#   profile  rocprofv3 trace + FETCH_SIZE / WRITE_SIZE passes of bench.py and the
#            per-launch HBM traffic keyed to the device code object
#            (scripts/profile_round.sh, pmc_summary.py)
#   dryalloc bench.py --collective-dry-alloc (one rank's C4 + C5 buffers)
#   gather   the out-of-phase gather A/B (tools/tune_misalign)
#   c3       BASELINE config 3: every dtype x op, 1 KiB - 1 GiB (sweep_c3.py), and
#            the lowest pairs interleaved with fp32 SUM (c3_interleaved.py)
# usage: scripts/gpu_r06.sh TAG step...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in "$@"; do
  echo "step $s $(date +%T)" >> $OUT/steps.log
  case $s in
  suite)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
        -p no:cacheprovider --durations=25 > $OUT/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc $rc" >> $OUT/steps.log
    [ $rc -le 1 ] || exit 1 ;;
  tests:*)
    timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "$(echo "${s#tests:}" | sed 's/,/ or /g')" > $OUT/pytest_subset.log 2>&1
    rc=$?; echo "pytest rc $rc" >> $OUT/steps.log
    [ $rc -le 1 ] || exit 1 ;;
  bench)
    timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; } ;;
  profile)
    bash scripts/profile_round.sh $TAG/prof > $OUT/profile.log 2>&1 || { tail -5 $OUT/profile.log; exit 1; }
    P=$OUT/prof
    python3 scripts/pmc_summary.py $(find $P/pmc_fetch -name "*counter_collection.csv" | head -1) \
        $(find $P/pmc_write -name "*counter_collection.csv" | head -1) $OUT/pmc_traffic.json \
        $P/lib_sha.txt $P/code_sha.txt > /dev/null 2>&1 ;;
  dryalloc)
    timeout -k 10 300 python bench.py --collective-dry-alloc > $OUT/dryalloc.json 2> $OUT/dryalloc.err || { tail -5 $OUT/dryalloc.err; exit 1; } ;;
  gather)
    timeout -k 10 200 tools/tune_misalign 5 > $OUT/tune_misalign.txt 2>&1 || exit 1 ;;
  c3)
    timeout -k 10 400 python scripts/sweep_c3.py $OUT/c3_sweep.json > $OUT/c3_sweep.log 2>&1 || exit 1
    timeout -k 10 300 python scripts/c3_interleaved.py $OUT/c3_interleaved.json > $OUT/c3_interleaved.log 2>&1 || exit 1 ;;
  esac
  echo "done $s $(date +%T)" >> $OUT/steps.log
done
