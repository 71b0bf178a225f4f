#!/bin/bash
# The multi-operand combine (k_reduce_multi, N = 8 fp32, in phase) against its
# own variants and ceilings (tools/tune_multi), then rocprofv3 PMC passes of the
# same harness at 64 MiB per operand: HBM bytes (FETCH_SIZE, WRITE_SIZE, each
# in its own pass), L2 hit rate (TCC_HIT/MISS) and wave stall cycles (SQ).
#   usage: scripts/multi_pmc.sh OUTDIR
set -u
OUT=$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 5 120 tools/tune_multi 24 5 > $OUT/tune_multi_24.txt 2>&1 || exit $?
timeout -k 5 180 tools/tune_multi 26 3 > $OUT/tune_multi_26.txt 2>&1 || exit $?
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_$tag -o m \
      -- tools/tune_multi 24 1 > $OUT/pmc_$tag.txt 2>&1 || exit $?
done
python3 scripts/pmc_kernels.py $OUT > $OUT/pmc_by_kernel.txt 2>&1
cat $OUT/pmc_by_kernel.txt
