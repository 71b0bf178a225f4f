#!/bin/bash
# rocprofv3 counters of the 8-operand one-shot kernel uncapped and capped at 8
# waves per CU (tools/tune_occ with TUNE_OCC_PMC=1, 64 MiB per operand):
# HBM bytes (FETCH_SIZE, WRITE_SIZE, separate passes) and the waves resident
# (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES).   usage: scripts/occ_pmc.sh OUTDIR
set -u
OUT=$1; mkdir -p $OUT
export TMPDIR=/tmp
export TUNE_OCC_PMC=1
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_$tag -o o \
      -- tools/tune_occ 24 3 > $OUT/pmc_$tag.txt 2>&1 || exit $?
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o o \
    -- tools/tune_occ 24 3 > $OUT/trace.txt 2>&1 || exit $?
find $OUT -name "*.csv" | sort
