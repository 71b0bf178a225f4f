#!/bin/bash
# Counter passes over scripts/shift_pmc.py (the realigning multi-operand
# kernels, N = 8, 64 MiB per operand): HBM bytes (FETCH_SIZE, WRITE_SIZE, one
# pass each) and the L2 hit rate (TCC_HIT_sum, TCC_MISS_sum); then the
# per-kernel averages (scripts/pmc_kernels.py).
#   usage: scripts/shift_pmc.sh OUTDIR
set -u
OUT=$1; mkdir -p $OUT
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
timeout -k 5 120 python3 $ROOT/scripts/shift_pmc.py 10 > $OUT/timing.txt 2>&1 || exit $?
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_$tag -o s \
      -- python3 $ROOT/scripts/shift_pmc.py 5 > $OUT/pmc_$tag.txt 2>&1 || exit $?
done
python3 $ROOT/scripts/pmc_kernels.py $OUT --json $OUT/pmc_by_kernel.json > $OUT/pmc_by_kernel.txt 2>&1
cat $OUT/timing.txt $OUT/pmc_by_kernel.txt
