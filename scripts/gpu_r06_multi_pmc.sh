#!/bin/bash
# r06: PMC attribution of k_reduce_multi at C4's shard size (8 x 512 MiB
# fp32, one arena) against its read-only and store-without-dependency
# ceilings: HBM bytes (FETCH_SIZE, WRITE_SIZE), L2 hit/miss,
# L2-to-fabric read requests, and the vector L1's address-translation misses,
# one counter group per pass.
# Usage: scripts/gpu_r06_multi_pmc.sh OUTDIR ["SPEC" ["FILTER" ["PASSES"]]]
#   SPEC: tune_multi_pf's arguments (default "multi 8 27 1"; with FILTER it
#   needs its stagger and separate arguments too), FILTER its variant filter,
#   PASSES ';'-separated counter groups (default: all five below)
set -u
OUT=$1; mkdir -p $OUT
SPEC=${2:-"multi 8 27 1"}
FILTER=${3:-}
PASSES=${4:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"}
read -r -a ARGS <<< "$SPEC"
if [ -n "$FILTER" ]; then ARGS+=("$FILTER"); fi
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || echo "list rc $?" >> $OUT/steps.log
IFS=';' read -r -a PLIST <<< "$PASSES"
for pass in "${PLIST[@]}"; do
  tag=$(echo $pass | cut -d' ' -f1)
  echo "pass $tag $(date +%T)" >> $OUT/steps.log
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_$tag -o m \
      -- tools/tune_multi_pf "${ARGS[@]}" > $OUT/pmc_$tag.txt 2>&1 || echo "pass $tag rc $?" >> $OUT/steps.log
done
python3 scripts/pmc_kernels.py $OUT > $OUT/pmc_by_kernel.txt 2>&1
echo "done $(date +%T)" >> $OUT/steps.log
