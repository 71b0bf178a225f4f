#!/bin/bash
# r06: k_reduce_multi at C4's per-GPU shard size (8 x 512 MiB fp32) - the
# prefetch distance, U vectors per lane, and operand stagger (operands a
# power of two apart) A/B (tools/tune_multi_pf).
# Usage: scripts/gpu_r06_multi.sh OUTDIR "spec;spec;..." [FILTER]
#   FILTER: variant-name substrings, ','-separated (tune_multi_pf's 7th
#   argument; every spec then needs its stagger and separate arguments)
OUT=${1:-gpurun_out/r06a}
SPECS=${2:-"multi 8 27 5 0;multi 8 27 5 4352;multi 8 26 5 0;multi 8 26 5 4352;multi 8 24 5 0"}
FILTER=${3:-}
mkdir -p $OUT
IFS=';'
for spec in $SPECS; do
    tag=$(echo $spec | tr ' ' '_')
    echo "step $tag $(date +%T)" >> $OUT/steps.log
    IFS=' ' read -r -a args <<< "$spec"
    if [ -n "$FILTER" ]; then args+=("$FILTER"); fi
    timeout -k 10 200 tools/tune_multi_pf "${args[@]}" > $OUT/pf_$tag.txt 2>&1 || exit $?
done
echo "done $(date +%T)" >> $OUT/steps.log
