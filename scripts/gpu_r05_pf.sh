#!/bin/bash
# r05: next-tile prefetch A/B for the in-phase multi-operand kernels
# (tools/tune_multi_pf). Usage: scripts/gpu_r05_pf.sh OUTDIR
OUT=${1:-gpurun_out/r05a}
mkdir -p $OUT
for spec in "multi 8 24" "multi 4 24" "multi 16 24" "multi 8 26" "tree 8 24" "tree 3 24" "tree 12 24" "tree 6 24"; do
    tag=$(echo $spec | tr ' ' '_')
    echo "step $tag $(date +%T)" >> $OUT/steps.log
    timeout -k 10 150 tools/tune_multi_pf $spec 7 > $OUT/pf_$tag.txt 2>&1 || exit $?
done
echo "done $(date +%T)" >> $OUT/steps.log
