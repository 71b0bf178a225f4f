#!/bin/bash
# Host buffers through the AM path (fragments in the rings) against the
# shared-memory remote-key steps (UCX_BUILTIN_SHM_ZCOPY_THRESH=1), fp32 SUM
# allreduce, 4 KiB / 1 MiB / 64 MiB at 4 and 8 processes, each bound to one
# core. usage: scripts/engine_zcopy.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
CPUS=($(python3 -c "import os;print(' '.join(map(str,sorted(os.sched_getaffinity(0)))))"))
run() { # name world count iters max_short zcopy
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        UCX_BUILTIN_SHM_ZCOPY_THRESH=$6 RANK=$r WORLD_SIZE=$w taskset -c ${CPUS[$((r % ${#CPUS[@]}))]} \
            timeout -k 10 200 tests/c/_build/c1_allreduce "/xucg_zc_${name}_$$" $4 $5 $3 \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_zcopy.log
    [ $rc -eq 0 ] || exit $rc
}
for w in 4 8; do
  run small_am_$w $w 1024 5000 256 ""
  run small_zc_$w $w 1024 5000 256 1
  run mid_am_$w $w 262144 200 8192 ""
  run mid_zc_$w $w 262144 200 8192 1
  run big_am_$w $w 16777216 5 65536 ""
  run big_zc_$w $w 16777216 5 65536 1
done
