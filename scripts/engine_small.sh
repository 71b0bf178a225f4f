#!/bin/bash
# Small device messages: the single-pass one-shot (every member reads all N
# buffers, one kernel) against reduce-scatter + all-gather
# (UCX_BUILTIN_DEVICE_ONESHOT_FULL=0), registered send buffers.
#   usage: scripts/engine_small.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_DEVICE_BUFFERS=1 C1_REGISTERED=1 UCX_BUILTIN_WAIT_TIMEOUT=60
run() { # name world count iters full
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        env ${5:+UCX_BUILTIN_DEVICE_ONESHOT_FULL=$5} RANK=$r WORLD_SIZE=$w timeout -k 10 150 \
            tests/c/_build/c1_allreduce "/xucg_small_${name}_$$" $4 256 $3 \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_small.log
    [ $rc -eq 0 ] || exit $rc
}
for w in 4 8; do
  for c in 1024 16384 262144; do
    run w${w}_c${c}_split $w $c 1000 0
    run w${w}_c${c}_full $w $c 1000 ""
  done
done
