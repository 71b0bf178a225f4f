#!/bin/bash
# Small device messages on a one-host tree (non-power-of-two groups): the
# single pass (every member folds all members' data in the root's order)
# against the tree's steps (UCX_BUILTIN_DEVICE_ONESHOT=n), registered send
# buffers.   usage: scripts/engine_tree_small.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_DEVICE_BUFFERS=1 C1_REGISTERED=1 UCX_BUILTIN_WAIT_TIMEOUT=60
run() { # name world count iters oneshot
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        UCX_BUILTIN_DEVICE_ONESHOT=$5 RANK=$r WORLD_SIZE=$w timeout -k 10 150 \
            tests/c/_build/c1_allreduce "/xucg_tsmall_${name}_$$" $4 256 $3 \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_tree_small.log
    [ $rc -eq 0 ] || exit $rc
}
for w in 3 6; do
  for c in 1024 262144; do
    run w${w}_c${c}_steps $w $c 1000 n
    run w${w}_c${c}_pass $w $c 1000 y
  done
done
