#!/bin/bash
# The operation engine end to end at a large size (row f1): N processes on
# one host allreduce 64 MiB of fp32 through the recursive-doubling plan over
# the shm transport (64 KiB messages), every combine on the host callback or
# staged on the box's GPU (C1_DEVICE_STAGING: forced, any size). Prints the
# member-0 JSON line of each run.   usage: scripts/engine_large.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
run() { # name world staging
    local name=$1 w=$2 dev=$3 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        if [ "$dev" = 1 ]; then export C1_DEVICE_STAGING=1; else unset C1_DEVICE_STAGING; fi
        RANK=$r WORLD_SIZE=$w timeout -k 10 240 tests/c/_build/c1_allreduce \
            "/xucg_big_${name}_$$" 5 65536 16777216 > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_large.log
    [ $rc -eq 0 ] || exit $rc
}
run host4 4 0
run dev4 4 1
run host8 8 0
run dev8 8 1
