#!/bin/bash
# scripts/devbuf_stress.py on 8 members (sockets of 4, the layout of the r02ts
# mismatch): the completion word and hipStreamSynchronize, buffers per op and
# once.   usage: scripts/devbuf_stress.sh TAG OPS
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export UCX_BUILTIN_WAIT_TIMEOUT=60
run() { # name completion alloc
    local name=$1 r rc=0 pids=""
    for r in $(seq 0 7); do
        STRESS_COMPLETION=$2 STRESS_ALLOC=$3 RANK=$r WORLD_SIZE=8 timeout -k 10 300 \
            python -u scripts/devbuf_stress.py "/xucg_stress_${name}_$$" $NOPS 8:8:4:8:2:4 \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc" | tee -a $OUT/devbuf_stress.log
    grep -h '"rank"' $OUT/${name}_*.log | cut -c1-400 >> $OUT/devbuf_stress.log
    # a mismatch is a finding, not a failure of the script; anything else stops it
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
NOPS=$2
run signal_op signal op
run sync_op sync op
run signal_once signal once
