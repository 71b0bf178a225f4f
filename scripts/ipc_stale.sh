#!/bin/bash
# tests/c/ipc_stale between two processes on the box's GPU: kernel reads and
# copy-engine reads of a peer buffer rewritten every iteration, at 64 KiB and
# 8 MiB.  usage: scripts/ipc_stale.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
run() { # name iters bytes read
    local r rc=0 pids=""
    for r in 0 1; do
        RANK=$r WORLD_SIZE=2 timeout -k 5 100 tests/c/_build/ipc_stale "/xucg_stale_$1_$$" $2 $3 $4 \
            > $OUT/$1_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$1 rc=$rc $(tail -1 $OUT/$1_1.log)" | tee -a $OUT/ipc_stale.log
    [ $rc -le 3 ] || exit $rc
}
run k64k 2000 65536 kernel
run d64k 2000 65536 dma
run k8m 300 8388608 kernel
# the writer waits on the engine's completion word instead of the runtime
export IPC_STALE_WAIT=signal
run k64k_sig 2000 65536 kernel
run d64k_sig 2000 65536 dma
run k8m_sig 300 8388608 kernel
