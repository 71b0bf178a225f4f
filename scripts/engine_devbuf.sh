#!/bin/bash
# The engine on device buffers (remote-key steps): N processes sharing the
# box's GPU allreduce fp32 SUM through the builtin plans, buffers in HBM, every
# receive one kernel reading the senders' buffers over IPC. 64 MiB with 2, 4
# and 8 processes (recursive doubling), 6 (the tree), and 4 KiB for the
# per-step latency. Prints member 0's JSON line.  usage: scripts/engine_devbuf.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_DEVICE_BUFFERS=1 UCX_BUILTIN_WAIT_TIMEOUT=60
run() { # name world count iters
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        RANK=$r WORLD_SIZE=$w timeout -k 10 150 tests/c/_build/c1_allreduce \
            "/xucg_dbuf_${name}_$$" $4 256 $3 > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_devbuf.log
    [ $rc -eq 0 ] || exit $rc
}
run big2 2 16777216 20
run big4 4 16777216 20
run big8 8 16777216 20
run big6 6 16777216 20
run small4 4 1024 2000
run small8 8 1024 2000
