#!/bin/bash
# The engine on device buffers with the send buffer from the group's
# registered memory (C1_REGISTERED: exposed in place, no init copy) beside
# the plain device buffers.   usage: scripts/engine_devbuf_reg.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_DEVICE_BUFFERS=1 UCX_BUILTIN_WAIT_TIMEOUT=60
run() { # name world count iters registered
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        env ${5:+C1_REGISTERED=$5} RANK=$r WORLD_SIZE=$w timeout -k 10 150 tests/c/_build/c1_allreduce \
            "/xucg_dreg_${name}_$$" $4 256 $3 > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_devbuf_reg.log
    [ $rc -eq 0 ] || exit $rc
}
for w in 2 4 8; do
  run big${w}_copy $w 16777216 20 ""
  run big${w}_reg $w 16777216 20 1
done
run small4_copy 4 1024 2000 ""
run small4_reg 4 1024 2000 1
