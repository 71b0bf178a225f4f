#!/bin/bash
# The engine's host code under ASan + UBSan (tests/c asan build; the device
# library as built) on device buffers: remote-key steps and the one-shot
# execution (two phases and the single pass), the tree's steps and its single
# pass, registered send buffers; 4 / 8 / 6 processes.
#   usage: scripts/asan_devbuf.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_DEVICE_BUFFERS=1 UCX_BUILTIN_WAIT_TIMEOUT=60
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1
run() { # name world count iters oneshot [registered]
    local name=$1 w=$2 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        env ${6:+C1_REGISTERED=$6} UCX_BUILTIN_DEVICE_ONESHOT=$5 RANK=$r WORLD_SIZE=$w timeout -k 10 150 \
            tests/c/_build/asan/c1_allreduce "/xucg_asan_${name}_$$" $4 256 $3 \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    bad=$(grep -l "Sanitizer\|runtime error" $OUT/${name}_*.log | wc -l)
    echo "$name rc=$rc sanitizer_reports=$bad $(tail -1 $OUT/${name}_0.log | cut -c1-150)" | tee -a $OUT/asan_devbuf.log
    [ $rc -eq 0 ] || exit $rc
}
run os4 4 300000 20 y
run st4 4 300000 20 n
run os8 8 100000 20 y
run tree6 6 300000 20 y
run pass4 4 1000 50 y
run tree6s 6 1000 50 y
run reg4 4 300000 20 y 1
run regpass8 8 1000 50 y 1
