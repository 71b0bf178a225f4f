#!/bin/bash
# A/B of the waypoints' fragment-by-fragment forwarding (UCX_BUILTIN_PIPELINE)
# in the engine on the host: 12 processes as 4 hosts of 3 with tree radix 2
# (member 6 is a waypoint at both network levels), fp32 SUM allreduce of
# 4 MiB in 8 KiB messages and of 64 KiB in 256-B messages, each member bound
# to one core. usage: scripts/engine_pipeline.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export C1_PPN=3 UCX_BUILTIN_TREE_RADIX=2
CPUS=($(python3 -c "import os;print(' '.join(map(str,sorted(os.sched_getaffinity(0)))))"))
run() { # name pipeline count max_short iters
    local name=$1 r rc=0 pids=""
    for r in $(seq 0 11); do
        UCX_BUILTIN_PIPELINE=$2 RANK=$r WORLD_SIZE=12 taskset -c ${CPUS[$((r % ${#CPUS[@]}))]} timeout -k 10 240 \
            tests/c/_build/c1_allreduce "/xucg_pipe_${name}_$$" $5 $4 $3 > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(tail -1 $OUT/${name}_0.log)" | tee -a $OUT/engine_pipeline.log
    [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2 3; do
  run big_on_$rep y 1048576 8192 40
  run big_off_$rep n 1048576 8192 40
  run small_on_$rep y 16384 256 400
  run small_off_$rep n 16384 256 400
done
