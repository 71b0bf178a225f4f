#!/bin/bash
# run the device-buffer engine worker directly, one log per member
# usage: scripts/rma_debug.sh TAG SPEC
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
N=${2%%:*}
export UCX_BUILTIN_WAIT_TIMEOUT=20 PYTHONPATH=$PWD WORLD_SIZE=$N
pids=""
for r in $(seq 0 $((N - 1))); do
    RANK=$r LOCAL_RANK=$r timeout -k 5 90 python -u tests/_worker_topo.py /xucg_rma_dbg_$$ rma 256 $2 > $OUT/w$r.log 2>&1 &
    pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for r in $(seq 0 $((N - 1))); do echo "== $r"; tail -15 $OUT/w$r.log; done
exit $rc
