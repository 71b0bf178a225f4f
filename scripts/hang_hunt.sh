#!/bin/bash
# Repeats the 5-member device-buffer runs that timed out in r02ev/r02ev2 (the
# engine fuzz with registered send buffers, the 5-host placement) with the
# timeout state dump on; stops at the first failing run.
#   usage: scripts/hang_hunt.sh TAG ROUNDS
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export UCX_BUILTIN_WAIT_TIMEOUT=20 UCX_BUILTIN_TIMEOUT_DUMP=y PYTHONPATH=$PWD
run() { # name world worker args...
    local name=$1 w=$2 wk=$3 r rc=0 pids=""; shift 3
    for r in $(seq 0 $((w - 1))); do
        RANK=$r WORLD_SIZE=$w timeout -k 10 90 python -u tests/$wk "$@" \
            > $OUT/${name}_$r.log 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait $p || rc=$?; done
    echo "$name rc=$rc $(date +%T)" | tee -a $OUT/hang_hunt.log
    return $rc
}
for i in $(seq 1 $2); do
    for seed in 14 21 22; do
        FUZZ_BUFFERS=device-reg run fz${i}_${seed}_reg 5 _worker_fuzz.py /xucg_hh_$$_${i}_$seed $seed 256 64 || exit 1
        FUZZ_BUFFERS=device run fz${i}_${seed}_dev 5 _worker_fuzz.py /xucg_hhd_$$_${i}_$seed $seed 256 64 || exit 1
    done
    run topo${i} 5 _worker_topo.py /xucg_ht_$$_$i rma 256 5:1:0:2:2:16 || exit 1
done
