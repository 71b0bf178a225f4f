#!/bin/bash
# A/B of the device-buffer placement tests with and without the occupancy cap
# of the multi-operand kernels (UCX_BUILTIN_DEV_MULTI_WAVES=0 vs the table),
# each case list repeated TOPO_REPEAT times, alternating.
#   usage: scripts/devbuf_ab.sh OUTDIR [rounds] [repeat]
set -u
OUT=$1; R=${2:-3}; REP=${3:-4}
mkdir -p $OUT
SEL='test_engine_placements_device_buffers and (8:8:0:8:2:16-n or 12:12:6 or 12:12:0 or 8:8:0:8:2:16-y)'
for r in $(seq 1 $R); do
  for mode in nocap table; do
    if [ $mode = nocap ]; then export UCX_BUILTIN_DEV_MULTI_WAVES=0; else unset UCX_BUILTIN_DEV_MULTI_WAVES; fi
    TOPO_REPEAT=$REP timeout -k 10 400 python -u -m pytest tests/test_topology.py -m gpu -q \
        --timeout 300 --timeout-method thread -p no:cacheprovider -k "$SEL" \
        > $OUT/${mode}_$r.log 2>&1
    rc=$?
    echo "$mode round $r rc=$rc $(tail -1 $OUT/${mode}_$r.log)"
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
done
