#!/bin/bash
# Allocation race probe (tools/src/alloc_race_probe.hip): NP processes on
# the one GPU allocate, upload, verify, use and free 2 MiB buffers with no
# engine code; then the same with every process exporting a buffer and
# importing every peer's.   usage: scripts/alloc_race.sh OUTDIR [NP] [ITERS]
set -u
OUT=$1; NP=${2:-12}; IT=${3:-400}
mkdir -p $OUT
for mode in ${MODES:-plain ipc}; do
  D=$(mktemp -d /tmp/arp.XXXXXX)
  pids=()
  for r in $(seq 0 $((NP - 1))); do
    timeout -k 10 240 tools/alloc_race_probe $r $NP $IT $mode $D > $OUT/${mode}_$r.out 2> $OUT/${mode}_$r.err &
    pids+=($!)
  done
  rcs=""
  for p in "${pids[@]}"; do wait $p; rcs="$rcs $?"; done
  rm -rf $D
  echo "$mode exit codes:$rcs"
  cat $OUT/${mode}_*.out
  for c in $rcs; do
    case $c in 0|4) ;; *) echo "probe process failed ($c)"; exit 1 ;; esac
  done
done
