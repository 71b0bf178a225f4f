#!/bin/bash
# The device-buffer engine tests under pytest, ROUNDS times in one session
# (where the 5-member timeouts of r02hh were seen), with the timeout dump and
# the slow-call notes on; stops at the first failing round.
#   usage: scripts/devbuf_repeat.sh TAG ROUNDS
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
for i in $(seq 1 $2); do
    echo "== round $i $(date +%T)" | tee -a $OUT/steps.log
    XUCG_LAUNCH_LOG=$PWD/$OUT/ranks_$i.log timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread --durations=12 \
        tests/test_gpu_combine.py tests/test_host_combine.py tests/test_ops_engine.py \
        tests/test_topology.py -k "device or completion_word" > $OUT/devbuf_$i.log 2>&1
    rc=$?
    tail -1 $OUT/devbuf_$i.log | tee -a $OUT/steps.log
    grep -h "ucg slow\|ucg timeout" $OUT/devbuf_$i.log $OUT/ranks_$i.log | head -40 | tee -a $OUT/steps.log
    [ $rc -eq 0 ] || exit $rc
done
