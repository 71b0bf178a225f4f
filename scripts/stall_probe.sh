#!/bin/bash
# Where the 10-40 s stalls of the 5-member device tests come from: the box's
# CPU limits and throttling (cgroup cpu.stat) and GPU busy sampled every
# 0.5 s while the 5-member placement test runs, next to the engine's
# timestamped slow-call notes.   usage: scripts/stall_probe.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
{
  echo "nproc $(nproc)"; grep -E "Cpus_allowed_list" /proc/self/status
  CG=/sys/fs/cgroup$(cut -d: -f3 /proc/self/cgroup | head -1)
  echo "cgroup $CG"; cat $CG/cpu.max 2>/dev/null; cat $CG/cpuset.cpus.effective 2>/dev/null
  cat $CG/cpu.stat 2>/dev/null
} > $OUT/box_cpu.txt 2>&1
CG=/sys/fs/cgroup$(cut -d: -f3 /proc/self/cgroup | head -1)
( while true; do
    echo "$(date +%s.%N) $(cat /sys/class/drm/card*/device/gpu_busy_percent 2>/dev/null | tr '\n' ' ') | $(grep -E 'nr_throttled|throttled_usec' $CG/cpu.stat 2>/dev/null | tr '\n' ' ') | load $(cut -d' ' -f1-3 /proc/loadavg)"
    sleep 0.5
  done ) > $OUT/samples.log 2>&1 &
SAMPLER=$!
run() { # tag spec extra-env...
    local tag=$1 spec=$2; shift 2
    env "$@" XUCG_LAUNCH_LOG=$PWD/$OUT/ranks_$tag.log timeout -k 10 200 python -u -m pytest -q \
        --timeout 180 --timeout-method thread --durations=5 \
        "tests/test_topology.py::test_engine_placements_device_buffers[$spec]" > $OUT/pytest_$tag.log 2>&1
    local rc=$?
    echo "$tag rc=$rc $(date +%s.%N) $(tail -1 $OUT/pytest_$tag.log)" | tee -a $OUT/steps.log
    grep -h "ucg slow" $OUT/ranks_$tag.log | head -20 | tee -a $OUT/steps.log
    return $rc
}
run a "5:1:0:2:2:16-y"
[ $? -lt 124 ] && run b "5:1:0:2:2:16-y" UCX_BUILTIN_WAIT_SPIN=64
[ $? -lt 124 ] && run c "8:8:0:8:2:16-y"
kill $SAMPLER
cat $OUT/box_cpu.txt
