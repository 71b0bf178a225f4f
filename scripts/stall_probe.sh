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
run() { # tag test-ids... (env from STALL_ENV)
    local tag=$1; shift
    env $STALL_ENV XUCG_LAUNCH_LOG=$PWD/$OUT/ranks_$tag.log timeout -k 10 400 python -u -m pytest -v \
        --timeout 180 --timeout-method thread --durations=8 "$@" > $OUT/pytest_$tag.log 2>&1
    local rc=$?
    echo "$tag rc=$rc $(date +%s.%N) $(tail -1 $OUT/pytest_$tag.log)" | tee -a $OUT/steps.log
    grep -h "s call" $OUT/pytest_$tag.log | head -8 | tee -a $OUT/steps.log
    grep -h "ucg slow" $OUT/ranks_$tag.log | head -20 | tee -a $OUT/steps.log
    return $rc
}
P5="tests/test_topology.py::test_engine_placements_device_buffers[5:1:0:2:2:16-y]"
F5="tests/test_ops_engine.py::test_engine_fuzz_device_buffers[14-5-256-64-device-reg]"
INPROC="tests/test_gpu_combine.py::test_stage_end_completion_word tests/test_host_combine.py::test_staged_step_on_device_matches_host_fallback tests/test_host_combine.py::test_default_policy_host_buffers_stay_on_host_device_buffers_on_gpu tests/test_host_combine.py::test_staged_step_into_device_resident_recv_buffer"
STALL_ENV="XUCG_TEST_ORDER=as-given"
case "${2:-order}" in
order)
  run multi $F5 $P5
  [ $? -lt 124 ] && run inproc $INPROC $P5 $F5
  ;;
split)
  # which in-process test leaves the parent in the state that stalls the workers
  run sig tests/test_gpu_combine.py::test_stage_end_completion_word $P5
  [ $? -lt 124 ] && run host tests/test_host_combine.py::test_staged_step_on_device_matches_host_fallback tests/test_host_combine.py::test_default_policy_host_buffers_stay_on_host_device_buffers_on_gpu tests/test_host_combine.py::test_staged_step_into_device_resident_recv_buffer $P5
  ;;
each)
  # one in-process test at a time, then the 5-member fuzz (3 s fresh, 30 s stalled)
  run t1 tests/test_host_combine.py::test_staged_step_on_device_matches_host_fallback $F5
  [ $? -lt 124 ] && run t2 tests/test_host_combine.py::test_default_policy_host_buffers_stay_on_host_device_buffers_on_gpu $F5
  [ $? -lt 124 ] && run t3 tests/test_host_combine.py::test_staged_step_into_device_resident_recv_buffer $F5
  ;;
esac
kill $SAMPLER
cat $OUT/box_cpu.txt
