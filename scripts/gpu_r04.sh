#!/bin/bash
# Round-4 evidence on the GPU box, one step per argument, each under its own
# time limit, stopping at the first failure:
#   bench    the driver's command (python bench.py), then smoke()
#   profile  rocprofv3 trace + FETCH_SIZE / WRITE_SIZE passes of bench.py and the
#            per-launch HBM traffic (scripts/profile_round.sh, pmc_summary.py)
#   layout   the two operand layouts under TCP UTCL1 / UTCL2 / traffic counters
#   shift    the realigning multi-operand kernels' traffic and L2 hits
#   suite    pytest -m gpu (test failures are recorded and the script goes
#            on; a crash, abort or time limit stops it)
#   ab       the occupancy-cap and misalignment A/B tools
#   ab2      the misalignment A/B and its FETCH_SIZE pass per kernel
#   ipc      the multi-process shareable-key tests (topology, one-shot, churn)
#   c1ab     the device-buffer allreduce latency A/B (scripts/c1_dev_ab.py)
# usage: scripts/gpu_r04.sh TAG step...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in "$@"; do
  echo "step $s $(date +%T)" >> $OUT/steps.log
  case $s in
  bench)
    timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; } ;;
  profile)
    bash scripts/profile_round.sh $TAG/prof > $OUT/profile.log 2>&1 || { tail -5 $OUT/profile.log; exit 1; }
    P=$OUT/prof
    python3 scripts/pmc_summary.py $(find $P/pmc_fetch -name "*counter_collection.csv" | head -1) \
        $(find $P/pmc_write -name "*counter_collection.csv" | head -1) $OUT/pmc_traffic.json > /dev/null 2>&1 ;;
  layout)
    bash scripts/layout_pmc.sh $TAG/layout > $OUT/layout.log 2>&1 || { tail -5 $OUT/layout.log; exit 1; } ;;
  suite)
    timeout -k 10 850 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
        -p no:cacheprovider --durations=25 > $OUT/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc $rc" >> $OUT/steps.log
    [ $rc -le 1 ] || exit 1 ;;
  ab)
    timeout -k 10 200 tools/tune_cap 24 5 joint > $OUT/tune_cap_joint.txt 2>&1 || exit 1
    timeout -k 10 200 tools/tune_cap 24 5 > $OUT/tune_cap.txt 2>&1 || exit 1
    timeout -k 10 120 tools/tune_misalign 5 > $OUT/tune_misalign.txt 2>&1 || exit 1 ;;
  ab2)
    timeout -k 10 120 tools/tune_misalign 5 > $OUT/tune_misalign.txt 2>&1 || exit 1
    export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/misalign_pmc/pmc_FETCH_SIZE \
        -o s -- tools/tune_misalign 1 > $OUT/misalign_pmc.txt 2>&1 || exit 1
    python3 scripts/pmc_kernels.py $OUT/misalign_pmc > $OUT/misalign_pmc_by_kernel.txt 2>&1 ;;
  ipc)
    timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "oneshot_reduce_scatter_over_ipc or engine_placements_device_buffers or ipc_keys or churn" \
        > $OUT/pytest_ipc.log 2>&1
    rc=$?; echo "pytest rc $rc" >> $OUT/steps.log
    [ $rc -le 1 ] || exit 1 ;;
  c1ab)
    C1_AB_PROFILE=$OUT/c1prof timeout -k 10 500 python -u scripts/c1_dev_ab.py $OUT/c1_dev_ab.json 1 r04 \
        > $OUT/c1_dev_ab.log 2>&1 || { tail -5 $OUT/c1_dev_ab.log; exit 1; } ;;
  shift)
    bash scripts/shift_pmc.sh $OUT/shift > $OUT/shift.log 2>&1 || { tail -5 $OUT/shift.log; exit 1; } ;;
  esac
  echo "done $s $(date +%T)" >> $OUT/steps.log
done
