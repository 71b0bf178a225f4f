#!/bin/bash
# One GPU session: parity tests -> bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; a crash/timeout (rc >= 124 or a
# signal) ends the script before anything else touches the GPU.
#   usage: scripts/gpu_round.sh TAG [tests|bench|prof|all]
set -u
TAG=${1:-r01}
WHAT=${2:-all}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp

fatal() { # rc -> 0 if the step may be followed by another GPU step
    local rc=$1
    if [ "$rc" -ge 124 ] || [ "$rc" -ge 128 ]; then
        echo "step ended with rc=$rc (timeout/signal): stopping" | tee -a "$OUT/steps.log"
        exit "$rc"
    fi
}

if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
    echo "== pytest -m gpu" | tee -a "$OUT/steps.log"
    timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.log"; tail -5 "$OUT/pytest_gpu.log"
    fatal $rc
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
    echo "== bench" | tee -a "$OUT/steps.log"
    timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
    fatal $rc
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
    echo "== rocprofv3 kernel trace" | tee -a "$OUT/steps.log"
    cd /tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" \
        --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
    rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/steps.log"
    cd "$ROOT"
    find "$OUT/prof" -name "*kernel_stats.csv" -exec head -20 {} \; 2>/dev/null
    fatal $rc
fi
echo "done" | tee -a "$OUT/steps.log"
