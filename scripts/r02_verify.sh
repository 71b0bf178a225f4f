#!/bin/bash
# Round-2 verification on one MI355X: box fingerprint, GPU tests, the
# fragment-aggregator fuzz (product and host-sanitizer builds, both flush
# paths), and the staged-step A/B. Each GPU step has its own limit; a failure
# ends the script before anything else touches the GPU.
#   usage: scripts/r02_verify.sh TAG
set -u
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() { local rc=$1 name=$2; echo "$name rc=$rc" | tee -a "$OUT/steps.log"; [ "$rc" -eq 0 ] || exit "$rc"; }

bash scripts/box_fingerprint.sh "$OUT/box" > "$OUT/box.log" 2>&1
step $? box
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
step $? pytest
tail -n 3 "$OUT/pytest_gpu.log"
bash scripts/stage_fuzz_gpu.sh "$TAG" 3000 1000 > "$OUT/fuzz.log" 2>&1
step $? stage_fuzz
timeout -k 10 300 tests/c/_build/stage_bench 67108864 8184 7 > "$OUT/stage_bench.json" 2> "$OUT/stage_bench.err"
step $? stage_bench
cat "$OUT/stage_bench.json"
echo done
