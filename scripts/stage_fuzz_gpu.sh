#!/bin/bash
# Row f1 fragment aggregator on the GPU box: the stage_fuzz harness as built
# (product library), then the device shim's host code under clang ASan+UBSan
# (tests/c/Makefile target asan-dev; host side only). Each step has its own
# limit; a timeout or signal ends the script. Both runs cover the zero-copy
# and the copy flush paths (six ring geometries, stage_fuzz.c).
#   usage: scripts/stage_fuzz_gpu.sh TAG [cases] [asan_cases]
#          (build first, on the CPU side: make -C tests/c all asan-dev)
set -u
TAG=${1:-r01}
CASES=${2:-300}
ACASES=${3:-120}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
t0=$(date +%s)
timeout -k 10 480 tests/c/_build/stage_fuzz "$CASES" 0x5EEDF022 > "$OUT/stage_fuzz.log" 2>&1
rc=$?; echo "stage_fuzz rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a "$OUT/stage_fuzz.log"
tail -n 2 "$OUT/stage_fuzz.log"
[ "$rc" -eq 0 ] || exit "$rc"
t0=$(date +%s)
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
timeout -k 10 480 tests/c/_build/asan-dev/stage_fuzz "$ACASES" 0xA5A5 > "$OUT/stage_fuzz_asan.log" 2>&1
rc=$?; echo "stage_fuzz (host ASan+UBSan) rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a "$OUT/stage_fuzz_asan.log"
tail -n 30 "$OUT/stage_fuzz_asan.log"
exit "$rc"
