#!/bin/bash
# Row f1 fragment aggregator on the GPU box: the stage_fuzz harness as built
# (product library), then the device shim's host code under clang ASan+UBSan
# (tests/c/Makefile target asan-dev; host side only). Each step has its own
# limit; a timeout or signal ends the script.
#   usage: scripts/stage_fuzz_gpu.sh TAG   (build first, on the CPU side:
#          make -C tests/c all asan-dev)
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 240 tests/c/_build/stage_fuzz 300 0x5EEDF022 > "$OUT/stage_fuzz.log" 2>&1
rc=$?; echo "stage_fuzz rc=$rc"; tail -3 "$OUT/stage_fuzz.log"
[ "$rc" -eq 0 ] || exit "$rc"
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
timeout -k 10 300 tests/c/_build/asan-dev/stage_fuzz 120 0xA5A5 > "$OUT/stage_fuzz_asan.log" 2>&1
rc=$?; echo "stage_fuzz (host ASan+UBSan) rc=$rc"; tail -30 "$OUT/stage_fuzz_asan.log"
exit "$rc"
