#!/bin/bash
# BASELINE config 1 through the engine with every combine staged on the GPU
# (C1_DEVICE_STAGING=1), from C: the product build, then the host engine
# under gcc ASan+UBSan (tests/c/Makefile target asan). N processes share the
# box's one GPU. Each run has its own limit; a failure ends the script.
#   usage: scripts/c1_device_gpu.sh TAG
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export C1_DEVICE_STAGING=1
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1

run() { # name exe world max_short plan iters
    local name=$1 exe=$2 w=$3 ms=$4 plan=$5 iters=$6 r rc=0 pids=""
    for r in $(seq 0 $((w - 1))); do
        RANK=$r WORLD_SIZE=$w UCX_BUILTIN_ALLREDUCE_PLAN=$plan \
            timeout -k 10 120 "$exe" "/xucg_c1dev_${name}_$$" "$iters" "$ms" \
            > "$OUT/c1dev_${name}_$r.log" 2>&1 &
        pids="$pids $!"
    done
    for p in $pids; do wait "$p" || rc=$?; done
    echo "$name world=$w max_short=$ms plan=$plan rc=$rc: $(tail -1 "$OUT/c1dev_${name}_0.log")" \
        | tee -a "$OUT/c1dev.log"
    [ "$rc" -eq 0 ] || exit "$rc"
}
run rec4 tests/c/_build/c1_allreduce 4 8192 auto 500
run rec4_frag tests/c/_build/c1_allreduce 4 256 auto 200
run tree3 tests/c/_build/c1_allreduce 3 256 tree 200
run asan_rec4 tests/c/_build/asan/c1_allreduce 4 256 auto 100
run asan_tree5 tests/c/_build/asan/c1_allreduce 5 256 tree 100
echo done
