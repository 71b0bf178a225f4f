#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box via gpurun):
#   1. kernel trace + stats of bench.py (the same command the driver runs)
#   2. PMC FETCH_SIZE pass, 3. PMC WRITE_SIZE pass (separate passes: TCC slots)
# usage: scripts/profile_round.sh TAG
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp

run() { # name, limit, args...
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" rocprofv3 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc" | tee -a "$OUT/steps.log"
    if [ "$rc" -ne 0 ]; then tail -5 "$OUT/$name.err"; exit "$rc"; fi
}

# the library every pass below runs (bench.py compares it with the one it
# loads: roofline.traffic_source.stale)
sha256sum "$ROOT/xucg_amd/lib/libucg_builtin_dev.so" > "$OUT/lib_sha.txt"
# and its device code alone (.hip_fatbin): what the counters are keyed to
python3 -c "import sys; sys.path.insert(0, '$ROOT'); from xucg_amd import _lib; print(_lib.code_object_sha16())" \
    > "$OUT/code_sha.txt"

# the same command as the driver's bench minus the CPU leg and the extra
# sizes, so every k_reduce launch in the trace is the headline 2^26 combine
run trace 600 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra
python3 "$ROOT/scripts/trace_summary.py" "$OUT/trace/bench_kernel_trace.csv" \
    "$OUT/trace_summary.json" > /dev/null
run pmc_fetch 600 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o bench \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-extra
run pmc_write 600 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o bench \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-extra
find "$OUT" -name "*.csv" | sort
echo done
