#!/bin/bash
# rocprofv3 counter passes over scripts/layout_pmc.py (the headline combine on
# one allocation, then on two separate ones): address translation (TCP
# UTCL1), HBM traffic (FETCH_SIZE, WRITE_SIZE) and UTCL2 activity, one pass
# each (TCP and TCC slot limits), then the per-layout summary.
# usage: scripts/layout_pmc.sh TAG
set -u
TAG=${1:-layout}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
pass() { # name, counters...
    local name=$1
    shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o lay \
        -- python3 "$ROOT/scripts/layout_pmc.py" 20 > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc" >> "$OUT/steps.log"
    if [ "$rc" -ne 0 ]; then tail -5 "$OUT/$name.err"; exit "$rc"; fi
}
pass utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
    TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass utcl2 GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
python3 "$ROOT/scripts/layout_pmc_summary.py" "$OUT" 20 > "$OUT/summary.json"
cat "$OUT/summary.json"
