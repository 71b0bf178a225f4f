#!/bin/bash
# Read-only fingerprint of the GPU box for the box-variance notes in DESIGN.md 5
# (product, memory vendor, power cap, perf level, clocks idle and under the
# streaming load of tools/tune_combine's ceiling probes at 1 GiB).
#   usage: scripts/box_fingerprint.sh OUTDIR   (tools built on the CPU side:
#          make -C xucg_amd/csrc tune)
set -u
OUT=${1:-gpurun_out/box}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$OUT"
cd "$ROOT"
(rocm-smi --showproductname --showmemvendor --showmaxpower --showperflevel \
    --showcomputepartition --showmemorypartition -c -P -t 2>/dev/null || true) \
    > "$OUT/smi_idle.txt"
# clocks sampled while the ceiling probes stream 1 GiB operands
( sleep 1.5; rocm-smi -c -P 2>/dev/null > "$OUT/smi_load.txt" || true ) &
sampler=$!
TUNE_CEILING=1 timeout -k 10 120 ./tools/tune_combine 28 40 > "$OUT/tune_ceiling_1GiB.txt" 2>&1
rc=$?
wait "$sampler"
grep -E "Card SKU|Card Series|vendor|Max Graphics|Performance Level|sclk|mclk|fclk|Power \(W\)" \
    "$OUT/smi_idle.txt" "$OUT/smi_load.txt" | sed 's/  */ /g'
cat "$OUT/tune_ceiling_1GiB.txt"
exit "$rc"
