#!/bin/bash
# Fingerprint of the GPU box for the box-variance notes in DESIGN.md 5:
# partition modes and clocks (read-only rocm-smi queries), then the headline
# kernel and its A/B variants. usage: scripts/box_probe.sh OUTDIR
set -u
OUT=${1:-gpurun_out/box}
mkdir -p "$OUT"
(rocm-smi --showcomputepartition --showmemorypartition --showclocks --showtemp \
    --showpower --showfwinfo 2>/dev/null || true) > "$OUT/rocm_smi.txt"
timeout -k 10 60 python scripts/runtime_probe.py torch > "$OUT/runtime.txt" 2>&1 || exit 1
timeout -k 10 200 ./tools/tune_combine 26 3 > "$OUT/tune.txt" 2>&1 || exit 1
grep -E "partition|Partition" "$OUT/rocm_smi.txt" | head -4
cat "$OUT/runtime.txt"
head -4 "$OUT/tune.txt"
