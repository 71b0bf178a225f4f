#!/bin/bash
# Which osHandle convention hipMemImportFromShareableHandle takes for a POSIX
# fd (the value cast to a pointer, or the address of the int) under
# /opt/rocm's HIP runtime and under the one torch bundles (scripts/vmm_probe.py).
OUT=${1:-gpurun_out/vmmconv}
mkdir -p $OUT
TORCH_LIB=$(python3 -c 'import torch, os; print(os.path.join(os.path.dirname(torch.__file__), "lib"))')
# the tool asks for libamdhip64.so.7; torch ships it as libamdhip64.so
RT=$(mktemp -d)
ln -s $TORCH_LIB/libamdhip64.so $RT/libamdhip64.so.7
for rt in rocm torch; do
  for conv in value pointer; do
    if [ $rt = torch ]; then export LD_LIBRARY_PATH=$RT:$TORCH_LIB; else unset LD_LIBRARY_PATH; fi
    VMM_FD_CONV=$conv timeout -k 5 60 python3 scripts/vmm_probe.py 16 > $OUT/${rt}_${conv}.log 2>&1
    echo "$rt $conv rc $?" >> $OUT/summary.txt
  done
done
