# smoke() with the staged step, then the engine at 64 MiB (host vs GPU-staged)
set -u
OUT=gpurun_out/r02n; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/engine_large.sh r02n
bash scripts/slow_hunt.sh r02n
