# completion word in stage_end: GPU tests, stage_fuzz (both completion modes,
# pinned/device/pageable recv), stage_bench A/B of the three contexts (r02g)
set -u
OUT=gpurun_out/r02g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/c/_build/stage_fuzz 1200 > $OUT/stage_fuzz.json 2> $OUT/stage_fuzz.err; rc=$?
echo "fuzz rc=$rc"; cat $OUT/stage_fuzz.json; tail -2 $OUT/stage_fuzz.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/c/_build/stage_bench 67108864 8184 7 > $OUT/stage_bench.json 2> $OUT/stage_bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/stage_bench.json; [ $rc -eq 0 ] || exit $rc
