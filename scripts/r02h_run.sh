# completion word + deferred slot events + whole-buffer/staged interference
# fix: GPU tests, stage_fuzz (product and host ASan+UBSan), stage_bench (r02h)
set -u
OUT=gpurun_out/r02h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/stage_fuzz_gpu.sh r02h 1500 400 > $OUT/fuzz_steps.log 2>&1; rc=$?
cat $OUT/fuzz_steps.log | grep -v "^stage_fuzz: " | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/c/_build/stage_bench 67108864 8184 7 > $OUT/stage_bench.json 2> $OUT/stage_bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/stage_bench.json; [ $rc -eq 0 ] || exit $rc
