# threaded dispatcher fuzz on the GPU, then the slow-box hunt rider (r02m)
set -u
OUT=gpurun_out/r02m; mkdir -p $OUT
timeout -k 10 300 tests/c/_build/thread_fuzz 200 > $OUT/thread_fuzz.json 2> $OUT/thread_fuzz.err; rc=$?
echo "thread_fuzz rc=$rc"; cat $OUT/thread_fuzz.json; tail -3 $OUT/thread_fuzz.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_host_combine.py -q -m gpu -x --timeout 120 --timeout-method thread -k thread > $OUT/pytest_thread.log 2>&1; rc=$?
tail -2 $OUT/pytest_thread.log; [ $rc -eq 0 ] || exit $rc
bash scripts/slow_hunt.sh r02m
