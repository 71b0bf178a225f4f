# placements planner on the GPU (device-staged waypoints) + full GPU tests +
# bench line (r02i)
set -u
OUT=gpurun_out/r02i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],r['frac'],r['kernel_avg_us_batches'],d['extra']['north_star_1gib_fp32_sum']['frac_of_8tbs'],d['extra']['f1_staged_step_64mib_fp32'].get('small_step_us_device_recv'))"
