set -u
OUT=gpurun_out/r02d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for b in 256 4096 65536; do timeout -k 10 120 tools/tune_latency $b 2000 7 > $OUT/latency_$b.txt 2>&1 || exit $?; done
cat $OUT/latency_*.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],r['frac'],r['kernel_avg_us'],r['measured_ceiling_same_box'],d['extra']['north_star_1gib_fp32_sum']['frac_of_8tbs'])"
