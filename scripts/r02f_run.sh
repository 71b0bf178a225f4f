# HBM-rate timeline from a cold process (ramp_probe) with clock samples, then
# the same bench command the driver runs (r02f)
set -u
OUT=gpurun_out/r02f; mkdir -p $OUT
rocm-smi -s > $OUT/smi_clk_idle.txt 2>&1 || true
( for i in 1 2 3 4 5 6; do sleep 0.5; rocm-smi -s > $OUT/smi_clk_load_$i.txt 2>&1; done ) &
sp=$!
timeout -k 10 120 python -u scripts/ramp_probe.py 4 $OUT/ramp1.json > $OUT/ramp1.log 2>&1; rc=$?
wait $sp
[ $rc -eq 0 ] || exit $rc
sleep 5
timeout -k 10 120 python -u scripts/ramp_probe.py 2 $OUT/ramp2.json > $OUT/ramp2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench.err || exit $?
grep -v amdgpu.ids $OUT/ramp1.log | head -40
grep -v amdgpu.ids $OUT/ramp2.log | head -12
python3 -c "import json;d=json.load(open('$OUT/bench_driver_cmd.json'));r=d['roofline'];print(d['value'],r['frac'],r['kernel_avg_us_batches'],d['extra']['north_star_1gib_fp32_sum']['frac_of_8tbs'])"
grep -h "fclk\|mclk\|socclk" $OUT/smi_clk_idle.txt | head; grep -h "\*" $OUT/smi_clk_load_*.txt | head -30
