# run the slow-box probes only when this box is a slow one (headline combine
# under 82% of 8 TB/s); usage: scripts/slow_hunt.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 120 python -u scripts/slow_probe.py $OUT/slow_probe.json > $OUT/slow_probe.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/slow_probe.log | head -3
slow=$(python3 -c "import json;r=json.load(open('$OUT/slow_probe.json'));print(int(r[0]['combine_frac']<0.82))")
echo "slow=$slow"
if [ "$slow" = 1 ]; then
  grep -v amdgpu.ids $OUT/slow_probe.log
  TUNE_CEILING=1 timeout -k 10 120 ./tools/tune_combine 28 20 > $OUT/tune_ceiling_1GiB.txt 2>&1 || exit $?
  cat $OUT/tune_ceiling_1GiB.txt
  timeout -k 10 180 ./tools/tune_combine 26 20 > $OUT/tune_variants_256MiB.txt 2>&1 || exit $?
  tail -30 $OUT/tune_variants_256MiB.txt
fi
