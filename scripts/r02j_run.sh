# round-2 rocprofv3 evidence on the current library (kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes of the bench command), then a 20 s HBM
# timeline with GPU/HBM temperatures sampled every second (r02j)
set -u
OUT=gpurun_out/r02j; mkdir -p $OUT
bash scripts/profile_round.sh r02j > $OUT/profile_steps.log 2>&1; rc=$?
tail -5 $OUT/profile_steps.log; [ $rc -eq 0 ] || exit $rc
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" | sort | tail -n 1)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" | sort | tail -n 1)
python3 scripts/pmc_summary.py "$F" "$W" $OUT/pmc_traffic.json > $OUT/pmc_summary.txt 2>&1 || true
tail -3 $OUT/pmc_summary.txt
( for i in $(seq 1 24); do echo "t=$i"; rocm-smi --showtemp 2>/dev/null | grep -i "temperature"; sleep 1; done ) > $OUT/temps.txt 2>&1 &
sp=$!
timeout -k 10 120 python -u scripts/ramp_probe.py 20 $OUT/ramp20.json > $OUT/ramp20.log 2>&1; rc=$?
wait $sp
[ $rc -eq 0 ] || exit $rc
python3 - <<'P'
import json
d=json.load(open('gpurun_out/r02j/ramp20.json'))['windows']
fr=[w['frac'] for w in d]; print('windows',len(fr),'min',min(fr),'max',max(fr))
slow=[w for w in d if w['frac']<0.82]; print('slow windows',len(slow), slow[:3])
P
head -12 $OUT/temps.txt
