# size/placement probe of the headline combine, product kernel and the
# temporal-store variant, plus the box fingerprint (r02e)
set -u
OUT=gpurun_out/r02e; mkdir -p $OUT
bash scripts/box_fingerprint.sh $OUT/box > $OUT/box.log 2>&1
timeout -k 10 300 python -u scripts/size_probe.py $OUT/size_probe_v0.json > $OUT/size_probe_v0.log 2>&1 || exit $?
UCX_BUILTIN_DEV_VARIANT=3 timeout -k 10 300 python -u scripts/size_probe.py $OUT/size_probe_v3.json > $OUT/size_probe_v3.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/size_probe.py $OUT/size_probe_v0b.json > $OUT/size_probe_v0b.log 2>&1 || exit $?
for f in $OUT/size_probe_*.log; do echo "== $f"; grep -v '^{' $f | tail -3; done
python3 - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/r02e/size_probe_*.json')):
    d=json.load(open(f)); print(f, {k:v['median_frac'] for k,v in d.items() if isinstance(v,dict)})
P
