# full GPU pass: -m gpu suite (sweep lines into $OUT/sweep.jsonl), smoke, default bench line
set -o pipefail
OUT=${OUT:-gpurun_out/full}
mkdir -p $OUT
WRNN_SWEEP_OUT=$OUT/sweep.jsonl timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -3
grep -E "^FAILED" $OUT/tests.log | head -20
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
echo "bench rc=$?"
python - $OUT/bench.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'us/step', round(r['us_per_step'],3), 'parity', d['parity']['labels_equal'], d['parity']['wave_bit_exact'])
PY
exit $rc
