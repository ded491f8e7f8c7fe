# round 5: row rotation -- its GPU tests, full-size parity, the plan, then the default bench line
set -o pipefail
OUT=${OUT:-gpurun_out/r05c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rotation.py tests/test_gpu_plan.py tests/test_gpu_fullsize.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|PASS|FAIL" $OUT/tests.log | tail -25
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
brc=$?
python - $OUT/bench.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'us/step', round(r['us_per_step'],3), 'launches', r.get('launches_per_generate'), 'parity', d['parity']['labels_equal'], d['parity']['wave_bit_exact'])
PY
echo "bench rc=$brc"
exit $rc
