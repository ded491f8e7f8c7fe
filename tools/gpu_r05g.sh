# round 5: time-sliced wide launches -- rotation / plan / full-size / wide tests, C4 bench, C2 bench
set -o pipefail
OUT=${OUT:-gpurun_out/r05g}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_rotation.py tests/test_gpu_plan.py tests/test_gpu_fullsize.py tests/test_gpu_wide.py tests/test_gpu_logits.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; grep -E "^FAILED" $OUT/tests.log | head
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for args in "--utts-per-gpu 8 --steps 3 --warmup 1 --cpu-seconds 0" "--steps 5 --warmup 1 --cpu-seconds 0"; do
  timeout -k 10 300 python -u bench.py $args > $OUT/bench_$(echo $args | cut -c3-7).log 2>&1 || { echo "bench fail $args"; exit 1; }
  python - $OUT/bench_$(echo $args | cut -c3-7).log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(d['config']['workload'][:30], 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'us/step', round(r['us_per_step'],3), 'call_us/step', round(r.get('call_us_per_step',0),3), 'steps/launch', r.get('steps_per_launch'), 'parity', d.get('parity',{}).get('labels_equal'))
PY
done
exit $rc
