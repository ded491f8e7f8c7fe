# round 5: time-sliced runtimeracer wide launches -- wide / logits / trained / rotation /
# plan / full-size tests, then benches: C4 (9-bit sliced), C2, and the fatchord 10-bit default
# batch (8 x 1000 frames at 3000 / 1500: 360 rows) on the wide kernel and on the
# register-resident plan (WRNN_PERSIST_WIDE=0)
set -o pipefail
OUT=${OUT:-gpurun_out/r05j}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_wide_rr.py tests/test_gpu_rotation.py tests/test_gpu_plan.py tests/test_gpu_logits.py tests/test_gpu_sweep.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; grep -E "^FAILED" $OUT/tests.log | head
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B10="--utts-per-gpu 8 --bits 10 --target 3000 --overlap 1500 --steps 3 --warmup 1 --cpu-seconds 0"
bench() {  # name, env, args
  env $2 timeout -k 10 300 python -u bench.py $3 > $OUT/bench_$1.log 2>&1 || { echo "bench $1 failed"; exit 1; }
  python - $OUT/bench_$1.log $1 <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[2], 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'us/step', round(r['us_per_step'],3), 'call_us/step', round(r.get('call_us_per_step',0),3), 'launches', r.get('launches_per_generate'), 'kernel', r.get('kernel'), 'parity', d.get('parity',{}).get('labels_equal'))
PY
}
R10="--model runtimeracer-wavernn --utts-per-gpu 8 --bits 10 --target 6000 --overlap 1000 --steps 3 --warmup 1 --cpu-seconds 0"
bench rr8 "WRNN_X=1" "$R10"
bench rr8unsl "WRNN_PERSIST_SLICE=0" "$R10"
bench c4 "WRNN_X=1" "--utts-per-gpu 8 --steps 3 --warmup 1 --cpu-seconds 0"
exit $rc
