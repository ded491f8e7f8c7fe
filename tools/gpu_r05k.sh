# round 5: rotated runtimeracer register-resident launches -- equality tests, then the 9-bit C2
# shape's single-launch step times at 2 / 3 rows per group and the rotated call
set -o pipefail
O=gpurun_out/rrrot
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_rotation.py -k runtimeracer -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -6 $O/tests.log; [ $rc -eq 0 ] || exit $rc
A="--steps 3 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 9 ${EXTRA:-}"
for nr in 2 3; do
  WRNN_PERSIST_ROT=0 WRNN_PERSIST_NR_MAX=$nr timeout -k 10 120 python bench.py $A > $O/nr$nr.log 2>&1 || exit 1
done
for r in ${RATES:-default}; do
  if [ $r = default ]; then timeout -k 10 120 python bench.py $A > $O/rot_$r.log 2>&1 || exit 1
  else WRNN_ROT_US=$r timeout -k 10 120 python bench.py $A > $O/rot_$r.log 2>&1 || exit 1; fi
done
for f in $O/nr2.log $O/nr3.log $O/rot_*.log; do
  grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', round(d['value']), round(r['us_per_step'],3), r.get('launches_per_generate'), (r.get('rotation') or {}).get('steps_per_launch_hi_rows'))"
done
