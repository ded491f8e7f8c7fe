set -u
O=gpurun_out/ab_ring; mkdir -p $O; export PYTHONUNBUFFERED=1
for mode in 1 0; do
  WRNN_P1_RING=$mode WRNN_PHASE_STEP=600 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $O/phase_$mode.log 2>&1 || exit $?
  WRNN_P1_RING=$mode timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_$mode.log 2>&1 || exit $?
  echo "== ring=$mode"; grep -E "^  (A|hop|B|C|D|sample|gru1|fc3)" $O/phase_$mode.log
  python3 -c "
import json,sys
for l in open('$O/bench_$mode.log'):
    if l.startswith('{'): d=json.loads(l); print('ring=$mode', 'ms %.2f' % d['ms_per_step'], 'us/step %.3f' % d['roofline']['us_per_step'])"
done
