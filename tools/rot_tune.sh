# Rotation balance A/B: the C2 call time for planner rates WRNN_ROT_US="t_hi,t_lo" (µs per step of
# the 3-row / 2-row groups), interleaved rounds (BENCH_ARGS: e.g. --mode MOL; TAGS: log name suffix)
set -u
mkdir -p gpurun_out/rot
for r in 1 2; do
  for rates in ${RATES:-"5.91,5.22" "5.91,5.28" "5.91,5.35" "5.91,5.42"}; do
    WRNN_ROT_US=$rates timeout -k 10 120 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/rot/$rates${TAGS:-}.r$r.log 2>&1 || { echo "fail $rates"; exit 1; }
    python - gpurun_out/rot/$rates${TAGS:-}.r$r.log "$rates${TAGS:-}" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[2], 'us/step %.3f' % r['us_per_step'], 'ms/call %.2f' % d['ms_per_step'], r.get('rotation', {}).get('steps_per_launch_hi_rows'), r.get('rotation', {}).get('steps_per_launch_lo_rows'))
PY
  done
done
