# Per-step cost of k_persist by rows per group (WRNN_PERSIST_NR_MAX forces the variant):
# 16 rows (900 frames) at 2 and at 3 rows per group (padding rows), 18 rows at 3.
set -u
mkdir -p gpurun_out/nr
for cfg in "900 2" "900 3" "1000 3" "1000 4"; do
  set -- $cfg
  WRNN_PERSIST_NR_MAX=$2 timeout -k 10 120 python bench.py --frames $1 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/nr/f$1_nr$2.log 2>&1 || { echo "fail $cfg"; tail -3 gpurun_out/nr/f$1_nr$2.log; exit 1; }
  python - gpurun_out/nr/f$1_nr$2.log "$cfg" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[2], 'us/step %.3f' % r['us_per_step'], 'launches', r.get('launches_per_generate'), 'value %.0f' % d['value'])
PY
done
