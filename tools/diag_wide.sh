set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 WRNN_DEBUG_WHERE=1
timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --utts-per-gpu 8 > gpurun_out/d_c4.log 2>&1; echo "c4 rc=$?"
grep -E "timeout|site" gpurun_out/d_c4.log | head -5
WRNN_WIDE_FORCE_XV=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --utts-per-gpu 7 > gpurun_out/d_xv16.log 2>&1; echo "xv16 rc=$?"
grep -E "timeout|site|us_per_step" gpurun_out/d_xv16.log | head -5
python - <<'PY'
import json
for f in ('gpurun_out/d_c4.log','gpurun_out/d_xv16.log'):
    for l in open(f):
        if l.startswith('{'):
            d=json.loads(l); print(f, d['config']['engine'], d['roofline'].get('us_per_step'), d['config'].get('fallback_reason'))
PY
