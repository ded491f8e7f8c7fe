#!/bin/bash
# Kernel A/B on one box: for each library build given (paths), one phase-stamped config-2 run
# and a short bench, each under its own time limit. Usage: tools/ab.sh exp/lib_a.so exp/lib_b.so
set -u
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for lib in "$@"; do
  n=$(basename "$lib" .so)${TAG:-}
  WRNN_LIB=$PWD/$lib WRNN_PHASE_STEP=${PHASE_STEP:-600} timeout -k 10 200 \
    python bench.py --steps 1 --warmup 0 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab/$n.phase 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n phase rc=$rc"; tail -5 gpurun_out/ab/$n.phase; exit $rc; }
  WRNN_LIB=$PWD/$lib timeout -k 10 200 \
    python bench.py --steps ${BSTEPS:-3} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab/$n.bench 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n bench rc=$rc"; tail -5 gpurun_out/ab/$n.bench; exit $rc; }
  echo "== $n"; grep -E "^  (A|hop|B|C|D|sample|gru1|fc3)" gpurun_out/ab/$n.phase
  python - "$n" <<'PY'
import json,sys
for l in open('gpurun_out/ab/%s.bench' % sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1], 'value %.0f' % d['value'], 'us/step %.3f' % d['roofline']['us_per_step'])
PY
done
