# Interleaved A/B of library builds on one box: ROUNDS x (each lib: one short bench), C2 µs per
# step from the bench line. Usage: ROUNDS=3 tools/ab_r05.sh exp/lib_a.so exp/lib_b.so ...
set -u
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    WRNN_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${BSTEPS:-5} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} \
      > gpurun_out/ab/$n.r$r.bench 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$n bench rc=$rc"; tail -5 gpurun_out/ab/$n.r$r.bench; exit $rc; }
    python - "$n" "$r" <<'PY'
import json,sys
for l in open('gpurun_out/ab/%s.r%s.bench' % (sys.argv[1], sys.argv[2])):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1], 'round', sys.argv[2], 'value %.0f' % d['value'], 'us/step %.3f' % d['roofline']['us_per_step'], 'labels_equal', d.get('parity', {}).get('labels_equal'))
PY
  done
done
