set -u
mkdir -p gpurun_out/rrmol
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread tests/test_gpu_rotation.py -k "mol" > gpurun_out/rrmol/tests.log 2>&1 || { tail -30 gpurun_out/rrmol/tests.log; exit 1; }
tail -3 gpurun_out/rrmol/tests.log
for rot in 0 1; do
  WRNN_PERSIST_ROT=$rot timeout -k 10 120 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --mode MOL > gpurun_out/rrmol/rot$rot.log 2>&1 || exit 1
  grep '^{' gpurun_out/rrmol/rot$rot.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot', $rot, d['value'], d['roofline'].get('us_per_step'), d['ms_per_step'], d['roofline'].get('rotation'))"
done
RATES="7.42,6.3 7.42,6.0 7.42,6.6 7.42,6.9" BENCH_ARGS="--model runtimeracer-wavernn --mode MOL" TAGS=.rrmol bash tools/rot_tune.sh
