set -u
mkdir -p gpurun_out/genrot
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread tests/test_gpu_rotation.py -k "runtimeracer_geneing" tests/test_gpu_plan.py > gpurun_out/genrot/tests.log 2>&1 || { tail -30 gpurun_out/genrot/tests.log; exit 1; }
tail -3 gpurun_out/genrot/tests.log
for rot in 0 1; do
  WRNN_PERSIST_ROT=$rot timeout -k 10 120 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model geneing-wavernn --mode BITS --bits 10 > gpurun_out/genrot/rot$rot.log 2>&1 || exit 1
  grep '^{' gpurun_out/genrot/rot$rot.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot', $rot, d['value'], d['roofline'].get('us_per_step'), d['ms_per_step'])"
done
RATES="3.91,3.26 3.91,3.1 3.91,3.4 3.91,2.95" BENCH_ARGS="--model geneing-wavernn --mode BITS --bits 10" TAGS=.gen bash tools/rot_tune.sh
