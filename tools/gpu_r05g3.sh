set -u
mkdir -p gpurun_out/genmol
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread tests/test_gpu_rotation.py -k "mol or geneing" > gpurun_out/genmol/tests.log 2>&1 || { tail -30 gpurun_out/genmol/tests.log; exit 1; }
tail -3 gpurun_out/genmol/tests.log
for rot in 0 1; do
  WRNN_PERSIST_ROT=$rot timeout -k 10 120 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model geneing-wavernn --mode MOL > gpurun_out/genmol/rot$rot.log 2>&1 || exit 1
  grep '^{' gpurun_out/genmol/rot$rot.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot', $rot, d['value'], d['roofline'].get('us_per_step'), d['ms_per_step'])"
done
RATES="2.6,2.06 2.6,1.95 2.6,2.15 2.6,2.25" BENCH_ARGS="--model geneing-wavernn --mode MOL" TAGS=.gmol bash tools/rot_tune.sh
