set -u
mkdir -p gpurun_out/ph
export PYTHONUNBUFFERED=1
timeout -k 10 200 env WRNN_PHASE_STEP=300 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --utts-per-gpu 8 > gpurun_out/ph/c4.log 2>&1 || exit 1
timeout -k 10 200 env WRNN_PHASE_STEP=300 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --bits 10 --target 3000 --overlap 1500 --utts-per-gpu 8 > gpurun_out/ph/b10.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_plan.py > gpurun_out/ph/plan_tests.log 2>&1
echo plan rc=$?
