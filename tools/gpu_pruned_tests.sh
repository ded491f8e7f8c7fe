set -u
mkdir -p gpurun_out/pp
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -v -s -rA --timeout 300 --timeout-method thread tests/test_gpu_trained.py tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_logits.py -k "pruned" > gpurun_out/pp/tests.log 2>&1
rc=$?
grep -E "rows diverged|near-tie check" gpurun_out/pp/tests.log | head -20
grep -E "passed|failed" gpurun_out/pp/tests.log | tail -1
exit $rc
