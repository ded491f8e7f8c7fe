#!/bin/bash
# x2-buffer change: C2 speed, the race stress, and the persistent-kernel test files
set -u
O=gpurun_out/x2; mkdir -p $O
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['value']), round(d['roofline']['us_per_step'],4), d['config']['lib_build'])" || exit 1; done
timeout -k 10 300 python -u tools/diag_sparse_race3.py 300 > $O/stress.log 2>&1; tail -1 $O/stress.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_trained.py tests/test_gpu_logits.py tests/test_gpu_rotation.py tests/test_gpu_fold_split.py > $O/tests.log 2>&1; tail -1 $O/tests.log
