#!/bin/bash
# The full-size sweep gate with every case (WRNN_SWEEP_ALL=1) on the final build: one JSON line
# per utterance in gpurun_out/r06/sweep/sweep.jsonl.
set -u
O=gpurun_out/r06/sweep
mkdir -p $O
export PYTHONUNBUFFERED=1
WRNN_SWEEP_ALL=1 WRNN_SWEEP_OUT=$O/sweep.jsonl timeout -k 10 1000 python -u -m pytest -v -s -rA --timeout 400 --timeout-method thread tests/test_gpu_sweep.py > $O/sweep.log 2>&1
rc=$?
grep -E "passed|failed" $O/sweep.log | tail -1
exit $rc
