#!/bin/bash
# Wide-row launch bring-up: parity tests, C4 bench, phase stamps. Each step time-limited;
# stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-wide,c4,phase}
[[ ,$STEPS, == *,wide,* ]] && run wide 400 python -u -m pytest tests/test_gpu_wide.py -v -rA --timeout 200 --timeout-method thread -x
[[ ,$STEPS, == *,c4,* ]] && run c4 300 python bench.py --utts-per-gpu 8 --steps 3 --warmup 1 --cpu-seconds 0
[[ ,$STEPS, == *,phase,* ]] && run phase 300 env WRNN_PHASE_STEP=${PHASE_STEP:-600} WRNN_PERSIST_WIDE=1 python bench.py --utts-per-gpu 8 --steps 1 --warmup 0 --cpu-seconds 0
[[ ,$STEPS, == *,full,* ]] && run full 600 python -u -m pytest tests/test_gpu_fullsize.py -v -rA --timeout 240 --timeout-method thread
exit 0
