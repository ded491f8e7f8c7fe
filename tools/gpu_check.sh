#!/bin/bash
# One gpurun call: parity tests, smoke, bench, each under its own time limit. Stops on any
# crash / timeout (exit codes other than 0 and pytest's 1 = "tests failed").
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-parity,smoke,bench}
[[ ,$STEPS, == *,parity,* ]] && run parity 600 python -m pytest tests/test_gpu_parity.py -q -x -rA ${PARITY_ARGS:-}
[[ ,$STEPS, == *,gputests,* ]] && run gputests 1000 python -u -m pytest tests -m gpu -v -rA --timeout 240 --timeout-method thread -k "${GPUTEST_K:-}" ${GPUTEST_ARGS:-}
[[ ,$STEPS, == *,phase,* ]] && run phase 300 env WRNN_PHASE_STEP=${PHASE_STEP:-600} python bench.py --steps 1 --warmup 0 --cpu-seconds 0
[[ ,$STEPS, == *,smoke,* ]] && run smoke 300 python __graft_entry__.py smoke
[[ ,$STEPS, == *,bench,* ]] && run bench 600 python bench.py --steps 3 --warmup 1 --cpu-seconds ${CPU_SECONDS:-10}
[[ ,$STEPS, == *,bench_c4,* ]] && run bench_c4 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
[[ ,$STEPS, == *,rehearse,* ]] && run rehearse 600 env WRNN_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --cpu-seconds ${CPU_SECONDS:-10}
[[ ,$STEPS, == *,prof,* ]] && run prof 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-timing
exit 0
