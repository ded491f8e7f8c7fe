#!/bin/bash
# P1 forms on one box: parity (incl. full size), then the C2 bench with the in-kernel ring
# (default), the k_p1_expand stream (WRNN_P1_RING=0) and the round-1 per-(step, row) GEMM
# (WRNN_P1_FRAMES=0), then a rocprof kernel trace of the default. Stops at the first crash.
set -u
O=gpurun_out/ab_p1
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -4 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python bench.py --steps 3 --warmup 1 --cpu-seconds 0"
S=${STEPS:-parity,fullsize,ring,stream,gemm,prof}
[[ ,$S, == *,parity,* ]] && run parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 240 --timeout-method thread
[[ ,$S, == *,fullsize,* ]] && run fullsize 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q -rf --timeout 240 --timeout-method thread
[[ ,$S, == *,ring,* ]] && run ring 300 $B
[[ ,$S, == *,stream,* ]] && run stream 300 env WRNN_P1_RING=0 $B
[[ ,$S, == *,gemm,* ]] && run gemm 300 env WRNN_P1_FRAMES=0 $B
[[ ,$S, == *,c4,* ]] && run c4 300 $B --utts-per-gpu 8
[[ ,$S, == *,prof,* ]] && run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-timing
exit 0
