#!/bin/bash
# Round-3 measurement pass on one MI355X box, each step under its own time limit; stops at the
# first crash / timeout. Outputs under gpurun_out/r03/ (copied to profiles/r03/final/ after).
#   tests  : the whole -m gpu suite;  smoke : __graft_entry__.smoke()
#   bench  : default bench line (C2, CPU baseline, parity, logit gate)
#   c4     : --utts-per-gpu 8;  rehearse : the N>1 path with 2 ranks on one GPU (gloo)
#   phase  : C2 phase stamps (WRNN_PHASE_STEP=600)
#   pmc    : tools/pmc_r03.sh (FETCH_SIZE / WRITE_SIZE / SQ passes, c2 and c4) + kernel-trace stats
set -u
O=gpurun_out/r03
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
S=${STEPS:-tests,smoke,bench,c4,rehearse,phase,pmc}
[[ ,$S, == *,tests,* ]] && run tests 700 python -u -m pytest tests -m gpu -v -rA --timeout 240 --timeout-method thread
[[ ,$S, == *,smoke,* ]] && run smoke 300 python __graft_entry__.py smoke
[[ ,$S, == *,bench,* ]] && run bench 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 12
[[ ,$S, == *,c4,* ]] && run c4 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
[[ ,$S, == *,rehearse,* ]] && run rehearse 400 env WRNN_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --cpu-seconds 10
[[ ,$S, == *,phase,* ]] && run phase 200 env WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0
[[ ,$S, == *,pmc,* ]] && STEPS=pmc,prof bash tools/pmc_r03.sh
exit 0
