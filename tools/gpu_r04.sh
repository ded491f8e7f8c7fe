#!/bin/bash
# Round-4 GPU steps, each under its own time limit; stops at the first crash / timeout.
# Outputs under gpurun_out/r04/<tag>/ (copied to profiles/r04/ after).
#   STEPS: comma list of  trained, tests (the whole -m gpu suite), smoke, bench, c4, rehearse,
#          phase (C2 phase stamps), phase_c4, prof (rocprof kernel-trace c2 + c4)
set -u
O=gpurun_out/r04/${TAG:-run}
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
PT="python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread"
S=${STEPS:-tests,smoke,bench,c4}
[[ ,$S, == *,trained,* ]] && run trained 600 $PT tests/test_gpu_trained.py tests/test_gpu_logits.py -k "peaked or chaotic or trained" -s
[[ ,$S, == *,gpufile,* ]] && run gpufile 600 $PT ${GPUFILES} -s
[[ ,$S, == *,tests,* ]] && run tests 900 $PT tests -m gpu
[[ ,$S, == *,smoke,* ]] && run smoke 300 python __graft_entry__.py smoke
[[ ,$S, == *,bench,* ]] && run bench 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 12
[[ ,$S, == *,c4,* ]] && run c4 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
[[ ,$S, == *,rehearse,* ]] && run rehearse 400 env WRNN_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --cpu-seconds 10
[[ ,$S, == *,phase,* ]] && run phase 200 env WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0
[[ ,$S, == *,phase_c4,* ]] && run phase_c4 200 env WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --utts-per-gpu 8
[[ ,$S, == *,prof,* ]] && run prof_c2 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_c2" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0
[[ ,$S, == *,prof,* ]] && run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_c4" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
exit 0
