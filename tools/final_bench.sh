#!/bin/bash
# Round-end GPU pass: every bench line kept under profiles/, the GPU test suite and smoke(),
# each under its own time limit; stops at the first crash or timeout.
set -u
O=gpurun_out/final
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  if [ $rc -ne 0 ]; then tail -8 "$O/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python bench.py --steps 3 --warmup 1 --cpu-seconds 0"
S=${STEPS:-bench,mol,rr9,rr10,rrmol,gen,genmol,beta,c4,c4p,wide,tests,smoke}
[[ ,$S, == *,bench,* ]] && run bench 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 12
[[ ,$S, == *,mol,* ]] && run mol 300 $B --mode MOL
[[ ,$S, == *,rr9,* ]] && run rr9 300 $B --model runtimeracer-wavernn --bits 9
[[ ,$S, == *,rr10,* ]] && run rr10 300 $B --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000
[[ ,$S, == *,rrmol,* ]] && run rrmol 300 $B --model runtimeracer-wavernn --mode MOL
[[ ,$S, == *,gen,* ]] && run gen 300 $B --model geneing-wavernn --mode BITS --bits 10
[[ ,$S, == *,genmol,* ]] && run genmol 300 $B --model geneing-wavernn --mode MOL
[[ ,$S, == *,beta,* ]] && run beta 300 $B --model geneing-wavernn --mode RAW
[[ ,$S, == *,c4,* ]] && run c4 400 $B --utts-per-gpu 8
# wide launch only (WRNN_PERSIST_WIDE=1): the step-time curve over rows per XCD group
if [[ ,$S, == *,wide,* ]]; then
  for u in 1 2 4 7; do run wide_u$u 300 env WRNN_PERSIST_WIDE=1 $B --utts-per-gpu $u; done
fi
[[ ,$S, == *,c4p,* ]] && run c4p 300 $B --utts-per-gpu 1 --frames 1700
[[ ,$S, == *,tests,* ]] && run tests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[[ ,$S, == *,smoke,* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
