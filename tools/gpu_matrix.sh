#!/bin/bash
# One gpurun call: bench lines for the other BASELINE configs + PMC passes on the persistent
# kernel. Every GPU step has its own time limit; the script stops at the first crash/timeout.
set -u
mkdir -p gpurun_out/matrix
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/matrix/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/matrix/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/matrix/steps.log
  tail -5 "gpurun_out/matrix/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python bench.py --steps 2 --warmup 1 --cpu-seconds 0"
[[ ,$STEPS, == *,mol,* ]] && run mol 300 $B --mode MOL
[[ ,$STEPS, == *,rr9,* ]] && run rr9 300 $B --model runtimeracer-wavernn --bits 9
[[ ,$STEPS, == *,gen,* ]] && run gen 300 $B --model geneing-wavernn --bits 10
[[ ,$STEPS, == *,rr10,* ]] && run rr10 300 $B --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000
[[ ,$STEPS, == *,c4,* ]] && run c4 600 $B --utts-per-gpu 8
[[ ,$STEPS, == *,c4p,* ]] && run c4p 600 $B --utts-per-gpu 1 --frames 1700
P="/usr/bin/python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-timing"
[[ ,$STEPS, == *,prof_rr,* ]] && run prof_rr 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/matrix/prof_rr" -o run --output-format csv -- $P --model runtimeracer-wavernn --bits 9
[[ ,$STEPS, == *,prof_gen,* ]] && run prof_gen 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/matrix/prof_gen" -o run --output-format csv -- $P --model geneing-wavernn --bits 10
[[ ,$STEPS, == *,pmc,* ]] && run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_persist -d "$PWD/gpurun_out/matrix/pmc_fetch" -o run --output-format csv -- $P
[[ ,$STEPS, == *,pmc,* ]] && run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_persist -d "$PWD/gpurun_out/matrix/pmc_write" -o run --output-format csv -- $P
exit 0
