#!/bin/bash
# Measurement pass for the committed profiles: rocprofv3 kernel-trace summaries of the bench
# command and the FETCH_SIZE / WRITE_SIZE PMC passes (one counter per run) of the dominant
# persistent kernel, per workload. Every step has its own time limit; stops at the first failure.
# Usage: WORKLOADS="c2 c4" STEPS=pmc,prof bash tools/measure.sh   (outputs under gpurun_out/measure/)
set -u
O=gpurun_out/measure
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
P="/usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0"
# workload -> bench arguments and the kernel its PMC passes count (tools/pmc_traffic.py WORKLOADS)
declare -A ARGS=([c2]="" [c4]="--utts-per-gpu 8" [c3]="--mode MOL" [rr]="--model runtimeracer-wavernn --bits 9" [gen]="--model geneing-wavernn --mode BITS --bits 10")
declare -A KRE=([c2]="k_persist<" [c4]="k_persist_wide" [c3]="k_persist<" [rr]="k_persist_rr<" [gen]="k_persist_gen<")
for m in ${WORKLOADS:-c2 c4}; do
  if [[ ,${STEPS:-pmc,prof}, == *,prof,* ]]; then
    run prof_$m 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_$m" -o run --output-format csv -- $P ${ARGS[$m]}
  fi
  if [[ ,${STEPS:-pmc,prof}, == *,pmc,* ]]; then
    run pmc_fetch_$m 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "${KRE[$m]}" -d "$PWD/$O/pmc_fetch_$m" -o run --output-format csv -- $P --no-timing ${ARGS[$m]}
    run pmc_write_$m 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "${KRE[$m]}" -d "$PWD/$O/pmc_write_$m" -o run --output-format csv -- $P --no-timing ${ARGS[$m]}
  fi
done
exit 0
