#!/bin/bash
# Round-3 counter passes behind the roofline claims, one rocprofv3 run per
# pass (counter slots per pass: MI355X_MICROARCH.md "rocprofv3 PMC slots"), each under its own
# time limit; stops at the first failure. Outputs under gpurun_out/pmc3/.
#   list  : rocprofv3 -L (the counters this ROCm exposes on gfx950)
#   per workload (c2: k_persist, C2; c4: k_persist_wide + k_persist + k_gemm, C4 per GPU):
#     fetch : FETCH_SIZE            write : WRITE_SIZE
#     sq    : SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
#             SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE + GRBM_GUI_ACTIVE
set -u
O=gpurun_out/pmc3
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
P="/usr/bin/python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-timing"
declare -A ARGS=([c2]="" [c4]="--utts-per-gpu 8")
declare -A KRE=([c2]="k_persist<" [c4]="k_persist|k_gemm")
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
[[ ,${STEPS:-list,pmc}, == *,list,* ]] && run list 120 rocprofv3 -L
for m in ${WORKLOADS:-c2 c4}; do
  if [[ ,${STEPS:-list,pmc}, == *,pmc,* ]]; then
    run ${m}_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "${KRE[$m]}" -d "$PWD/$O/${m}_fetch" -o run --output-format csv -- $P ${ARGS[$m]}
    run ${m}_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "${KRE[$m]}" -d "$PWD/$O/${m}_write" -o run --output-format csv -- $P ${ARGS[$m]}
    run ${m}_sq 240 rocprofv3 --pmc $SQ --kernel-include-regex "${KRE[$m]}" -d "$PWD/$O/${m}_sq" -o run --output-format csv -- $P ${ARGS[$m]}
  fi
  if [[ ,${STEPS:-list,pmc}, == *,prof,* ]]; then
    run ${m}_prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/${m}_prof" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 ${ARGS[$m]}
  fi
done
exit 0
