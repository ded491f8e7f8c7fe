#!/bin/bash
# Round-6 measurement pass on one MI355X box: every step under its own time limit, stops at the
# first crash / timeout. Outputs under gpurun_out/r06/<TAG>/ (copied to profiles/r06/<TAG>/ after).
#   tests    : the whole -m gpu suite            smoke : __graft_entry__.smoke()
#   pmc      : FETCH_SIZE / WRITE_SIZE / SQ passes of the dominant kernels (C2, C4, rr), each its own
#              rocprofv3 run; folded on the box into gpurun_out/r06/<TAG>/pmc_traffic.json with
#              this library's build id (bench lines then name counters of the binary they time)
#   bench    : default line (C2, CPU baseline, parity, logit gate), counters from the pass above
#   c4       : --utts-per-gpu 8                  rr    : runtimeracer 10-bit defaults, 8 utts
#   b10      : fatchord 10-bit defaults (3000 / 1500), 8 utts (the 1024-class wide slices)
#   gen      : geneing 10-bit C2 shape (the rotated k_persist_gen), rotation off and on; the other
#              rotated C2-shape lines: geneing MOL, runtimeracer MOL and 9-bit, fatchord MOL (C3)
# (three gpurun calls: STEPS=tests,smoke | pmc,bench,c4,rr,b10 | rehearse,phase,prof -- with
#  WRNN_PMC_TRAFFIC pointing the later benches at the pass's pmc_traffic.json)
#   rehearse : the N>1 path with 2 ranks on one GPU (gloo), CPU baseline + parity on rank 0
#   phase    : C2 phase stamps                   prof  : rocprofv3 kernel-trace --stats of c2, c4, rr
set -u
T=${TAG:-final}
O=gpurun_out/r06/$T
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
S=${STEPS:-tests,smoke,pmc,bench,c4,rr,b10,rehearse,phase,prof}
PT=${PT:-"python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread"}
RR="--model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8"
B10="--bits 10 --target 3000 --overlap 1500 --utts-per-gpu 8"
[[ ,$S, == *,tests,* ]] && run tests 900 $PT tests -m gpu
[[ ,$S, == *,smoke,* ]] && run smoke 300 python __graft_entry__.py smoke
if [[ ,$S, == *,pmc,* ]]; then
  P=$O/pmc
  mkdir -p $P
  python -c "import sys; sys.path[:0]=['.', 'real-time-voice-cloning_amd']; import bench; print(bench.lib_build_id())" > $P/lib_build
  B="/usr/bin/python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-timing"
  SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  for m in ${PMC_SET:-c2 c4 rr b10 gen u10 spc2}; do
    A=""; K="k_persist<"
    [ $m = gen ] && A="--model geneing-wavernn --mode BITS --bits 10" && K="k_persist_gen<"
    [ $m = c4 ] && A="--utts-per-gpu 8" && K="k_persist_wide<"
    [ $m = rr ] && A="$RR" && K="k_persist_wide_rr"
    [ $m = b10 ] && A="$B10" && K="k_persist_wide<"
    [ $m = u10 ] && A="--bits 10 --target 3000 --overlap 1500" && K="k_persist_wide<"
    [ $m = spc2 ] && A="--prune 0.9 --sparse 1"
    run ${m}_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d "$PWD/$P/${m}_fetch" -o run --output-format csv -- $B $A
    run ${m}_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d "$PWD/$P/${m}_write" -o run --output-format csv -- $B $A
    run ${m}_sq 240 rocprofv3 --pmc $SQ --kernel-include-regex "$K" -d "$PWD/$P/${m}_sq" -o run --output-format csv -- $B $A
  done
  run pmc_fold 120 python tools/pmc_traffic.py $P $O $O/pmc_traffic.json
  export WRNN_PMC_TRAFFIC=$PWD/$O/pmc_traffic.json
fi
[[ ,$S, == *,bench,* ]] && run bench 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 12
[[ ,$S, == *,c4,* ]] && run c4 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
[[ ,$S, == *,rr,* ]] && run rr 500 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 $RR
[[ ,$S, == *,b10,* ]] && run b10 500 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 $B10
if [[ ,$S, == *,gen,* ]]; then
  run gen 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model geneing-wavernn --mode BITS --bits 10
  run gen_norot 300 env WRNN_PERSIST_ROT=0 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model geneing-wavernn --mode BITS --bits 10
  run gen_mol 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model geneing-wavernn --mode MOL
  run rr_mol 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --mode MOL
  run rr9 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 9
  run c3 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --mode MOL
fi
# the fork's default single-utterance fatchord shape (VERDICT r5 missing #2): one 1000-frame mel,
# 10 bits, target 3000 / overlap 1500 (45 rows x 6,000 steps) -- the default plan and the
# alternatives (register-resident only, wide only, no rotation)
U10="--bits 10 --target 3000 --overlap 1500"
if [[ ,$S, == *,u10,* ]]; then
  run u10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $U10
  run u10_reg 300 env WRNN_PERSIST_WIDE=0 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $U10
  run u10_wide 300 env WRNN_PERSIST_WIDE=1 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $U10
  run u10_norot 300 env WRNN_PERSIST_WIDE=0 WRNN_PERSIST_ROT=0 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $U10
  for nr in 1 2 3 4; do
    run u10_nr$nr 300 env WRNN_PERSIST_NR_MAX=$nr WRNN_PERSIST_WIDE=0 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 $U10
  done
fi
# pruned checkpoints: the sparse GPU tests, then 90 %-pruned bench lines at C2
# and at the 8-utterance shape, each beside the dense kernels on the same pruned weights
[[ ,$S, == *,sparse,* ]] && run sparse 600 $PT tests/test_gpu_sparse.py
if [[ ,$S, == *,sp,* ]]; then
  run sp_c2 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --prune 0.9
  run sp_c2_dense 300 env WRNN_SPARSE=0 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --prune 0.9
  run sp_c4 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --prune 0.9 --utts-per-gpu 8
  run sp_c4_dense 400 env WRNN_SPARSE=0 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --prune 0.9 --utts-per-gpu 8
  for nr in 1 2 3 4; do
    run sp_nr$nr 300 env WRNN_PERSIST_NR_MAX=$nr WRNN_PERSIST_ROT=0 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --prune 0.9
  done
fi
# planner rates: the 9-bit C2-shape step time at each rows-per-group variant
# (no rotation), then the per-build rate table from this pass's probes
if [[ ,$S, == *,rates,* ]]; then
  for nr in 1 2 3 4; do
    run nr$nr 300 env WRNN_PERSIST_NR_MAX=$nr WRNN_PERSIST_ROT=0 python bench.py --steps 3 --warmup 1 --cpu-seconds 0
  done
  run make_rates 60 python tools/make_rates.py $O/rates_mi355x.txt $O
fi
[[ ,$S, == *,rehearse,* ]] && run rehearse 400 env WRNN_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --cpu-seconds 10
[[ ,$S, == *,phase,* ]] && run phase 200 env WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0
if [[ ,$S, == *,prof,* ]]; then
  run prof_c2 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_c2" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0
  run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_c4" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
  run prof_rr 400 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_rr" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 $RR
  run prof_b10 400 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_b10" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 $B10
  run prof_u10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_u10" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --bits 10 --target 3000 --overlap 1500
  run prof_spc2 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_spc2" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --prune 0.9 --sparse 1
fi
# round-6 final lines: the fork's 10-bit single utterance, C2 on 90 %-pruned weights (planner's
# choice = dense, and the sparse instances forced), the 8-utterance shape on pruned weights
if [[ ,$S, == *,r6lines,* ]]; then
  run u10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --bits 10 --target 3000 --overlap 1500
  run spc2_auto 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --prune 0.9
  run spc2 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --prune 0.9 --sparse 1
  run spc4 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --prune 0.9 --utts-per-gpu 8
fi
exit 0
