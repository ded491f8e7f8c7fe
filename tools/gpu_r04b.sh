#!/bin/bash
# Round-4 GPU call: runtimeracer wide tests, k_persist in-kernel-noise A/B, rr bench.
set -u
O=gpurun_out/r04/${TAG:-b}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -4 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
S=${STEPS:-rrtests,ab,rrbench}
[[ ,$S, == *,rrtests,* ]] && run rrtests 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_wide_rr.py -k "golden or every"
if [[ ,$S, == *,ab,* ]]; then
  i=0
  for lib in exp/lib_base.so exp/lib_nlicm.so exp/lib_nz1.so exp/lib_base.so exp/lib_nz1.so; do
    i=$((i + 1))
    n=$(basename $lib .so)_$i
    run ab_$n 200 env WRNN_LIB=$PWD/$lib python bench.py --steps 3 --warmup 1 --cpu-seconds 0
    grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' $O/ab_$n.log | tr '\n' ' '; echo
  done
  run ab_nz1_parity 300 env WRNN_LIB=$PWD/exp/lib_nz1.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "c2_full or c4"
fi
if [[ ,$S, == *,abrr,* ]]; then
  i=0
  for lib in exp/lib_rrv1.so exp/lib_rrv2.so exp/lib_rrv1.so exp/lib_rrv2.so; do
    i=$((i + 1))
    n=$(basename $lib .so)_$i
    run abrr_$n 300 env WRNN_LIB=$PWD/$lib python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8
    grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' $O/abrr_$n.log | tr '\n' ' '; echo
  done
fi
if [[ ,$S, == *,abps,* ]]; then
  # rr wide kernel: serialized vs batched partial-sum reads (exp/lib_ps0 vs exp/lib_ps1)
  i=0
  for lib in exp/lib_ps0.so exp/lib_ps1.so exp/lib_ps0.so exp/lib_ps1.so; do
    i=$((i + 1))
    n=$(basename $lib .so)_$i
    run abps_$n 300 env WRNN_LIB=$PWD/$lib python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8
    grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' $O/abps_$n.log | tr '\n' ' '; echo
  done
  run phase_ps1 300 env WRNN_LIB=$PWD/exp/lib_ps1.so WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8
fi
[[ ,$S, == *,widetests,* ]] && run widetests 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_fullsize.py -k "wide or c4"
if [[ ,$S, == *,abfw,* ]]; then
  # fatchord wide kernel: pairwise vs batched partial-sum reads (exp/lib_fw0 vs exp/lib_fw1), C4
  i=0
  for lib in exp/lib_fw0.so exp/lib_fw1.so exp/lib_fw0.so exp/lib_fw1.so; do
    i=$((i + 1))
    n=$(basename $lib .so)_$i
    run abfw_$n 300 env WRNN_LIB=$PWD/$lib python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
    grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*\|"stages_us": {[^}]*}' $O/abfw_$n.log | tr '\n' ' '; echo
  done
  run phase_fw1 300 env WRNN_LIB=$PWD/exp/lib_fw1.so WRNN_PHASE_STEP=600 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --utts-per-gpu 8
fi
if [[ ,$S, == *,wsrc,* ]]; then
  # where do the wide kernel's HBM writes come from? WRITE_SIZE of the shipped build against
  # builds without the ring's noise stores (wnn) / P1 stores (wnp); outputs of those are wrong
  # (each build copied over the in-tree library of this scratch copy: under WRNN_LIB the
  # profiler recorded no dispatches)
  L=real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so
  cp $L exp/lib_shipped.so
  for lib in exp/lib_shipped.so ${WSRC_LIBS:-exp/lib_wnn.so exp/lib_wnp.so}; do
    n=$(basename $lib .so)
    cp $lib $L
    run wsrc_$n 240 env WRNN_WIDE_ALLOW_SCRATCH=1 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_persist_wide -d "$PWD/$O/wsrc_$n" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-timing --utts-per-gpu 8
    python3 -c "
import csv,collections,sys
d=collections.defaultdict(float); n=set()
for r in csv.DictReader(open('$O/wsrc_$n/run_counter_collection.csv')):
    if 'k_persist_wide' in r['Kernel_Name']: d[r['Counter_Name']]+=float(r['Counter_Value']); n.add(r['Dispatch_Id'])
print('$n', {k: v*1024/1e9/len(n) for k,v in d.items()}, 'GB per launch,', len(n), 'launches')" | tee -a $O/steps.log
  done
  # and the C4 timing of each (in-place copies again)
  for lib in exp/lib_shipped.so ${WSRC_LIBS:-} exp/lib_shipped.so ${WSRC_LIBS:-}; do
    n=$(basename $lib .so)
    cp $lib $L
    run wsab_$n 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --utts-per-gpu 8
    grep -o '"value": [0-9.]*\|"stages_us": {[^}]*}' $O/wsab_$n.log | tr '\n' ' ' | tee -a $O/steps.log; echo | tee -a $O/steps.log
  done
  cp exp/lib_shipped.so $L
fi
if [[ ,$S, == *,abgen,* ]]; then
  # generic A/B: AB_LIBS (space-separated builds), alternated twice, bench args AB_ARGS
  i=0
  for lib in ${AB_LIBS} ${AB_LIBS}; do
    i=$((i + 1))
    n=$(basename $lib .so)_$i
    run abgen_$n 300 env WRNN_LIB=$PWD/$lib python bench.py --steps 5 --warmup 2 --cpu-seconds 0 ${AB_ARGS:-}
    grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*\|"stages_us": {[^}]*}' $O/abgen_$n.log | tr '\n' ' ' | tee -a $O/steps.log; echo | tee -a $O/steps.log
  done
fi
[[ ,$S, == *,c2tests,* ]] && run c2tests 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_callback.py tests/test_gpu_logits.py
[[ ,$S, == *,rrbench,* ]] && run rrbench 500 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8
[[ ,$S, == *,rrbench0,* ]] && run rrbench0 600 env WRNN_PERSIST_WIDE=0 python bench.py --steps 1 --warmup 1 --cpu-seconds 0 --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8
exit 0
