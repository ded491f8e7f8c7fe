#!/bin/bash
# fc3 in float64 (tools/variants/fc3_f64.py) against the product build on the trained-like
# full-size cases: the c2pk sweep cases (near-tie analysis per diverged row,
# one JSON line per utterance) and the peaked reference fixtures on the register-resident kernel,
# then the C2 step time. Outputs gpurun_out/r06/fc3f64/.
set -u
O=gpurun_out/r06/fc3f64
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$PWD/exp/v_fc3f64/real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so
P=$PWD/real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so
PT="python -u -m pytest -v -s -rA --timeout 300 --timeout-method thread"
for tag in product f64; do
  lib=$P; [ $tag = f64 ] && lib=$V
  WRNN_LIB=$lib WRNN_SWEEP_OUT=$O/sweep_$tag.jsonl timeout -k 10 700 $PT tests/test_gpu_sweep.py -k c2pk > $O/sweep_$tag.log 2>&1
  rc=$?; echo "sweep $tag rc=$rc"; [ $rc -gt 1 ] && exit $rc
  WRNN_LIB=$lib timeout -k 10 600 $PT tests/test_gpu_trained.py -k "peaked and persist" > $O/trained_$tag.log 2>&1
  rc=$?; echo "trained $tag rc=$rc"; [ $rc -gt 1 ] && exit $rc
  WRNN_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/c2_$tag.log 2>&1
  rc=$?; echo "c2 $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  WRNN_LIB=$lib WRNN_PERSIST_WIDE=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --bits 10 --target 3000 --overlap 1500 > $O/u10reg_$tag.log 2>&1
  rc=$?; echo "u10reg $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
grep -h "rows diverged\|near-tie check" $O/*.log | head -40
exit 0
