#!/bin/bash
# Near-tie analysis of label differences in the runtimeracer wide-kernel parity sweep
# (profiles/r04/parity_sweep/rr8_*.jsonl): teacher-forced logits at the first differing decision.
set -u
O=gpurun_out/r04/near_tie_rr
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/near_tie_gpu.py default 101 301 8 7 27 6723 runtimeracer > $O/default_case1_u7.json 2> $O/a.err || exit $?
timeout -k 10 300 python tools/near_tie_gpu.py peaked 100 300 8 0 10 326 runtimeracer > $O/peaked_case0_u0.json 2> $O/b.err || exit $?
timeout -k 10 300 python tools/near_tie_gpu.py peaked 100 300 8 7 12 5599 runtimeracer > $O/peaked_case0_u7.json 2> $O/c.err || exit $?
timeout -k 10 300 python tools/near_tie_gpu.py peaked 101 301 8 0 7 1486 runtimeracer > $O/peaked_case1_u0.json 2> $O/d.err || exit $?
cat $O/*.json
