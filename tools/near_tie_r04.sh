#!/bin/bash
# The two label differences of the round-4 peaked parity sweep (profiles/r04/parity_sweep/):
# teacher-forced logits at the differing decision against its top-2 gap.
set -u
O=gpurun_out/r04/near_tie
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/near_tie_gpu.py peaked 102 302 1 0 16 10850 > $O/c2_case2.json 2> $O/c2_case2.err || exit $?
timeout -k 10 300 python tools/near_tie_gpu.py peaked 101 301 8 7 6 11017 > $O/c4_case1.json 2> $O/c4_case1.err || exit $?
cat $O/*.json
