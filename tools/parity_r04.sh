#!/bin/bash
# Round-4 full-size parity sweep on one MI355X (tools/parity_sweep.py): default-init and
# trained-like (peaked) weights at C2, peaked at the C4 per-GPU shape; one JSON line per check.
set -u
O=gpurun_out/r04/parity_sweep
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/parity_sweep.py 4 default 1 > $O/c2_default.jsonl 2> $O/c2_default.err || exit $?
timeout -k 10 300 python tools/parity_sweep.py 4 peaked 1 > $O/c2_peaked.jsonl 2> $O/c2_peaked.err || exit $?
timeout -k 10 300 python tools/parity_sweep.py 2 peaked 8 > $O/c4_peaked.jsonl 2> $O/c4_peaked.err || exit $?
cat $O/*.jsonl
