#!/bin/bash
# Round-4 full-size parity sweep on one MI355X (tools/parity_sweep.py): default-init and
# trained-like (peaked) weights at C2, peaked at the C4 per-GPU shape, and the runtimeracer
# defaults at the 8-utterance shape (its wide kernel); one JSON line per check.
# STEPS=rr runs only the runtimeracer part.
set -u
O=gpurun_out/r04/parity_sweep
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ "${STEPS:-all}" != rr ]; then
timeout -k 10 300 python tools/parity_sweep.py 4 default 1 > $O/c2_default.jsonl 2> $O/c2_default.err || exit $?
timeout -k 10 300 python tools/parity_sweep.py 4 peaked 1 > $O/c2_peaked.jsonl 2> $O/c2_peaked.err || exit $?
timeout -k 10 300 python tools/parity_sweep.py 2 peaked 8 > $O/c4_peaked.jsonl 2> $O/c4_peaked.err || exit $?
fi
timeout -k 10 300 python tools/parity_sweep.py 2 default 8 runtimeracer > $O/rr8_default.jsonl 2> $O/rr8_default.err || exit $?
timeout -k 10 300 python tools/parity_sweep.py 2 peaked 8 runtimeracer > $O/rr8_peaked.jsonl 2> $O/rr8_peaked.err || exit $?
cat $O/*.jsonl
