#!/bin/bash
# A/B of two library builds over the persistent-kernel workloads (C2 RAW, C2 MOL,
# runtimeracer, geneing BITS, C4 wide), one bench per (workload, build). Usage:
#   tools/ab_matrix.sh exp/lib_a.so exp/lib_b.so
set -u
for w in "c2:" "mol:--mode MOL" "rr:--model runtimeracer-wavernn" \
         "gen:--model geneing-wavernn --mode BITS --bits 10" "c4:--utts-per-gpu 8"; do
  tag=${w%%:*} args=${w#*:}
  TAG=_$tag BENCH_ARGS="$args" bash tools/ab.sh "$@" || exit $?
done
