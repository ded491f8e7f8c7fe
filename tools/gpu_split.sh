#!/bin/bash
# Fold-split (wrnn_set_fold_ranges) GPU checks: its tests, the 1-GPU latency table and a 2-rank
# gloo rehearsal of bench.py --split folds (both ranks on the one GPU: timings meaningless).
set -u
O=gpurun_out/split
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread \
  tests/test_gpu_fold_split.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/split_latency.py > $O/latency.jsonl 2> $O/latency.err || { tail -20 $O/latency.err; exit 1; }
cat $O/latency.jsonl | cut -c1-400
timeout -k 10 300 env WRNN_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --split folds --steps 2 --warmup 1 \
  --cpu-seconds 5 > $O/rehearse.log 2>&1 || { tail -30 $O/rehearse.log; exit 1; }
tail -c 1500 $O/rehearse.log
