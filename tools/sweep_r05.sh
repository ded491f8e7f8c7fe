#!/bin/bash
# Round-5 sweep on one MI355X box: the bench lines of the other topologies / modes
# (tools/final_bench.sh steps) and the configs[4]-shape end-to-end demo on one GPU; outputs under
# gpurun_out/final/ (copied to profiles/r05/sweep/).
set -u
STEPS=mol,rr9,rr10,rrmol,gen,genmol,beta,c4p bash tools/final_bench.sh || exit $?
timeout -k 10 400 python real-time-voice-cloning_amd/demo_cli.py --random-weights 0 --seed 0 --utterances 8 --max-frames 400 > gpurun_out/final/e2e.log 2>&1
echo "e2e rc=$?"
tail -3 gpurun_out/final/e2e.log
