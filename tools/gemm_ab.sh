#!/bin/bash
# GEMM A/B: rocprof kernel stats of a config-2 bench (3 steps) per library build exp/lib_<name>.so
# (kernels_gemm.hip built with -DWRNN_GEMM_WIDE_NT / -DWRNN_GEMM_WPE and linked with the other objects).
set -u
mkdir -p gpurun_out/gab
for n in "$@"; do
  WRNN_LIB=$PWD/exp/lib_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/gab/$n" -o run --output-format csv -- /usr/bin/python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-timing > gpurun_out/gab/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/gab/$n.log; exit 1; }
  grep -h "k_gemm<[24], 1" gpurun_out/gab/$n/run_kernel_stats.csv | cut -d, -f1-4
done
