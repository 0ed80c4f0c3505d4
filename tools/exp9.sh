#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" > gpurun_out/e9_tests.log 2>&1
timeout -k 10 200 python tools/gemm_tune.py --variants 8,208,13,213,30,230,31,231 --iters 50 > gpurun_out/e9_tune.log 2>&1
for cfg in "8,21,13,21,21 2,2,2,2,1" "30,21,30,21,21 1,2,1,2,1" "30,21,30,21,21 2,2,2,2,1" "31,21,31,21,21 2,2,2,2,1"; do
  set -- $cfg
  echo "var=$1 xcd=$2" >> gpurun_out/e9_bench.log
  CLIPVIT_GEMM_VARIANTS=$1 CLIPVIT_GEMM_XCD=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 >> gpurun_out/e9_bench.log 2>&1
done
