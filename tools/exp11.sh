#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" > gpurun_out/e11_tests.log 2>&1
timeout -k 10 200 python tools/gemm_tune.py --variants 8,28,21,29,30,34,32,33 --iters 50 > gpurun_out/e11_tune.log 2>&1
for cfg in "8,21,13,21,21 2,2,2,2,1" "30,21,30,21,21 2,2,2,2,1" "34,29,34,29,29 2,2,2,2,1" "28,29,28,29,29 2,2,2,2,1"; do
  set -- $cfg
  echo "var=$1 xcd=$2" >> gpurun_out/e11_bench.log
  CLIPVIT_GEMM_VARIANTS=$1 CLIPVIT_GEMM_XCD=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 >> gpurun_out/e11_bench.log 2>&1
done
