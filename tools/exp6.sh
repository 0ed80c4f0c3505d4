#!/bin/bash
# XCD 2-D tile partition: kernel parity, isolated GEMM timings, whole-forward bench.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k gemm > gpurun_out/e6_tests.log 2>&1
timeout -k 10 200 python tools/gemm_tune.py --variants 8,208,21,221,13,213,22,222 --iters 50 > gpurun_out/e6_tune.log 2>&1
for x in "1,1,1,1,1" "2,1,2,1,1" "2,2,2,2,1" "1,1,2,1,1"; do
  for v in "8,21,21,21,21"; do
    echo "xcd=$x var=$v" >> gpurun_out/e6_bench.log
    CLIPVIT_GEMM_XCD=$x CLIPVIT_GEMM_VARIANTS=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 >> gpurun_out/e6_bench.log 2>&1
  done
done
