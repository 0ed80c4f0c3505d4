#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/blas_ref.py > gpurun_out/e7_blas.log 2>&1
for x in "2,2,2,2,1"; do
  for v in "8,21,13,21,21" "8,21,21,21,21"; do
    echo "xcd=$x var=$v" >> gpurun_out/e7_bench.log
    CLIPVIT_GEMM_XCD=$x CLIPVIT_GEMM_VARIANTS=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 >> gpurun_out/e7_bench.log 2>&1
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 10 --warmup 3 > gpurun_out/e7_l14.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --model ViT-B/16 --steps 10 --warmup 3 > gpurun_out/e7_b16.log 2>&1
