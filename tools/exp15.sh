#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mx8.py -x -q -s > gpurun_out/e15_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype mxfp8 --batch 512 --steps 20 > gpurun_out/e15_b512.log 2>&1
CLIPVIT_MX8_SKIP= timeout -k 10 200 python bench.py --no-cpu-baseline --dtype mxfp8 --batch 512 --steps 20 > gpurun_out/e15_b512_all.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype bf16 --batch 512 --steps 20 > gpurun_out/e15_b512_bf16.log 2>&1
