#!/bin/bash
set -e
mkdir -p gpurun_out
true
timeout -k 10 400 python -m pytest tests/test_gpu_mx8.py -x -q -s > gpurun_out/e12_tests.log 2>&1 || true
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype mxfp8 --steps 20 > gpurun_out/e12_bench8.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype mxfp8 --batch 512 --steps 20 > gpurun_out/e12_bench8_512.log 2>&1
