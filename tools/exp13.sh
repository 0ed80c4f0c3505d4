#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mx8.py -x -q -s -k "config5" > gpurun_out/e13_tests.log 2>&1 || true
timeout -k 10 200 python tools/gemm_tune.py --dtype 3 --variants 1,2,201,202 --iters 50 > gpurun_out/e13_tune.log 2>&1
