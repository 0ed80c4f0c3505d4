#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_tune.py --variants 8,9,30,32,33 --iters 50 > gpurun_out/e10_tune.log 2>&1
timeout -k 10 200 python tools/gemm_tune.py --variants 8,9 --iters 50 --epi 6 > gpurun_out/e10_tune_discard.log 2>&1
