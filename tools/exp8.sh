#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_tune.py --variants 8,21,13,208,213 --iters 50 > gpurun_out/e8_tune.log 2>&1
timeout -k 10 200 python tools/gemm_tune.py --variants 8,21,13,208,213 --iters 50 --epi 6 > gpurun_out/e8_tune_discard.log 2>&1
