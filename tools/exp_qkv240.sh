#!/bin/bash
# 240x256 QKV tiles (variants 98 / 99) against the 256x256 default (80): kernel tests first,
# then the in-model A/B of tools/exp_env.sh (compare the qkv_gemm family per forward).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "98 or 99 or staged or identity" > gpurun_out/qkv240_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/qkv240_tests.log; exit 1; }
tail -2 gpurun_out/qkv240_tests.log
bash tools/exp_env.sh "CLIPVIT_X=0" "CLIPVIT_GEMM_VARIANTS=98,82,13,82,22" "CLIPVIT_GEMM_VARIANTS=99,82,13,82,22" "CLIPVIT_GEMM_VARIANTS=80,82,13,82,22"
