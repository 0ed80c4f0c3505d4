#!/bin/bash
# 256x192 12-wave tiles (variant 89) for out_proj / c_proj / patch against the defaults
# (82 / 82 / 22); both arms forced through CLIPVIT_GEMM_VARIANTS (no c_fc split in either).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "89 or identity" > gpurun_out/v89_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/v89_tests.log; exit 1; }
tail -2 gpurun_out/v89_tests.log
bash tools/exp_env.sh "CLIPVIT_GEMM_VARIANTS=98,82,13,82,22" "CLIPVIT_GEMM_VARIANTS=98,89,13,89,22" "CLIPVIT_GEMM_VARIANTS=98,82,13,82,89"
