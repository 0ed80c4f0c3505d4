#!/bin/bash
# Class-token tail GEMM tile: 64x64 (v90) against 32x64 one-wave tiles (v96 / v97).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "96 or 97 or identity" > gpurun_out/tail_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/tail_tests.log | head; tail -5 gpurun_out/tail_tests.log; exit 1; }
tail -1 gpurun_out/tail_tests.log
CLIPVIT_TAIL_VARIANT=96 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prune" > gpurun_out/tail_tests2.log 2>&1 || { echo "prune tests failed"; grep -E "FAIL|assert|Error" gpurun_out/tail_tests2.log | head; tail -5 gpurun_out/tail_tests2.log; exit 1; }
tail -1 gpurun_out/tail_tests2.log
bash tools/exp_env.sh "CLIPVIT_TAIL_VARIANT=90" "CLIPVIT_TAIL_VARIANT=96" "CLIPVIT_TAIL_VARIANT=97"
