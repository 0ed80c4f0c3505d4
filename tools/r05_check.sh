#!/bin/bash
# Round 5: GEMM kernel tests of variant 72 / blocked W after the header clean-up, then the
# reference-harness fixtures. Output under gpurun_out/r05_check/.
set -o pipefail
out=gpurun_out/r05_check
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm and (72 or 100)" > $out/kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 $out/kernels.log; exit 1; }
tail -1 $out/kernels.log
bash tools/r05_golden.sh
